#!/bin/bash
# A/B of the A_0 recompute (MLEARN_A0_RECOMPUTE) over library variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  if [ "$v" = base ]; then lib=madrona-learn_amd/madrona_learn/_lib/libmlearn.so
  else lib=madrona-learn_amd/madrona_learn/_lib/libmlearn_$v.so; fi
  for a in ${A0R:-0 1}; do
    MADRONA_LEARN_LIB=$PWD/$lib MLEARN_A0_RECOMPUTE=$a timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/ab_${v}_$a.json 2> gpurun_out/ab_${v}_$a.err
    rc=$?; if [ $rc -ne 0 ]; then echo "$v a0r=$a rc=$rc"; tail -5 gpurun_out/ab_${v}_$a.err; exit $rc; fi
    python -c "import json; d=json.load(open('gpurun_out/ab_${v}_$a.json')); print('$v a0r=$a', round(d['ms_per_step'],4), 'ms')"
  done
done
