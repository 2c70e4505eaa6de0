#!/bin/bash
# A/B of library variants on the emulated W-rank shares (bench.py
# --emulate-world W) for W in $WS; VARIANTS as tools/variants_bench.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/emu
for v in ${VARIANTS}; do
  if [ "$v" = base ]; then lib=madrona-learn_amd/madrona_learn/_lib/libmlearn.so
  else lib=madrona-learn_amd/madrona_learn/_lib/libmlearn_$v.so; fi
  export MADRONA_LEARN_LIB=$PWD/$lib
  for W in ${WS:-8 4 2}; do
    timeout -k 10 300 python bench.py --emulate-world $W --steps ${STEPS:-10} --warmup 3 > gpurun_out/emu/ab_${v}_$W.json 2> gpurun_out/emu/ab_${v}_$W.err
    rc=$?; if [ $rc -ne 0 ]; then echo "$v W=$W rc=$rc"; tail -5 gpurun_out/emu/ab_${v}_$W.err; exit $rc; fi
    python -c "import json; d=json.loads(open('gpurun_out/emu/ab_${v}_$W.json').read().strip().splitlines()[-1]); print('$v', 'W=$W', round(d['ms_per_update_rank_share'],3), 'ms share; N=1', round(d['n1_ms_per_update'],3))"
  done
done
