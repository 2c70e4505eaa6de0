#!/bin/bash
# Bench-only A/B of library variants (variants/libmlearn_<name>.so,
# built by tools/build_variant.sh): one headline bench line per variant, no
# parity tests (run those on the variant that is kept).  Stops at the first
# step that faults / aborts / times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  if [ "$v" = base ]; then lib=madrona-learn_amd/madrona_learn/_lib/libmlearn.so
  else lib=madrona-learn_amd/variants/libmlearn_$v.so; fi
  export MADRONA_LEARN_LIB=$PWD/$lib
  timeout -k 10 240 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$v bench rc=$rc"; tail -5 gpurun_out/var_$v.err; exit $rc; fi
  python -c "import json; d=json.load(open('gpurun_out/var_$v.json')); k=d.get('kernels',{}); r=d.get('roofline',{}); print('$v', round(d['ms_per_step'],4), 'ms', r.get('kernel'), r.get('avg_launch_us'), 'rollout_us', k.get('policy_rollout',{}).get('avg_launch_us'), 'minibatch', k.get('minibatch'))"
done
