#!/bin/bash
# A/B of library variants (variants/libmlearn_<name>.so): GPU parity
# tests of the policy / train paths, then the default bench, per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  if [ "$v" = base ]; then lib=madrona-learn_amd/madrona_learn/_lib/libmlearn.so
  else lib=madrona-learn_amd/variants/libmlearn_$v.so; fi
  export MADRONA_LEARN_LIB=$PWD/$lib
  timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_train.py tests/test_gpu_lstm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/var_$v.test.log 2>&1
  rc=$?; echo "$v tests rc=$rc $(tail -1 gpurun_out/var_$v.test.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$v bench rc=$rc"; tail -5 gpurun_out/var_$v.err; exit $rc; fi
  python -c "import json,sys; d=json.load(open('gpurun_out/var_$v.json')); k=d.get('kernels',{}); print('$v', round(d['ms_per_step'],4), 'ms', d.get('roofline',{}).get('avg_launch_us'), k.get('policy_step',{}).get('avg_launch_us'))"
done
