#!/bin/bash
# Round 6: parity of the new pieces, then bench A/B of library variants and a
# kernel-stats profile of the product library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r06c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -s -m pytest -x -v --timeout 900 --timeout-method thread -p no:cacheprovider \
  ${TESTS:-tests/test_gpu_optim_fused.py tests/test_gpu_policy.py::test_optimizer_step tests/test_gpu_lstm.py::test_lstm_optimizer_step_and_images tests/test_gpu_obsnorm.py::test_bare_obs_normalizer_state_survives_checkpoint tests/test_gpu_generic.py::test_wide_head_routes_to_torch_path tests/test_gpu_headline_e2e.py} > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|oracle chains" $O/pytest.log | tail -4
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then lib=madrona-learn_amd/madrona_learn/_lib/libmlearn.so
  else lib=madrona-learn_amd/variants/libmlearn_$v.so; fi
  MADRONA_LEARN_LIB=$PWD/$lib timeout -k 10 240 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $O/var_$v.json 2> $O/var_$v.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$v bench rc=$rc"; tail -5 $O/var_$v.err; exit $rc; fi
  python -c "import json; d=json.load(open('$O/var_$v.json')); k=d.get('kernels',{}); r=d.get('roofline',{}); print('$v', round(d['ms_per_step'],4), 'ms', r.get('kernel'), r.get('avg_launch_us'), 'minibatch', k.get('minibatch'))"
done
if [ "${PROF:-1}" = "1" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
fi
exit $rc
