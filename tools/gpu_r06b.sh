#!/bin/bash
# Round 6: fused optimizer parity + ADVICE tests, headline bench, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r06b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -s -m pytest -x -v --timeout 900 --timeout-method thread -p no:cacheprovider \
  ${TESTS:-tests/test_gpu_optim_fused.py tests/test_gpu_policy.py::test_optimizer_step tests/test_gpu_lstm.py::test_lstm_optimizer_step_and_images tests/test_gpu_obsnorm.py::test_bare_obs_normalizer_state_survives_checkpoint tests/test_gpu_generic.py::test_wide_head_routes_to_torch_path tests/test_gpu_headline_e2e.py} > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS:-} > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 $O/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROF:-1}" = "1" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
fi
exit $rc
