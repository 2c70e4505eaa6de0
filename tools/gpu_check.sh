#!/bin/bash
# One GPU-box session: parity tests, then a short bench.  Stops at the first
# step that faults/aborts/times out (exit codes other than 0 or 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-10}
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -n 30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"; tail -n 20 gpurun_out/bench.log
exit $rc2
