#!/bin/bash
# Tests, then rocprofv3 kernel stats of a short bench, then the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SKIP_BENCH=1 bash tools/gpu_check.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_prof.sh
rc2=$?
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 600 python bench.py --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc3=$?
echo "bench rc=$rc3"; tail -n 3 gpurun_out/bench.log
exit $rc3
