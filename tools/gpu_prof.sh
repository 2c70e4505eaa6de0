#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC counters here).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-prof}
timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG -o run --output-format csv -- python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/$TAG.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -n 5 gpurun_out/$TAG.log
find gpurun_out/$TAG -name "*stats*.csv" | head
exit $rc
