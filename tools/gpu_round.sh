#!/bin/bash
# One GPU session: B1 bench line + rocprofv3 kernel stats, the -m gpu parity
# suite, then the L (LSTM) bench line + kernel stats.  Stops at the first
# step that faults / aborts / times out (exit status other than 0 or 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/steps.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
rm -f gpurun_out/steps.txt
step bench_b1 420 python bench.py --steps 20 --warmup 3
step prof_b1 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
step bench_lstm 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline
step prof_lstm 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lstm -o run --output-format csv -- python bench.py --config lstm --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
exit 0
