#!/bin/bash
# Row-split step kernel: parity tests, then the headline bench and a kernel
# profile.  Each GPU step has its own time limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-rows}
mkdir -p "$out"
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 30 "$out/$name.out"; tail -n 5 "$out/$name.err"; exit $rc; fi
}
run pytest_rows 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_fullsize.py tests/test_gpu_train.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
tail -n 1 "$out/bench.out" | cut -c1-400
run prof 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
