#!/bin/bash
# Round-4: gradient reduction fused into the weight-gradient launch.
# Targeted parity first, then the headline and W=8-share bench lines with a
# kernel-stats profile, then the whole -m gpu suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04d
mkdir -p $OUT
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
run t_grad 400 $PYT tests/test_gpu_policy.py tests/test_gpu_fullsize.py tests/test_gpu_train.py tests/test_gpu_generic.py
run bench 240 python bench.py --steps 20 --warmup 3 --no-separate-sim-line
run emu8 240 python bench.py --steps 10 --warmup 3 --emulate-world 8
run prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-separate-sim-line
run t_all 1000 $PYT tests -m gpu
exit 0
