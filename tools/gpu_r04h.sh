#!/bin/bash
# Round-4: fragment-native A/dZ spill.  Parity of every bf16 update path,
# then the headline bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04h
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
run t_grad 500 $PYT tests/test_gpu_policy.py tests/test_gpu_fullsize.py tests/test_gpu_train.py tests/test_gpu_configs.py tests/test_gpu_dp.py tests/test_gpu_emulated_dp.py
run bench 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-separate-sim-line
run emu8 240 python bench.py --steps 10 --warmup 3 --emulate-world 8
exit 0
