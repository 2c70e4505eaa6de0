#!/bin/bash
# Round-3 parity configurations: production-size L / P updates, world-2 DP
# at H=256 bf16, the HIP-path rollout KAT, and the bf16 bound reports.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03b}
mkdir -p "$out"
export TMPDIR=/tmp MLEARN_TEST_REPORT_DIR=$out/bf16
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 40 "$out/$name.out"; tail -n 5 "$out/$name.err"; exit $rc; fi
}
run kat 300 python -u -m pytest tests/test_gpu_rollout_kat.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run bf16 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_pbt.py tests/test_gpu_lstm.py tests/test_gpu_dp.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "bf16 or dp"
run configs 900 python -u -m pytest tests/test_gpu_configs.py -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread --durations=0
exit 0
