#!/bin/bash
# Round-3: parity configurations + env kernel + policy stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03c}
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
run kat 300 python -u -m pytest tests/test_gpu_rollout_kat.py tests/test_gpu_kernels.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run pstamps 300 env MADRONA_LEARN_LIB=madrona-learn_amd/madrona_learn/_lib/libmlearn_stamps.so python tools/stamp_policy.py
cat "$out/pstamps.out"
run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
python -c "import json; d=json.load(open('$out/bench.out')); print('ms', round(d['ms_per_step'],3), 'step_us', round(d['roofline']['avg_launch_us'],1))"
run bf16 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_pbt.py tests/test_gpu_lstm.py tests/test_gpu_dp.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "bf16 or dp"
run configs 900 python -u -m pytest tests/test_gpu_configs.py -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread --durations=0
exit 0
