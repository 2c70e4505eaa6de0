#!/bin/bash
# Round-3: fused env step (policy launch), past-policy snapshots; A/B bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03d}
mkdir -p "$out"
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 40 "$out/$name.out"; tail -n 5 "$out/$name.err"; exit $rc; fi
}
run fused 900 python -u -m pytest tests/test_gpu_fused_env.py tests/test_gpu_pbt.py tests/test_gpu_train.py tests/test_gpu_lstm.py tests/test_gpu_configs.py -x -v -p no:cacheprovider --timeout 600 --timeout-method thread
tail -n 2 "$out/fused.out"
run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
python -c "import json; d=json.load(open('$out/bench.out')); print('fused ms', round(d['ms_per_step'],3), 'step_us', round(d['roofline']['avg_launch_us'],1))"
run bench_sep 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --separate-sim
python -c "import json; d=json.load(open('$out/bench_sep.out')); print('separate ms', round(d['ms_per_step'],3))"
run bench_lstm 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
python -c "import json; d=json.load(open('$out/bench_lstm.out')); print('lstm ms', round(d['ms_per_step'],3))"
run prof_lstm 420 rocprofv3 --kernel-trace --stats -d "$out/prof_lstm" -o run --output-format csv -- python bench.py --config lstm --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
run prof 420 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
exit 0
