#!/bin/bash
# Round-3 checkpoint: full GPU suite, headline bench, W=8 emulation, profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03a}
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
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 2 "$out/pytest_gpu.out"
run bench 420 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
python -c "import json; d=json.load(open('$out/bench.out')); print('ms', round(d['ms_per_step'],3), 'step_us', round(d['roofline']['avg_launch_us'],1), d['collectives'])"
run emulate8 420 python bench.py --emulate-world 8 --steps 10 --warmup 3
cat "$out/emulate8.out"
run prof 420 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
run prof8 420 rocprofv3 --kernel-trace --stats -d "$out/prof8" -o run --output-format csv -- python bench.py --emulate-world 8 --steps 5 --warmup 2
exit 0
