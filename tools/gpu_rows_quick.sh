#!/bin/bash
# Row-split kernel: quick parity (rows tests), phase stamps, headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-rowsq}
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
run pytest_rows 300 python -u -m pytest tests/test_gpu_rows.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
MADRONA_LEARN_LIB=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn_stamps.so run stamps 300 python tools/stamp_rows.py
cat "$out/stamps.out"
run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
python -c "import json; d=json.load(open('$out/bench.out')); print('ms', round(d['ms_per_step'],3), 'step_us', round(d['roofline']['avg_launch_us'],1))"
exit 0
