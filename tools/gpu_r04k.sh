#!/bin/bash
# Round-4: persistent forward LSTM scan (bit identity vs per-step launches,
# then the LSTM suite and config L A/B), then the torch-path tests and the
# whole -m gpu suite, then the spill-layout profiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04k
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
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
run t_scan 240 $PYT tests/test_gpu_lstm.py -k "launch_forms"
run t_lstm 400 $PYT tests/test_gpu_lstm.py tests/test_gpu_configs.py
run bench_lstm 200 python bench.py --config lstm --lstm-scan 2 --steps 5 --warmup 2 --no-cpu-baseline --no-separate-sim-line
run bench_lstm_ps 200 python bench.py --config lstm --steps 5 --warmup 2 --no-cpu-baseline --no-separate-sim-line --lstm-scan 1
run t_all 1000 $PYT tests -m gpu
exit 0
