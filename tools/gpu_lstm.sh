#!/bin/bash
# LSTM session: -m gpu LSTM parity tests, then the L bench line (C = 1 and 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_boundary.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/lstm_tests.log 2>&1
rc=$?; echo "lstm tests rc=$rc $(tail -1 gpurun_out/lstm_tests.log)"
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/lstm_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_lstm.json 2> gpurun_out/bench_lstm.err
rc=$?; echo "lstm bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_lstm.err; exit $rc; }
timeout -k 10 300 python bench.py --config lstm --bptt-chunks 2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_lstm_c2.json 2> gpurun_out/bench_lstm_c2.err
rc=$?; echo "lstm c2 bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_lstm_c2.err; exit $rc; }
python -c "import json; [print(f, round(json.load(open('gpurun_out/'+f))['ms_per_step'],3), 'ms') for f in ('bench_lstm.json','bench_lstm_c2.json')]"
exit 0
