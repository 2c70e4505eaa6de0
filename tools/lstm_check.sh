#!/bin/bash
# LSTM parity (tests/test_gpu_lstm.py, the config-L test) then the config-L
# bench line and its rocprofv3 kernel stats.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lstm
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_configs.py -k "lstm" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/lstm/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/lstm/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/lstm/bench.json 2> gpurun_out/lstm/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/lstm/bench.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/lstm/bench.json')); print(d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lstm/prof -o run --output-format csv -- python bench.py --config lstm --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/lstm/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/lstm/prof/**/*kernel_stats.csv',recursive=True)[0]
r=list(csv.DictReader(open(f)))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:8]: print(x['Name'][:50], x['Calls'], round(float(x['AverageNs'])/1e3,2))
PY
