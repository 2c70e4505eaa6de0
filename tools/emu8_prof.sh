#!/bin/bash
# Emulated W-rank share (bench.py --emulate-world W) and its rocprofv3 kernel
# stats.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/emu
export TMPDIR=/tmp
W=${W:-8}
timeout -k 10 300 python bench.py --emulate-world $W --steps 10 --warmup 3 > gpurun_out/emu/emu$W.json 2> gpurun_out/emu/emu$W.err
rc=$?; echo "emulate rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/emu/emu$W.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/emu/emu$W.json')); print({k: d[k] for k in ('ms_per_update_rank_share','n1_ms_per_update','implied_scaling_1_to_W')})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/emu/prof$W -o run --output-format csv -- python bench.py --emulate-world $W --steps 5 --warmup 2 > gpurun_out/emu/prof$W.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv,glob,os
W=os.environ.get('W','8')
f=glob.glob(f'gpurun_out/emu/prof{W}/**/*kernel_stats.csv',recursive=True)[0]
r=list(csv.DictReader(open(f)))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:16]: print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,2))
PY
