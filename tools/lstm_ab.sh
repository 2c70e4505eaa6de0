#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/lstm_ab
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then dir=madrona_learn/_lib; lib=libmlearn.so; else dir=variants; lib=libmlearn_$v.so; fi
  export MADRONA_LEARN_LIB=$PWD/madrona-learn_amd/$dir/$lib
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lstm_ab/$v -o run --output-format csv -- python bench.py --config lstm --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/lstm_ab/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/lstm_ab/$v.log; exit $rc; fi
  python3 - $v <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/lstm_ab/{sys.argv[1]}/**/*kernel_stats.csv',recursive=True)[0]
for x in csv.DictReader(open(f)):
    if 'lstm' in x['Name']: print(sys.argv[1], x['Name'][:40], x['Calls'], round(float(x['AverageNs'])/1e3,2))
PY
done
