#!/bin/bash
# Round-4: LDS counters of the weight-gradient kernel, row vs tile-native dZ.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04n
mkdir -p $OUT
export TMPDIR=/tmp
for v in base dzt; do
  if [ $v = base ]; then unset MADRONA_LEARN_LIB; else export MADRONA_LEARN_LIB=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn_$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-include-regex "wgrad" -d $OUT/$v -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-roofline --no-separate-sim-line > $OUT/$v.log 2>&1 || exit 4
done
exit 0
