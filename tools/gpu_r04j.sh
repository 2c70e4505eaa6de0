#!/bin/bash
# Round-4: row-major vs tiled A/dZ spill (ML_TILED_SPILL variant library):
# kernel stats and HBM / L2 counters of the step and weight-gradient kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04j
mkdir -p $OUT
export TMPDIR=/tmp
for v in rows tiled; do
  if [ $v = rows ]; then unset MADRONA_LEARN_LIB; else export MADRONA_LEARN_LIB=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn_tiled.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-separate-sim-line > $OUT/prof_$v.log 2>&1 || exit 3
  for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
    n=$(echo $pass | tr ' ' '_')
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pass --kernel-include-regex "ppo_step|wgrad" -d $OUT/pmc_$v/$n -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-roofline --no-separate-sim-line > $OUT/pmc_${v}_$n.log 2>&1 || exit 4
  done
done
exit 0
