#!/bin/bash
# Round-4: tiled spill layout with per-split padding (variant libraries) vs
# the row layout, headline bench; then parity of the padded variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04m
mkdir -p $OUT
export TMPDIR=/tmp
for v in base tiled base2 tiled2; do
  if [ ${v%2} = base ]; then unset MADRONA_LEARN_LIB; else export MADRONA_LEARN_LIB=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn_${v%2}.so; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-separate-sim-line > $OUT/$v.log 2>&1 || exit 3
done
export MADRONA_LEARN_LIB=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn_tiled.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_policy.py tests/test_gpu_fullsize.py tests/test_gpu_train.py > $OUT/t_pad.log 2>&1
echo "t_pad rc=$?"; tail -2 $OUT/t_pad.log
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-include-regex "wgrad|ppo_step" -d $OUT/pmc_tiled -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-roofline --no-separate-sim-line > $OUT/pmc_tiled.log 2>&1
exit 0
