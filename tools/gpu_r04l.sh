#!/bin/bash
# Round-4: tiled spill layout with per-split padding (variant libraries) vs
# the row layout, headline bench; then parity of the padded variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04l
mkdir -p $OUT
export TMPDIR=/tmp
for v in base tiled tiledpad tiledpad2; do
  if [ $v = base ]; then unset MADRONA_LEARN_LIB; else export MADRONA_LEARN_LIB=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn_$v.so; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-separate-sim-line > $OUT/$v.log 2>&1 || exit 3
done
export MADRONA_LEARN_LIB=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn_tiledpad.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_policy.py tests/test_gpu_fullsize.py tests/test_gpu_train.py > $OUT/t_pad.log 2>&1
echo "t_pad rc=$?"; tail -2 $OUT/t_pad.log
exit 0
