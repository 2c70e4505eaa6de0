#!/bin/bash
# Round-4: four-wave LSTM forward step (ML_LSTM_FWD4 variant): parity on the
# variant library, config-L A/B, kernel stats of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04o
mkdir -p $OUT
export TMPDIR=/tmp
V=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn_fwd4.so
[ -n "${SKIP_TESTS:-}" ] || MADRONA_LEARN_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lstm.py tests/test_gpu_configs.py -k "lstm" > $OUT/t_fwd4.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/t_fwd4.log; exit 3; }
tail -2 $OUT/t_fwd4.log
VARIANTS="base fwd4 base fwd4" STEPS=10 BENCH_ARGS="--config lstm --no-separate-sim-line" timeout -k 10 600 bash tools/variants_bench.sh || exit 4
for v in base fwd4; do
  if [ $v = base ]; then unset MADRONA_LEARN_LIB; else export MADRONA_LEARN_LIB=$V; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python bench.py --config lstm --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-separate-sim-line > $OUT/prof_$v.log 2>&1 || exit 5
done
exit 0
