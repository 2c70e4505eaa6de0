#!/bin/bash
# Round-4: 16-env half tiles in the whole-rollout launch when 32-env tiles fill <= half the slots:
# parity, then B1 / emulated W = 8 / headline A/B against the ML_ROLL_HALF_TILES=0 variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04v
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused_env.py tests/test_gpu_train.py tests/test_gpu_configs.py tests/test_gpu_policy.py tests/test_gpu_rollout_kat.py tests/test_gpu_pbt.py tests/test_gpu_ckpt.py tests/test_gpu_dp.py > $OUT/t.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/t.log; exit 3; }
tail -1 $OUT/t.log
VARIANTS="base nohalf base nohalf" STEPS=10 BENCH_ARGS="--config b1 --no-separate-sim-line" timeout -k 10 400 bash tools/variants_bench.sh || exit 4
for v in base nohalf; do
  if [ $v = base ]; then unset MADRONA_LEARN_LIB; else export MADRONA_LEARN_LIB=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn_$v.so; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --emulate-world 8 > $OUT/emu8_$v.log 2>&1 || { echo "emu rc=$?"; exit 6; }
  python -c "
import json
L=[l for l in open('$OUT/emu8_$v.log') if l.startswith('{')]
d=json.loads(L[-1]); print('W=8 $v share', round(d['ms_per_update_rank_share'],4), 'n1', round(d['n1_ms_per_update'],4))"
done
exit 0
