#!/bin/bash
# Round-4: 8-wave feature split of the rollout policy (ML_POL_MAXW=8 variant) vs 4 waves:
# B1 (256 tiles, one workgroup per CU), headline, W = 8 share.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VARIANTS="base pw8 base pw8" STEPS=10 BENCH_ARGS="--config b1 --no-separate-sim-line" timeout -k 10 400 bash tools/variants_bench.sh || exit 4
VARIANTS="base pw8" STEPS=10 BENCH_ARGS="--no-separate-sim-line" timeout -k 10 400 bash tools/variants_bench.sh || exit 5
for v in base pw8; do
  if [ $v = base ]; then unset MADRONA_LEARN_LIB; else export MADRONA_LEARN_LIB=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn_$v.so; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --emulate-world 8 > gpurun_out/emu_$v.json 2> gpurun_out/emu_$v.err || exit 6
  python -c "import json; d=json.load(open('gpurun_out/emu_$v.json')); print('emu8 $v', round(d['ms_per_update_rank_share'],4), round(d['n1_ms_per_update'],4))"
done
exit 0
