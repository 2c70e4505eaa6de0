#!/bin/bash
# Round-4: a population's whole rollouts as one launch (mlearn_policy_rollout_env_pop):
# parity (fused-env bit identity incl. population cases, PBT / configs / ckpt tests),
# then config P A/B (population launch vs one launch per policy), headline check.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04p
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused_env.py tests/test_gpu_pbt.py tests/test_gpu_configs.py tests/test_gpu_ckpt.py tests/test_abi.py > $OUT/t.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/t.log; exit 3; }
tail -1 $OUT/t.log
for v in pop per pop per; do
  if [ $v = per ]; then A=--per-policy-rollouts; else A=; fi
  timeout -k 10 200 python bench.py --config pbt --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-separate-sim-line $A > $OUT/pbt_$v.json 2> $OUT/pbt_$v.err || { echo "bench rc=$?"; tail -5 $OUT/pbt_$v.err; exit 4; }
  python -c "import json; d=json.load(open('$OUT/pbt_$v.json')); print('$v', round(d['ms_per_step'],4), 'ms', round(d['ms_per_update_median'],4))"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/headline.json 2> $OUT/headline.err || { echo "headline rc=$?"; exit 5; }
python -c "import json; d=json.load(open('$OUT/headline.json')); print('headline', round(d['ms_per_step'],4), d['kernels']['policy_rollout']['avg_launch_us'], d['roofline']['avg_launch_us'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_pbt -o run --output-format csv -- python bench.py --config pbt --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-separate-sim-line > $OUT/prof_pbt.log 2>&1 || exit 6
exit 0
