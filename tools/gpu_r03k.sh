#!/bin/bash
# Round-3 A/B: whole-rollout kernel without its loop spill (parameters staged
# once) forced to one launch at the headline's 2 048 tiles, vs per-step;
# the W=8 share with the rollout as one launch vs per-step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03k}
mkdir -p "$out"
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 40 "$out/$name.out"; tail -n 5 "$out/$name.err"; exit $rc; fi
}
run tests 900 python -u -m pytest tests/test_gpu_fused_env.py tests/test_gpu_lstm.py tests/test_gpu_train.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 "$out/tests.out"
MLEARN_ROLLOUT_ONE_LAUNCH=1 run b_one 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run b_step 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
MLEARN_ROLLOUT_ONE_LAUNCH=1 run b_one2 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run b_step2 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run e8_one 300 python bench.py --emulate-world 8 --steps 10 --warmup 3
MLEARN_ROLLOUT_PER_STEP=1 run e8_step 300 python bench.py --emulate-world 8 --steps 10 --warmup 3
run l_one 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
for f in b_one b_step b_one2 b_step2 l_one; do
  tail -1 $out/$f.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3))"
done
for f in e8_one e8_step; do
  tail -1 $out/$f.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_update_rank_share'],3), round(d['n1_ms_per_update'],3))"
done
MLEARN_ROLLOUT_ONE_LAUNCH=1 run prof 420 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
exit 0
