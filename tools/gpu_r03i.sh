#!/bin/bash
# Round-3 A/B: whole-rollout launch vs per-step launches (feed-forward: 4-wave
# split, recurrent: 8-wave split), recurrent whole-rollout at 4 vs 3 waves/SIMD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03i}
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
run tests 900 python -u -m pytest tests/test_gpu_fused_env.py tests/test_gpu_train.py tests/test_gpu_lstm.py tests/test_gpu_policy.py tests/test_gpu_boundary.py tests/test_gpu_ckpt.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 "$out/tests.out"
V=madrona-learn_amd/madrona_learn/_lib/libmlearn_rnn3.so
run b_whole 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
MLEARN_WHOLE_ROLLOUT=0 run b_step 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run b_whole2 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
MLEARN_WHOLE_ROLLOUT=0 run b_step2 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run l_whole 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
MLEARN_WHOLE_ROLLOUT=0 run l_step 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
MADRONA_LEARN_LIB=$V run l_whole3 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
for f in b_whole b_step b_whole2 b_step2 l_whole l_step l_whole3; do
  python -c "import json; d=json.load(open('$out/$f.out')); print('$f', round(d['ms_per_step'],3), d['config'].get('sim_step'))"
done
run prof 420 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
run prof_l 420 rocprofv3 --kernel-trace --stats -d "$out/prof_l" -o run --output-format csv -- python bench.py --config lstm --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
exit 0
