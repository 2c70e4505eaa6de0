#!/bin/bash
# Round-3 A/B: (1) LSTM per-step scans with the cell's operands (done flag,
# biases; backward: gates / c / dh rows) loaded before the product instead of
# after it, 1-wave (default, D) vs 4-wave (A) forward; (2) rollout policy
# kernel at 4 workgroups per CU (R: W1 ring 4, 128 VGPRs, 76 B scratch) vs 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03m}
mkdir -p "$out"
export TMPDIR=/tmp
V=$PWD/madrona-learn_amd/madrona_learn/_lib/var
MAIN=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn.so
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 40 "$out/$name.out"; tail -n 5 "$out/$name.err"; exit $rc; fi
}
lib() { if [ $1 = D ]; then echo $MAIN; else echo $V/libmlearn_$1.so; fi; }
for v in D A R; do
  MADRONA_LEARN_LIB=$(lib $v) run t_$v 600 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_fused_env.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
  tail -n 1 "$out/t_$v.out"
done
for v in D A D A; do
  MADRONA_LEARN_LIB=$(lib $v) run l_$v 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  tail -1 $out/l_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('l_$v', round(d['ms_per_step'],3))"
done
for v in D R D R; do
  MADRONA_LEARN_LIB=$(lib $v) run b_$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
  tail -1 $out/b_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b_$v', round(d['ms_per_step'],3))"
done
for v in D A; do
  MADRONA_LEARN_LIB=$(lib $v) run p_$v 300 rocprofv3 --kernel-trace --stats -d "$out/p_$v" -o run --output-format csv -- python bench.py --config lstm --steps 3 --warmup 1 --no-cpu-baseline --no-roofline
  grep -E "lstm_(fwd|bwd)_step" $(find $out/p_$v -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4
done
MADRONA_LEARN_LIB=$(lib R) run p_R 300 rocprofv3 --kernel-trace --stats -d "$out/p_R" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline
grep -E "policy_rollout" $(find $out/p_R -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4
exit 0
