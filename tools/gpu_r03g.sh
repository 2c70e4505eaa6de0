#!/bin/bash
# Round-3 A/B: rollout policy kernel with 8 waves per 32-env workgroup
# (NBW = 1, <= 128 VGPRs, 2 workgroups per CU = whole rounds of 512) vs the
# 4-wave default; parity of the variant on the rollout tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03g}
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
V=madrona-learn_amd/madrona_learn/_lib/libmlearn_polw8.so
MADRONA_LEARN_LIB=$V run tests_w8 900 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_fused_env.py tests/test_gpu_boundary.py tests/test_gpu_obsnorm.py tests/test_gpu_train.py tests/test_gpu_lstm.py tests/test_gpu_pbt.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 "$out/tests_w8.out"
for v in main w8 main w8; do
  lib=madrona-learn_amd/madrona_learn/_lib/libmlearn.so
  [ $v = w8 ] && lib=$V
  MADRONA_LEARN_LIB=$lib run bench_$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  python -c "import json; d=json.load(open('$out/bench_$v.out')); print('$v', round(d['ms_per_step'],3), 'policy_us', round(d['kernels']['policy_step']['avg_launch_us'],1))"
done
for v in main w8; do
  lib=madrona-learn_amd/madrona_learn/_lib/libmlearn.so
  [ $v = w8 ] && lib=$V
  MADRONA_LEARN_LIB=$lib run lstm_$v 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  python -c "import json; d=json.load(open('$out/lstm_$v.out')); print('lstm $v', round(d['ms_per_step'],3))"
done
MADRONA_LEARN_LIB=$V run prof_w8 420 rocprofv3 --kernel-trace --stats -d "$out/prof_w8" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
exit 0
