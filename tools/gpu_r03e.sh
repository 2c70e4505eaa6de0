#!/bin/bash
# Round-3: policy kernel with every f32 observation fragment in flight at once
# (A/B against ML_POL_OBS_PRE=0), then PMC passes of the headline (fused env)
# and of config L.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03e}
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
run tests 900 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_fused_env.py tests/test_gpu_boundary.py tests/test_gpu_obsnorm.py tests/test_gpu_train.py tests/test_gpu_lstm.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 2 "$out/tests.out"
for v in main noobspre main noobspre; do
  lib=madrona-learn_amd/madrona_learn/_lib/libmlearn.so
  [ $v != main ] && lib=madrona-learn_amd/madrona_learn/_lib/libmlearn_$v.so
  MADRONA_LEARN_LIB=$lib run bench_$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  python -c "import json; d=json.load(open('$out/bench_$v.out')); print('$v', round(d['ms_per_step'],3), 'policy_us', round(d['kernels']['policy_step']['avg_launch_us'],1))"
done
run prof 420 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
KRE='ppo_step|wgrad|policy_step|gae|reduce_grads|adam|project' bash tools/gpu_pmc.sh > "$out/pmc.log" 2>&1 || { echo pmc failed; tail "$out/pmc.log"; exit 1; }
cat "$out/pmc.log"
python tools/pmc_traffic.py gpurun_out/pmc "$out/pmc_headline.json" && mv gpurun_out/pmc "$out/pmc_headline"
KRE='lstm|wgrad|project|policy_step|ppo_step' BENCH_ARGS='--config lstm' bash tools/gpu_pmc.sh > "$out/pmc_lstm.log" 2>&1 || { echo pmc lstm failed; tail "$out/pmc_lstm.log"; exit 1; }
cat "$out/pmc_lstm.log"
python tools/pmc_traffic.py gpurun_out/pmc "$out/pmc_lstm.json" && mv gpurun_out/pmc "$out/pmc_lstm"
exit 0
