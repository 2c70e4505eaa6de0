#!/bin/bash
# Round-3 full session: the -m gpu suite, every bench line profiles/ keeps,
# the W=8 emulation and the rocprofv3 summaries.  Each step has its own time
# limit; the script stops at the first step that faults / aborts / times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03f}
mkdir -p "$out"
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 30 "$out/$name.out"; tail -n 5 "$out/$name.err"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 "$out/pytest_gpu.out"
run bench_headline 420 python bench.py --steps 20 --warmup 3
run bench_separate 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --separate-sim
run emulate8 420 python bench.py --emulate-world 8 --steps 10 --warmup 3
run prof_emulate8 420 rocprofv3 --kernel-trace --stats -d "$out/prof_emulate8" -o run --output-format csv -- python bench.py --emulate-world 8 --steps 5 --warmup 2
run bench_b1 300 python bench.py --config b1 --steps 20 --warmup 3 --no-cpu-baseline
run bench_twohot 300 python bench.py --critic twohot --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
run bench_lstm 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline
run bench_lstm_c2 300 python bench.py --config lstm --bptt-chunks 2 --steps 10 --warmup 3 --no-cpu-baseline
run bench_pbt 300 python bench.py --config pbt --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
run prof_headline 420 rocprofv3 --kernel-trace --stats -d "$out/prof_headline" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run prof_lstm 420 rocprofv3 --kernel-trace --stats -d "$out/prof_lstm" -o run --output-format csv -- python bench.py --config lstm --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
for f in bench_headline bench_separate emulate8 bench_b1 bench_twohot bench_lstm bench_lstm_c2 bench_pbt; do
  tail -1 "$out/$f.out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d.get('ms_per_step', d.get('ms_per_update_rank_share', 0)),3), d.get('value', d.get('implied_scaling_1_to_W')))"
done
if [ "${PMC:-0}" = 1 ]; then
  rm -rf gpurun_out/pmc
  KRE='ppo_step|wgrad|policy_rollout|gae|reduce_grads|adam|project' bash tools/gpu_pmc.sh > "$out/pmc.log" 2>&1 || { echo pmc failed; tail "$out/pmc.log"; exit 1; }
  cat "$out/pmc.log"
  python tools/pmc_traffic.py gpurun_out/pmc "$out/pmc_headline.json" && mv gpurun_out/pmc "$out/pmc_headline"
  KRE='lstm|wgrad|project|policy_rollout|ppo_step' BENCH_ARGS='--config lstm' bash tools/gpu_pmc.sh > "$out/pmc_lstm.log" 2>&1 || { echo pmc lstm failed; tail "$out/pmc_lstm.log"; exit 1; }
  cat "$out/pmc_lstm.log"
  python tools/pmc_traffic.py gpurun_out/pmc "$out/pmc_lstm.json" && mv gpurun_out/pmc "$out/pmc_lstm"
fi
exit 0
