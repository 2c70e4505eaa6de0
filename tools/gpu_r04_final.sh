#!/bin/bash
# Round-4 final measurements (one GPU session): the -m gpu suite, every bench
# line, kernel stats of the headline and config L, the headline's PMC passes,
# the W = 8 share projection.  Outputs under gpurun_out/r04f/ (copied into
# profiles/ by hand afterwards).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04final
mkdir -p $OUT
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 2 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then exit $rc; fi
}
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
run suite 1100 $PYT tests -m gpu
run bench_headline 400 python bench.py --steps 20 --warmup 3
run bench_b1 200 python bench.py --config b1 --steps 10 --warmup 3 --no-cpu-baseline --no-separate-sim-line
run bench_twohot 200 python bench.py --critic twohot --steps 10 --warmup 3 --no-cpu-baseline --no-separate-sim-line
run bench_lstm 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-separate-sim-line
run bench_lstm_c2 300 python bench.py --config lstm --bptt-chunks 2 --steps 10 --warmup 3 --no-cpu-baseline --no-separate-sim-line
run bench_pbt 300 python bench.py --config pbt --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-separate-sim-line
run emu8 300 python bench.py --steps 10 --warmup 3 --emulate-world 8
run prof_headline 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_headline -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-separate-sim-line
run prof_lstm 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_lstm -o run --output-format csv -- python bench.py --config lstm --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-separate-sim-line
PASSES="FETCH_SIZE
WRITE_SIZE
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_BANK_CONFLICT
TCC_HIT_sum TCC_MISS_sum" KRE="ppo_step|wgrad|policy_rollout|gae|reduce_grads|adam|project" PASS_TIMEOUT=180 run pmc 900 bash tools/gpu_pmc.sh
exit 0
