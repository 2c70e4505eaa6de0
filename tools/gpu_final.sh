#!/bin/bash
# Round-end GPU session: every bench line and rocprofv3 summary that
# profiles/ keeps.  Each step has its own time limit; the script stops at the
# first step that faults / aborts / times out.  (The -m gpu suite runs in
# tools/gpu_suite.sh.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-final}
mkdir -p $O
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 5 "$O/$name.err"; exit $rc; fi
}
run bench_headline 420 python bench.py --steps 20 --warmup 3
run bench_headline_nofusedgae 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --no-fused-gae
run bench_headline2 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run prof_headline 420 rocprofv3 --kernel-trace --stats -d $O/prof_headline -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run bench_b1 300 python bench.py --config b1 --steps 20 --warmup 3 --no-cpu-baseline
run bench_twohot 300 python bench.py --critic twohot --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
run bench_lstm 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline
run bench_lstm_c2 300 python bench.py --config lstm --bptt-chunks 2 --steps 10 --warmup 3 --no-cpu-baseline
run prof_lstm 420 rocprofv3 --kernel-trace --stats -d $O/prof_lstm -o run --output-format csv -- python bench.py --config lstm --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
run bench_pbt 300 python bench.py --config pbt --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
run emu8 300 python bench.py --emulate-world 8 --steps 20 --warmup 3
run emu4 300 python bench.py --emulate-world 4 --steps 20 --warmup 3
run emu2 300 python bench.py --emulate-world 2 --steps 20 --warmup 3
exit 0
