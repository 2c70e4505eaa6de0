#!/bin/bash
# Round-2 GPU session: headline bench line + rocprofv3 stats, the -m gpu
# parity suite, the B1 line.  Every step has its own time limit; the script
# stops at the first step that faults / aborts / times out (exit status
# other than 0 or 1).  STEPS_LIST selects steps (default: all).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 to=$2
    shift 2
    case " ${STEPS_LIST:-bench prof pytest b1} " in *" ${name%%_*} "*) ;; *) return 0 ;; esac
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/steps.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
rm -f gpurun_out/steps.txt
step bench_headline 420 python bench.py --steps 20 --warmup 3
step prof_headline 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_headline -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS:-}
step b1_bench 300 python bench.py --config b1 --steps 20 --warmup 3 --no-cpu-baseline
exit 0
