#!/bin/bash
# Round-4: the wide-tile step kernel.  Targeted parity tests first (every
# tile width forced through mlearn_ppo_hparams.row_blocks, the 65,536-row
# minibatch, the production-size configs), then the headline bench line,
# then the rest of the -m gpu suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/r04b/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 12 "gpurun_out/r04b/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
run debug 200 python -u tools/debug_wide.py
run t_wide 600 $PYT tests/test_gpu_policy.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py
run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
run t_all 900 $PYT tests -m gpu --deselect tests/test_gpu_policy.py --deselect tests/test_gpu_fullsize.py --deselect tests/test_gpu_configs.py
exit 0
