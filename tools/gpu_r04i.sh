#!/bin/bash
# Round-4: torch-path trees (fp16 + DynamicScale, MLP shapes outside the
# kernels, BackboneSeparate), then the whole -m gpu suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04i
mkdir -p $OUT
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
run t_generic 300 $PYT tests/test_gpu_generic.py
run t_all 1000 $PYT tests -m gpu
exit 0
