#!/bin/bash
# Quick GPU session: GPU parity suite then the headline bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-base}
mkdir -p "$out"
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 20 "$out/$name.out"; tail -n 5 "$out/$name.err"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
run bench_headline 420 python bench.py --steps 20 --warmup 3
tail -n 1 "$out/bench_headline.out"
exit 0
