#!/bin/bash
# Round-3 A/B: LSTM gate-weight wgrad split target 1024 (T1024) vs 512 (D) on config L.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03r}
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
for v in D T1024 D T1024; do
  MADRONA_LEARN_LIB=$(lib $v) run l_$v 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  tail -1 $out/l_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('l_$v', round(d['ms_per_step'],3))"
done
exit 0
