#!/bin/bash
# Round-3 A/B: policy W1 ring 6 (V1), MLP weight-gradient split target 256 (V2),
# split chunks per workgroup 16 (V3) vs the defaults (D): headline and W=8 share.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03s}
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
for v in D V1 V2 V3 D V1 V2 V3; do
  MADRONA_LEARN_LIB=$(lib $v) run b_$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
  tail -1 $out/b_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b_$v', round(d['ms_per_step'],3))"
done
for v in D V2 V3; do
  MADRONA_LEARN_LIB=$(lib $v) run e_$v 300 python bench.py --emulate-world 8 --steps 10 --warmup 3
  tail -1 $out/e_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('e_$v', round(d['ms_per_update_rank_share'],3))"
done
exit 0
