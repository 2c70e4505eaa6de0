#!/bin/bash
# Round-3 A/B of the weight-gradient split target at the W=8 rank share
# (emulation) and at W=1: ML_WG_TARGET 128 (default) / 64 / 32.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03j}
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
L=madrona-learn_amd/madrona_learn/_lib
for v in main wgt64 wgt32 main wgt64; do
  lib=$L/libmlearn.so; [ $v != main ] && lib=$L/libmlearn_$v.so
  MADRONA_LEARN_LIB=$lib run e8_$v 300 python bench.py --emulate-world 8 --steps 10 --warmup 3
  python -c "import json; d=json.load(open('$out/e8_$v.out')); print('e8 $v', round(d['ms_per_update_rank_share'],3), 'n1', round(d['n1_ms_per_update'],3))"
done
exit 0
