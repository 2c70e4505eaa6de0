#!/bin/bash
# Round-3 A/B: LSTM per-step scan ring depths (k-steps of Wh / dG fragments
# in flight per wave) and the 4-wave forward, as variant libraries
# (MADRONA_LEARN_LIB): default (fwd 1-wave depth 8, bwd 4-wave depth 8),
# A (fwd 4-wave 17, bwd 17), B (fwd 4-wave 12, bwd 17), C (fwd 1-wave 12, bwd 12).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03l}
mkdir -p "$out"
export TMPDIR=/tmp
V=madrona-learn_amd/madrona_learn/_lib/var
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$out/$name.out" 2> "$out/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 40 "$out/$name.out"; tail -n 5 "$out/$name.err"; exit $rc; fi
}
for v in A B C; do
  MADRONA_LEARN_LIB=$PWD/$V/libmlearn_$v.so run t_$v 600 python -u -m pytest tests/test_gpu_lstm.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
  tail -n 1 "$out/t_$v.out"
done
for v in D A B C D A B C; do
  lib=$PWD/$V/libmlearn_$v.so; [ $v = D ] && lib=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn.so
  MADRONA_LEARN_LIB=$lib run l_$v 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  tail -1 $out/l_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('l_$v', round(d['ms_per_step'],3))"
done
for v in D A B C; do
  lib=$PWD/$V/libmlearn_$v.so; [ $v = D ] && lib=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn.so
  MADRONA_LEARN_LIB=$lib run p_$v 300 rocprofv3 --kernel-trace --stats -d "$out/p_$v" -o run --output-format csv -- python bench.py --config lstm --steps 3 --warmup 1 --no-cpu-baseline --no-roofline
  f=$(ls $out/p_$v/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(find $out/p_$v -name '*kernel_stats.csv' | head -1)
  grep -E "lstm_(fwd|bwd)_step" "$f" | cut -d, -f1-4
done
exit 0
