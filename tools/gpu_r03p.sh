#!/bin/bash
# Round-3 A/B: reduce_grads with its strided sums issued four loads at a time
# (head weight: the four parameters' loads together), project_kernel slot partials and
# sumsq_partial_kernel loads batched likewise, Adam's grid-stride parameters
# loaded before the global norm (D) vs the serial loops (O).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03p}
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
run t_D 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 "$out/t_D.out"
for v in D O D O; do
  MADRONA_LEARN_LIB=$(lib $v) run b_$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
  tail -1 $out/b_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b_$v', round(d['ms_per_step'],3))"
done
for v in D O; do
  MADRONA_LEARN_LIB=$(lib $v) run e_$v 300 python bench.py --emulate-world 8 --steps 10 --warmup 3
  tail -1 $out/e_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('e_$v', round(d['ms_per_update_rank_share'],3))"
done
for v in D O D O; do
  MADRONA_LEARN_LIB=$(lib $v) run l_$v 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  tail -1 $out/l_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('l_$v', round(d['ms_per_step'],3))"
done
for v in D O; do
  MADRONA_LEARN_LIB=$(lib $v) run p_$v 300 rocprofv3 --kernel-trace --stats -d "$out/p_$v" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline
  grep -E "reduce_grads|adam|project|sumsq" $(find $out/p_$v -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4
done
MADRONA_LEARN_LIB=$(lib D) run pl_D 300 rocprofv3 --kernel-trace --stats -d "$out/pl_D" -o run --output-format csv -- python bench.py --config lstm --steps 3 --warmup 1 --no-cpu-baseline --no-roofline
grep -E "reduce_grads|adam|project" $(find $out/pl_D -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4
exit 0
