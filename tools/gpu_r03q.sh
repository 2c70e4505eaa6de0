#!/bin/bash
# Round-3 A/B: the optimizer chain with batched loads (reduce_grads strided
# sums four loads at a time; adam_kernel<PRE> preloading its grid-stride
# parameters; project_kernel<T, NS> loading every slot partial at once) (D) vs
# the serial loops (O); the LSTM gate weights' wgrad split target 256 / 512
# workgroups (T256, T512) vs 128 (D) on config L.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03q}
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
stats() {
  python - "$1" <<'PY'
import csv,sys,glob
f=glob.glob(sys.argv[1]+'/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('reduce_grads','adam','project','sumsq','wgrad')): print(' ',r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1000,2))
PY
}
run t_D 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 "$out/t_D.out"
MADRONA_LEARN_LIB=$(lib T256) run t_T256 600 python -u -m pytest tests/test_gpu_lstm.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 "$out/t_T256.out"
for v in D O D O; do
  MADRONA_LEARN_LIB=$(lib $v) run b_$v 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
  tail -1 $out/b_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b_$v', round(d['ms_per_step'],3))"
done
for v in D O D O; do
  MADRONA_LEARN_LIB=$(lib $v) run e_$v 300 python bench.py --emulate-world 8 --steps 10 --warmup 3
  tail -1 $out/e_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('e_$v', round(d['ms_per_update_rank_share'],3))"
done
for v in D O T256 T512 D O T256 T512; do
  MADRONA_LEARN_LIB=$(lib $v) run l_$v 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  tail -1 $out/l_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('l_$v', round(d['ms_per_step'],3))"
done
for v in D O; do
  MADRONA_LEARN_LIB=$(lib $v) run p_$v 300 rocprofv3 --kernel-trace --stats -d "$out/p_$v" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline
  echo p_$v; stats "$out/p_$v"
done
for v in D T256; do
  MADRONA_LEARN_LIB=$(lib $v) run pl_$v 300 rocprofv3 --kernel-trace --stats -d "$out/pl_$v" -o run --output-format csv -- python bench.py --config lstm --steps 3 --warmup 1 --no-cpu-baseline --no-roofline
  echo pl_$v; stats "$out/pl_$v"
done
exit 0
