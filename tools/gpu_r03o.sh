#!/bin/bash
# Round-3 A/B:
# LSTM dF_{t+1} = dG_{t+1} Wi^T inside the 4-wave reverse steps (default, D) vs the separate full-grid lstm_dfeat_kernel (F).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03o}
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
run t_D 600 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_fused_env.py tests/test_gpu_ckpt.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 "$out/t_D.out"
for v in D F D F; do
  MADRONA_LEARN_LIB=$(lib $v) run l_$v 300 python bench.py --config lstm --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
  tail -1 $out/l_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('l_$v', round(d['ms_per_step'],3))"
done
run p_D 300 rocprofv3 --kernel-trace --stats -d "$out/p_D" -o run --output-format csv -- python bench.py --config lstm --steps 3 --warmup 1 --no-cpu-baseline --no-roofline
head -8 $(find $out/p_D -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4
exit 0
