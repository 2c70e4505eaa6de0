#!/bin/bash
# Round-6 spill probes (verdict r05 item 1): headline bench A/B of the
# X0 / A0 store probes (timing only), the weight-gradient launch run twice
# (second launch reads cache-hot operands) under a kernel trace, and the
# two-rank slice (32 768 rows: half-minibatch step / wgrad) under a trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r06p}
mkdir -p $O
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$O/$name.out" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 5 "$O/$name.err"; exit $rc; fi
}
V=$PWD/madrona-learn_amd/variants
B=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn.so
for rep in 1 2; do
  for v in base nox0 noa0; do
    lib=$B; [ $v != base ] && lib=$V/libmlearn_$v.so
    MADRONA_LEARN_LIB=$lib run ab_${v}_$rep 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
    python -c "import json; d=json.load(open('$O/ab_${v}_$rep.out')); k=d.get('kernels',{}); print('$v', round(d['ms_per_step'],4), 'ms', {x: round(y,2) if isinstance(y,float) else y for x,y in k.get('minibatch',{}).items()})"
  done
done
MADRONA_LEARN_LIB=$V/libmlearn_wg2.so run prof_wg2 420 rocprofv3 --kernel-trace --stats -d $O/prof_wg2 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
python tools/wg_pairs.py $(find $O/prof_wg2 -name "*kernel_trace.csv" | head -1)
run prof_emu2 420 rocprofv3 --kernel-trace --stats -d $O/prof_emu2 -o run --output-format csv -- python bench.py --emulate-world 2 --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
python tools/prof_summary.py $(find $O/prof_emu2 -name "*kernel_stats.csv" | head -1) | head -12
run prof_base 420 rocprofv3 --kernel-trace --stats -d $O/prof_base -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline
python tools/prof_summary.py $(find $O/prof_base -name "*kernel_stats.csv" | head -1) | head -12
exit 0
