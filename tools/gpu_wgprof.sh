#!/bin/bash
# Weight-gradient staging A/B under rocprofv3 kernel traces: RUNS is a
# ;-separated list of name=variant:bench-args (variant "base" = the product
# library); prints the wgrad / step kernel averages of each run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-wgprof}
mkdir -p $O
export TMPDIR=/tmp
IFS=';' read -ra R <<< "${RUNS}"
for run in "${R[@]}"; do
  name=${run%%=*}; rest=${run#*=}; v=${rest%%:*}; a=${rest#*:}
  lib=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn.so
  [ "$v" != base ] && lib=$PWD/madrona-learn_amd/variants/libmlearn_$v.so
  MADRONA_LEARN_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline $a > $O/$name.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 $O/$name.log; exit $rc; fi
  f=$(find $O/$name -name "*kernel_stats.csv" | head -1)
  python - "$f" "$name" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    for k, tag in (("wgrad_kernel", "wgrad"), ("ppo_rows16_kernel<false", "step"), ("reduce_grads", "reduce"), ("rollout16_kernel", "rollout")):
        if k in n:
            out.append(f"{tag} {float(r['AverageNs'])/1e3:.2f}us x{r['Calls']}")
print(sys.argv[2], " | ".join(out))
PY
done
exit 0
