#!/bin/bash
# Parity tests (TESTS, may be empty), then bench A/B lines: each entry of the
# ;-separated ARGS list is one bench.py run (name=args).  Stops at the first
# step that faults / aborts / times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -s -m pytest -x -v --timeout 900 --timeout-method thread -p no:cacheprovider $TESTS > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|oracle chains" $O/pytest.log | tail -4
  if [ $rc -ne 0 ]; then grep -E "^E " $O/pytest.log | head -10; exit $rc; fi
fi
IFS=';' read -ra RUNS <<< "${ARGS:-}"
for run in "${RUNS[@]}"; do
  name=${run%%=*}; a=${run#*=}
  # name@variant: bench with madrona-learn_amd/variants/libmlearn_<variant>.so
  lib=""; if [[ "$name" == *@* ]]; then lib=$PWD/madrona-learn_amd/variants/libmlearn_${name#*@}.so; fi
  MADRONA_LEARN_LIB=${lib:-$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn.so} timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline $a > $O/$name.json 2> $O/$name.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 $O/$name.err; exit $rc; fi
  python -c "import json; d=json.load(open('$O/$name.json')); k=d.get('kernels',{}); print('$name', round(d['ms_per_step'],4), 'ms', 'mb', {x: round(y,2) if isinstance(y,float) else y for x,y in k.get('minibatch',{}).items()})"
done
exit 0
