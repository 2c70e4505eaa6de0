#!/bin/bash
# Headline bench under HIP runtime environment settings (launch-path A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-envab}
mkdir -p $O
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > $O/$name.json 2> $O/$name.err
  local rc=$?; if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -3 $O/$name.err; exit $rc; fi
  python -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['ms_per_step'],4))"
}
run base X=1
run devkarg1 HIP_FORCE_DEV_KERNARG=1
run devkarg0 HIP_FORCE_DEV_KERNARG=0
run pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run base2 X=1
exit 0
