#!/bin/bash
# rocprofv3 kernel stats of one bench config: CFG=<headline|b1|lstm|pbt> EXTRA="<bench args>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-prof_${CFG:-headline}}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag -o run --output-format csv -- python bench.py --config ${CFG:-headline} --steps 5 --warmup 2 --no-cpu-baseline ${EXTRA:-} > gpurun_out/$tag.log 2>&1
rc=$?; echo "$tag rc=$rc"; exit $rc
