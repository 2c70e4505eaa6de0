#!/bin/bash
# Diagnostic GPU session: step-kernel phase stamps (diagnostic .so) and PMC
# passes at the headline config.  Each step has its own time limit; stop at
# the first step that faults / aborts / times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${STAMPS:-1}" ] && [ "${STAMPS:-1}" != 0 ]; then
  MADRONA_LEARN_LIB=madrona-learn_amd/madrona_learn/_lib/libmlearn_stamps.so \
    timeout -k 10 300 python tools/stamp_run.py > gpurun_out/stamps.log 2>&1
  rc=$?; echo "stamps rc=$rc"; tail -n 25 gpurun_out/stamps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
bash tools/gpu_pmc.sh
