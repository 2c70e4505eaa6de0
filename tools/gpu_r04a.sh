#!/bin/bash
# Round-4 check: the full -m gpu parity suite (new: gamma*lambda constant,
# env tiles in series in the whole-rollout launch, headline tile rounds;
# dead kernel variants removed), then one headline bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r04a/pytest.log 2>&1
rc=$?
tail -n 15 gpurun_out/r04a/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.err
rc=$?
tail -c 600 gpurun_out/r04a/bench.json
exit $rc
