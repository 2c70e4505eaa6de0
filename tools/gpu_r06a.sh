#!/bin/bash
# Round-6 first session: counter list, the new ADVICE tests, a headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06a
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/r06a/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_obsnorm.py::test_bare_obs_normalizer_state_survives_checkpoint \
  tests/test_gpu_generic.py::test_wide_head_routes_to_torch_path > gpurun_out/r06a/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r06a/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/r06a/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r06a/bench.log
exit $rc
