#!/bin/bash
# Round 6: counter list, torch-path population + generic parity, PMC passes
# (MFMA busy, HBM bytes) over the headline kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_generic.py tests/test_gpu_dp_generic.py tests/test_gpu_optim_fused.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -3
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $O/pytest.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
KRE='ppo_rows16|wgrad|rollout16|reduce_grads|adam_kernel|project_kernel|gae_kernel' PASSES='SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum' bash tools/gpu_pmc.sh
rc=$?
cp -r gpurun_out/pmc $O/pmc 2>/dev/null
exit $rc
