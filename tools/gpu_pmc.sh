#!/bin/bash
# PMC counter passes (one rocprofv3 process per pass, --kernel-trace only
# alongside --pmc) over a short eager bench run, restricted to the kernels
# matching $KRE.  Writes gpurun_out/pmc/<pass>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
KRE=${KRE:-ppo_step|wgrad|policy_step|gae}
ARGS="--steps ${STEPS:-2} --warmup 1 --no-graph --no-cpu-baseline --no-roofline ${BENCH_ARGS:-}"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 ${PASS_TIMEOUT:-300} rocprofv3 --kernel-trace --pmc $line --kernel-include-regex "$KRE" \
     -d gpurun_out/pmc/p$i -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i ($line) rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    tail -n 5 gpurun_out/pmc/p$i.log
    # a counter set the profiler refuses exits 1 or 255 without touching the GPU
    if [ $rc -ne 255 ]; then exit $rc; fi
  fi
done <<< "${PASSES:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES
TCC_HIT_sum TCC_MISS_sum
TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum
FETCH_SIZE
WRITE_SIZE}"
exit 0
