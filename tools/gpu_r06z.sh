#!/bin/bash
# Round 6 final counters: PMC passes (MFMA busy, HBM bytes) over the headline
# kernels of the final build, config L with both weight-gradient staging
# forms under a kernel trace, and the torch-path update timing at a small N.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06z
mkdir -p $O
export TMPDIR=/tmp
KRE='ppo_rows16|wgrad|rollout16|reduce_grads|adam_kernel|project_kernel|gae_kernel' PASSES='SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum' bash tools/gpu_pmc.sh
rc=$?; rm -rf $O/pmc; cp -r gpurun_out/pmc $O/pmc 2>/dev/null
if [ $rc -ne 0 ]; then exit $rc; fi
for f in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lstm_f$f -o run --output-format csv -- python bench.py --config lstm --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --wgrad-form $f > $O/lstm_f$f.log 2>&1
  rc=$?; echo "lstm form $f rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/lstm_f$f.log; exit $rc; fi
  python tools/prof_summary.py $(find $O/lstm_f$f -name "*kernel_stats.csv" | head -1) 7 | grep -E "wgrad|total"
done
timeout -k 10 300 python tools/torch_path_bench.py 1024 8 > $O/torch_path_1024.txt 2>&1
rc=$?; tail -1 $O/torch_path_1024.txt; exit $rc
