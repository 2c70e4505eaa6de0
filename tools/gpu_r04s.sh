#!/bin/bash
# Round-4: the small-slice split cap as the default: parity of the affected paths, emulated shares.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04s
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dp.py tests/test_gpu_emulated_dp.py tests/test_gpu_fullsize.py tests/test_gpu_train.py tests/test_gpu_policy.py tests/test_gpu_configs.py > $OUT/t.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/t.log; exit 3; }
tail -1 $OUT/t.log
for w in 8 4 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --emulate-world $w > $OUT/emu$w.log 2>&1 || { echo "emu rc=$?"; tail -5 $OUT/emu$w.log; exit 6; }
  python -c "
import json
L=[l for l in open('$OUT/emu$w.log') if l.startswith('{')]
d=json.loads(L[-1]); print('W=$w share', round(d['ms_per_update_rank_share'],4), 'n1', round(d['n1_ms_per_update'],4), 'modeled', round(d['ms_per_update_rank_share_with_modeled_allreduce'],4))"
done
exit 0
