#!/bin/bash
# Round-4: cap on weight-gradient splits at small minibatch slices (ML_WG_MIN_CHUNKS variants):
# emulated W = 8 / 4 / 2 rank shares and the headline, per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04r
mkdir -p $OUT
for rep in 1 2; do
for v in base mc8 mc16; do
  if [ $v = base ]; then unset MADRONA_LEARN_LIB; else export MADRONA_LEARN_LIB=$PWD/madrona-learn_amd/madrona_learn/_lib/libmlearn_$v.so; fi
  for w in 8 4; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --emulate-world $w > $OUT/emu${w}_$v.log 2>&1 || { echo "emu rc=$?"; tail -5 $OUT/emu${w}_$v.log; exit 6; }
    python -c "
import json
L=[l for l in open('$OUT/emu${w}_$v.log') if l.startswith('{')]
d=json.loads(L[-1]); print('rep $rep W=$w $v share', round(d['ms_per_update_rank_share'],4), 'n1', round(d['n1_ms_per_update'],4))"
  done
done
done
exit 0
