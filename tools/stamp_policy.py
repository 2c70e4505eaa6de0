"""Diagnostic: per-phase cycle stamps of the rollout policy kernel at the
headline shape (65 536 envs, MLP[256,256], bf16).  Run with
MADRONA_LEARN_LIB=madrona-learn_amd/madrona_learn/_lib/libmlearn_stamps.so
(tools/build_stamps.sh)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "madrona-learn_amd")]
import bench  # noqa: E402
from madrona_learn import _native as nat  # noqa: E402

dev = torch.device("cuda:0")
N = 65536
mgr = bench.make(dev, N, 0, N, use_graph=False)
mgr.update_iter()
torch.cuda.synchronize()
L = nat.lib()
L.mlearn_debug_set_policy_stamp_buffer.argtypes = [ctypes.c_void_p]
W = 4  # waves per policy workgroup at H = 256 (ML_POL_MAXW)
buf = torch.zeros((N // 32 * W, 16), dtype=torch.int64, device=dev)
L.mlearn_debug_set_policy_stamp_buffer(buf.data_ptr())
for _ in range(3):
    mgr.update_iter()
    torch.cuda.synchronize()
st = buf.cpu().numpy().astype(np.int64)
names = {0: "prologue", 1: "L0 gemm (obs gather)", 2: "L0 stats+barrier",
         3: "L0 apply+xchg+L1 gemm", 4: "L1 stats+barrier", 5: "L1 apply", 6: "heads+reduce",
         7: "gumbel (philox)", 8: "pick+store", 9: "values/end"}
idx = sorted(names)
print("blocks", N // 32, "cycles per phase (median / mean over waves), last sampling launch of the update:")
for a, b in zip(idx[:-1], idx[1:]):
    d = st[:, b] - st[:, a]
    print(f"  {names[b]:28s} {np.median(d):10.0f} {d.mean():10.0f}")
tot = st[:, 9] - st[:, 0]
print("wave total median", np.median(tot), "mean", tot.mean())
print("kernel span", st[:, 9].max() - st[:, 0].min())
