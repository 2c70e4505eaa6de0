"""Diagnostic: per-phase cycle stamps of the row-split minibatch kernel
(ppo_rows_kernel) at the headline shape.  Run with
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
mgr = bench.make(dev, 65536, 0, 65536, use_graph=False)
mgr.update_iter()
torch.cuda.synchronize()
L = nat.lib()
L.mlearn_debug_set_stamp_buffer.argtypes = [ctypes.c_void_p]
algo = mgr.algo
ps, ts = mgr.state.policy_states, mgr.state.train_states
M = algo.mb * algo.bptt
ntiles = ((M + 63) // 64 * 64) // 32
buf = torch.zeros((ntiles, 16), dtype=torch.int64, device=dev)
L.mlearn_debug_set_stamp_buffer(buf.data_ptr())
names = {0: "tile start", 1: "L0 gather+gemm", 2: "L0 LN", 3: "Z0/A0 store", 4: "L1 W1 product",
         5: "L1 LN + A1 store", 6: "task loads + heads", 7: "loss", 8: "dhead + head bwd",
         9: "L1 LN bwd + dZ1 store", 10: "W1^T product", 11: "L0 LN bwd", 12: "dZ0 store"}
for it in range(3):
    seqs = algo.perm[0, :algo.mb]
    nat.check(L.mlearn_ppo_minibatch_grad(ps.desc, algo.view, nat.ptr(seqs), algo.mb,
                                          nat.ptr(algo.adv_stats[0, 0]), algo.hp,
                                          nat.ptr(ts.grads), None, nat.ptr(algo.ws),
                                          nat.stream_handle()))
    torch.cuda.synchronize()
st = buf.cpu().numpy().astype(np.int64)
idx = sorted(names)
print("tiles", ntiles, "cycles per phase (median / mean / max over tiles):")
for a, b in zip(idx[:-1], idx[1:]):
    d = st[:, b] - st[:, a]
    print(f"  {names[b]:28s} {np.median(d):10.0f} {d.mean():10.0f} {d.max():10.0f}")
tot = st[:, 12] - st[:, 0]
print("tile total median", np.median(tot), "mean", tot.mean())
print("kernel span", st[:, 12].max() - st[:, 0].min())
first = np.sort(st[:, 0])
print("tile start spread: first", 0, "median", np.median(first - first[0]), "max", first[-1] - first[0])
