"""Diagnostic: per-phase cycle stamps of the fused PPO minibatch kernel (B1
shape).  Run with MADRONA_LEARN_LIB=madrona-learn_amd/build_stamps/libmlearn_stamps.so
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
mgr = bench.make(dev, use_graph=False)
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
names = ["start", "L0 gemm", "L0 ln", "L1 gemm", "L1 ln", "heads", "loss", "dhead+bwd head gemm",
         "bwd L1 ln", "bwd W1 gemm", "bwd L0 ln"]
for it in range(3):
    seqs = algo.perm[0, :algo.mb]
    nat.check(L.mlearn_ppo_minibatch_grad(ps.desc, algo.view, nat.ptr(seqs), algo.mb,
                                          nat.ptr(algo.adv_stats[0, 0]), algo.hp,
                                          nat.ptr(ts.grads), None, nat.ptr(algo.ws),
                                          nat.stream_handle()))
    torch.cuda.synchronize()
st = buf.cpu().numpy().astype(np.int64)[:, :len(names)]
d = np.diff(st, axis=1)
print("tiles", ntiles, "cycles per phase (median / mean over tiles):")
for i in range(1, len(names)):
    print(f"  {names[i]:22s} {np.median(d[:, i-1]):10.0f} {d[:, i-1].mean():10.0f}")
tot = st[:, len(names) - 1] - st[:, 0]
print("tile total median", np.median(tot), "mean", tot.mean())
print("kernel span", st.max() - st.min())
