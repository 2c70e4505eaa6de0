"""Diagnostic: per-phase cycle stamps of the fused PPO minibatch kernel (headline
shape).  Run with MADRONA_LEARN_LIB=madrona-learn_amd/madrona_learn/_lib/libmlearn_stamps.so
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
W = 8  # waves per step-kernel workgroup at H = 256 (ML_STEP_MAXW)
buf = torch.zeros((ntiles * W, 16), dtype=torch.int64, device=dev)
L.mlearn_debug_set_stamp_buffer(buf.data_ptr())
# stamp index -> phase ending there (L = 2)
names = {0: "prologue", 1: "L0 gemm", 2: "L0 stats+barrier", 4: "L0 apply+xchg+L1 gemm",
         5: "L1 stats+barrier", 6: "L1 apply", 7: "heads+reduce", 8: "loss+partials",
         9: "dhead/hb", 10: "bwd head gemm+L1 bwd pass1", 11: "L1 su/sv xchg+dz",
         12: "dz xchg+W1 gemm", 13: "L0 bwd pass1", 14: "L0 xchg+dz", 15: "end"}
for it in range(3):
    seqs = algo.perm[0, :algo.mb]
    nat.check(L.mlearn_ppo_minibatch_grad(ps.desc, algo.view, nat.ptr(seqs), algo.mb,
                                          nat.ptr(algo.adv_stats[0, 0]), algo.hp,
                                          nat.ptr(ts.grads), None, nat.ptr(algo.ws),
                                          nat.stream_handle()))
    torch.cuda.synchronize()
st = buf.cpu().numpy().astype(np.int64)
idx = sorted(names)
print("tiles", ntiles, "cycles per phase (median / mean over waves):")
for a, b in zip(idx[:-1], idx[1:]):
    d = st[:, b] - st[:, a]
    print(f"  {names[b]:30s} {np.median(d):10.0f} {d.mean():10.0f}")
tot = st[:, 15] - st[:, 0]
print("wave total median", np.median(tot), "mean", tot.mean())
print("kernel span", st[:, 15].max() - st[:, 0].min())
