"""Diagnostic: per-phase cycle stamps of the wide fused PPO step kernel
(ppo_wide_kernel, headline shape: 65,536 rows, 128-row tiles).  Run with
MADRONA_LEARN_LIB=madrona-learn_amd/madrona_learn/_lib/libmlearn_stamps.so
(tools/build_stamps.sh); the product library never stamps."""
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
rb = int(sys.argv[1]) if len(sys.argv) > 1 else 4
algo.hp.row_blocks = rb
ntiles = ((M + 127) // 128 * 128) // (32 * rb)
W = 8
buf = torch.zeros((max(ntiles, (M + 63) // 32) * W, 16), dtype=torch.int64, device=dev)
L.mlearn_debug_set_stamp_buffer(buf.data_ptr())
names = {0: "start", 1: "gather+params+barrier", 2: "L0 product", 3: "L0 stats+barrier",
         4: "L0 apply+xchg+barrier", 5: "L1 product (+A0 stores)", 6: "L1 stats+barrier",
         7: "L1 apply+xchg+barrier", 8: "heads product (+A1 stores)", 9: "combine+barrier",
         10: "loss+metrics+barrier", 11: "dhead/hbias + bwd head product",
         12: "L1 bwd pass1 + colsums", 13: "su/sv barrier", 14: "dz + xchg + W1 product",
         15: "L0 bwd + stores"}
for it in range(3):
    seqs = algo.perm[0, :algo.mb]
    nat.check(L.mlearn_ppo_minibatch_fwd_bwd(ps.desc, algo.view, nat.ptr(seqs), algo.mb,
                                             nat.ptr(algo.adv_stats[0, 0]), algo.hp,
                                             nat.ptr(algo.ws), nat.stream_handle()))
    torch.cuda.synchronize()
st = buf.cpu().numpy().astype(np.int64)[:ntiles * W]
idx = sorted(names)
print(f"row_blocks {rb}: {ntiles} workgroups; cycles per phase (median / mean over waves):")
for a, b in zip(idx[:-1], idx[1:]):
    d = st[:, b] - st[:, a]
    print(f"  {names[b]:36s} {np.median(d):10.0f} {d.mean():10.0f}")
tot = st[:, 15] - st[:, 0]
print("wave total median", np.median(tot), "mean", tot.mean())
print("kernel span", st[:, 15].max() - st[:, 0].min())
