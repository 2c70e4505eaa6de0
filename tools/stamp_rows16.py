"""Diagnostic: per-phase s_memtime stamps of the row-split step kernel
(ppo_rows16.h) at the headline shape.  Run with
MADRONA_LEARN_LIB=madrona-learn_amd/variants/libmlearn_stamps.so
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
tiles = ((M + 63) // 64 * 64) // 16  # 16-row tiles
buf = torch.zeros((tiles, 16), dtype=torch.int64, device=dev)
L.mlearn_debug_set_stamp_buffer(buf.data_ptr())
names = {1: "L0 x loads + fwd + stats", 2: "X0/dZ0 stores + LN0 apply",
         3: "task loads + L1 product + stats", 4: "A0 store + LN1 apply",
         5: "heads + A1 store + logits", 6: "loss", 7: "dhead store + hb sums",
         8: "head bwd + LN1 bwd", 9: "W1^T product", 10: "dZ1 store",
         11: "Z0 recompute", 12: "LN0 bwd"}
for it in range(3):
    buf.zero_()
    seqs = algo.perm[0, :algo.mb]
    nat.check(L.mlearn_ppo_minibatch_grad(ps.desc, algo.view, nat.ptr(seqs), algo.mb,
                                          nat.ptr(algo.adv_stats[0, 0]), algo.hp,
                                          nat.ptr(ts.grads), None, nat.ptr(algo.ws),
                                          nat.stream_handle()))
    torch.cuda.synchronize()
st = buf.cpu().numpy().astype(np.int64)
w0 = st[0::2]  # tile 0 rows of each wave: [13] entry, [14] after prologue, [15] end
print("per wave (cycles, median / max): prologue", np.median(w0[:, 14] - w0[:, 13]),
      (w0[:, 14] - w0[:, 13]).max(), "| tiles", np.median(st[1::2, 12] - w0[:, 0]),
      "| epilogue (last stores done)", np.median(w0[:, 15] - st[1::2, 12]),
      (w0[:, 15] - st[1::2, 12]).max(), "| entry..end", np.median(w0[:, 15] - w0[:, 13]),
      (w0[:, 15] - w0[:, 13]).max())
# per workgroup (8 waves, one CU): wave time entry..end by wave index, and the
# spread inside a workgroup vs across workgroups
tw = (w0[:, 15] - w0[:, 13]).reshape(-1, 8)
print("wave time by wave index (median over WGs):", [int(x) for x in np.median(tw, 0)])
print("WG max/min ratio median", float(np.median(tw.max(1) / tw.min(1))),
      "| WG max: median", float(np.median(tw.max(1))), "max", int(tw.max()),
      "| WG mean: min", float(tw.mean(1).min()), "max", float(tw.mean(1).max()))
end_rel = (w0[:, 15] - w0[:, 13].reshape(-1, 8).min(1).repeat(8)).reshape(-1, 8)
print("WG finish (from its first wave's entry): median", float(np.median(end_rel.max(1))),
      "max", int(end_rel.max()))
ok = st[:, 12] != 0
st = st[ok]
print("tiles stamped", int(ok.sum()), "of", tiles, "- cycles per phase (median / mean / max):")
for i in range(1, 13):
    d = st[:, i] - st[:, i - 1]
    print(f"  {names[i]:34s} {np.median(d):9.0f} {d.mean():9.0f} {d.max():9.0f}")
tot = st[:, 12] - st[:, 0]
print("tile total median", np.median(tot), "mean", tot.mean())
print("kernel span", st[:, 12].max() - st[:, 0].min())
first = st[:, 0] - st[:, 0].min()
print("tile start spread: median", np.median(first), "max", first.max())
