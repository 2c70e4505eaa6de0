"""Data-parallel protocol of the PPO update (madrona_learn/ppo.py
update_program + dist.DataParallel) on world_size 2 over gloo (CPU).

Each rank owns its own environment shard (env_offset = rank * N) and rollout;
per epoch the ranks all-reduce the per-minibatch advantage sums (zscore_data
over the global minibatch, algo_common.py:133-140) and per minibatch the flat
gradient computed with loss_scale = 1/world, then apply the identical
optimizer step.  The result must equal the single-process update over the
union of the ranks' minibatches (oracle ppo_update with both stores), and
both ranks must hold identical parameters.  The arithmetic runs on the
oracle (the GPU kernels are covered by the -m gpu tests); the collectives
run through the product's DataParallel wrapper."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import native
from oracle import ppo_ref as ref

BUCKETS = [4, 8, 5, 5, 2, 2]
N, D, H, L, T = 16, 16, 64, 2, 8
EPOCHS, MB = 2, 8
HP = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
      "normalize_advantages": True}
LR, MAXN = 3e-4, 0.5
KEY = (17, 23)


def make_params():
    lay = ref.param_layout(D, H, L, sum(BUCKETS))
    rng = np.random.default_rng(0)
    p = rng.standard_normal(lay["total"]) * 0.2
    for o, shp in lay["s"]:
        p[o:o + shp[0]] += 1.0
    init = np.array([np.linalg.norm(ref.unflatten(p, lay)["W"][l]) for l in range(L)])
    return lay, p, init


def rank_store(rank, lay, p):
    env = native.Env(N, D, 5, 6, rank * N)
    env.reset()
    store, _ = ref.rollout(p, lay, env, T, BUCKETS, (1, 2), 0, mode="f64")
    adv, ret = ref.gae(store["rewards"], store["values"], store["dones"], store["bootstrap"],
                       0.99, 0.95)
    store["advantages"], store["returns"] = adv, ret
    return store


def dp_update(rank, world, lay, p, init, store, comm):
    """PPO.update_program's exchange protocol, arithmetic on the oracle."""
    nseq = N  # bptt = T, one chunk
    nmb = nseq // MB
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    count = 0
    for e in range(EPOCHS):
        perm = ref.epoch_permutation(KEY[0], KEY[1], e, rank, nseq)
        # per-minibatch advantage sums, all-reduced once per epoch
        sums = torch.zeros(2 * nmb, dtype=torch.float64)
        batches = []
        for j in range(nmb):
            b = ref.gather_minibatch(store, ref.minibatch_rows(perm[j * MB:(j + 1) * MB], N, T))
            a = np.asarray(b["advantages"], np.float64)
            sums[2 * j], sums[2 * j + 1] = a.sum(), (a * a).sum()
            batches.append(b)
        comm.all_reduce_sum_(sums)
        cnt = world * MB * T
        for j in range(nmb):
            mean = sums[2 * j].item() / cnt
            var = sums[2 * j + 1].item() / cnt - mean * mean
            _, G, _, _ = ref.ppo_loss_grads(ref.unflatten(p, lay), batches[j], HP, BUCKETS,
                                            "f64", adv_stats=(mean, var), loss_scale=1.0 / world)
            g = torch.from_numpy(ref.flatten(G, lay))
            comm.all_reduce_sum_(g)
            p, m, v, _ = ref.optimizer_step(p, g.numpy(), m, v, count, lay, init, LR, MAXN)
            count += 1
    return p


def worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from madrona_learn.dist import DataParallel
        comm = DataParallel()
        assert comm.world_size == world and comm.rank == rank
        lay, p, init = make_params()
        store = rank_store(rank, lay, p)
        p_dp = dp_update(rank, world, lay, p, init, store, comm)
        gathered = [None] * world
        dist.all_gather_object(gathered, (p_dp, {k: store[k] for k in store}))
        if rank == 0:
            stores = [g[1] for g in gathered]
            p_ref, _, _ = ref.ppo_update(p.copy(), (np.zeros_like(p), np.zeros_like(p), 0), stores,
                                         HP, BUCKETS, lay, init, num_epochs=EPOCHS,
                                         minibatch_size=MB, bptt=T, key=KEY, epoch_base=0,
                                         mode="f64", lr=LR, max_grad_norm=MAXN)
            np.save(out, np.stack([gathered[0][0], gathered[1][0], p_ref, p]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_dp_world2_equals_union_update(tmp_path):
    out = str(tmp_path / "params.npy")
    mp.spawn(worker, args=(2, _free_port(), out), nprocs=2, join=True)
    p0, p1, p_ref, p_init = np.load(out)
    assert np.array_equal(p0, p1), "ranks diverged"
    assert not np.allclose(p0, p_init)
    np.testing.assert_allclose(p0, p_ref, rtol=1e-10, atol=1e-12)
