"""Data-parallel PPO iteration on the GPU path: two ranks (processes) share the
box's one GPU, collectives over gloo (the product issues the same
all-reduces over RCCL on a multi-GPU node).  Global semantics (SURVEY §8(d)
B8): TrainConfig.num_worlds = 2N and minibatch_size = 32 sequences describe
the whole job; each rank simulates its N-env shard and contributes 16
sequences to every global minibatch.  After one update (eager) and two more
(HIP-graph replay) both ranks must hold identical parameters, and the first
update must equal the oracle's single-process update over the union of both
ranks' minibatches: f32 at H=64 (tolerances of test_gpu_train), and bf16 at
H=256 (the production width; 256 envs and 32 sequences per rank per
minibatch) held to the per-tensor bound of tests/bf16_bound.py against the
oracle's bf16 and f32 modes (ref.ppo_update(stores=[rank0, rank1]))."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]
D, T = 64, 32
# mode -> (dtype, envs per rank N, width H, sequences per rank per minibatch, epochs)
CASES = {"f32": (torch.float32, 64, 64, 16, 2), "bf16": (torch.bfloat16, 256, 256, 32, 2),
         # the per-rank grid of the 8-GPU headline job (65,536 envs / 8 ranks, global
         # minibatch 2048 = 256 sequences per rank): 8,192-row minibatch slices, the
         # step kernel's 256 workgroups, 32 optimizer steps per epoch (one epoch
         # keeps the oracle's host time bounded)
         "bf16_w8grid": (torch.bfloat16, 8192, 256, 256, 1)}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, outdir, mode):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import madrona_learn as ml
        from madrona_learn.envs import DummyVecEnv
        from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        dtype, N, H, mbl, epochs = CASES[mode]
        env = DummyVecEnv(N, D, 6, seed=2, env_offset=rank * N, device=dev)
        cfg = ml.TrainConfig(
            num_worlds=world * N, num_agents_per_world=1, num_updates=3,
            actions={"actions": ml.DiscreteActionsConfig(BUCKETS)}, steps_per_update=T,
            lr=3e-4, algo=ml.PPOConfig(num_epochs=epochs, minibatch_size=mbl * world, clip_coef=0.2,
                                       value_loss_coef=0.5, entropy_coef={"actions": 0.01},
                                       max_grad_norm=0.5),
            num_bptt_chunks=1, gamma=0.99, gae_lambda=0.95, seed=5, metrics_buffer_size=4,
            dreamer_v3_critic=False, compute_dtype=dtype)
        policy = ml.Policy(actor_critic=ml.ActorCritic(
            backbone=ml.BackboneShared(encoder=ml.BackboneEncoder(net=MLP(H, 2, dtype))),
            actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dtype),
            critic=DenseLayerCritic(dtype)))
        mgr = ml.init_training(dev, cfg, env.sim_fns(), policy, use_graph=True)
        ps, ts = mgr.state.policy_states, mgr.state.train_states
        assert mgr.rollout_mgr.N == N and mgr.algo.mb == mbl, "global config must split per rank"
        p0 = ps.params.cpu().numpy()
        mgr.update_iter()
        torch.cuda.synchronize()
        s = mgr.rollout_mgr.store
        store = {k: (v.float() if v.dtype == torch.bfloat16 else v).cpu().numpy()
                 for k, v in s.as_dict().items()}
        p1 = ps.params.cpu().numpy()
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), p0=p0, p1=p1,
                 init_norms=ps.init_norms.cpu().numpy(), key=np.array(ts.update_prng_key),
                 **{f"s_{k}": v for k, v in store.items()})
        for _ in range(2):
            mgr.update_iter()
        torch.cuda.synchronize()
        np.save(os.path.join(outdir, f"rank{rank}_p3.npy"), ps.params.cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["f32", "bf16", "bf16_w8grid"])
def test_dp_two_ranks_one_gpu(tmp_path, mode):
    from oracle import ppo_ref as ref
    _, N, H, mbl, epochs = CASES[mode]
    mp.spawn(worker, args=(2, _free_port(), str(tmp_path), mode), nprocs=2, join=True)
    r = [np.load(os.path.join(tmp_path, f"rank{i}.npz")) for i in range(2)]
    p3 = [np.load(os.path.join(tmp_path, f"rank{i}_p3.npy")) for i in range(2)]
    assert np.array_equal(r[0]["p0"], r[1]["p0"]), "initial params differ across ranks"
    assert np.array_equal(r[0]["p1"], r[1]["p1"]), "ranks diverged after the eager update"
    assert np.array_equal(p3[0], p3[1]), "ranks diverged under graph replay"
    assert not np.array_equal(r[0]["s_obs"], r[1]["s_obs"]), "env shards must differ"
    stores = [{k[2:]: ri[k] for k in ri.files if k.startswith("s_")} for ri in r]
    lay = ref.param_layout(D, H, 2, sum(BUCKETS))
    p0 = r[0]["p0"].astype(np.float64)
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
          "normalize_advantages": True}
    z = np.zeros_like(p0)
    upd = dict(num_epochs=epochs, minibatch_size=mbl, bptt=T,
               key=tuple(int(x) for x in r[0]["key"]), epoch_base=0, lr=3e-4, max_grad_norm=0.5)
    norms = r[0]["init_norms"].astype(np.float64)
    omode = "bf16" if mode.startswith("bf16") else mode
    p_ref, _, _ = ref.ppo_update(p0, (z, z.copy(), 0), stores, hp, BUCKETS, lay, norms,
                                 mode=omode, **upd)
    if mode == "f32":
        np.testing.assert_allclose(r[0]["p1"], p_ref, rtol=1e-4, atol=2e-5)
        return
    from tests.bf16_bound import check_bf16_update
    p_f32, _, _ = ref.ppo_update(p0, (z, z.copy(), 0), stores, hp, BUCKETS, lay, norms,
                                 mode="f32", **upd)
    check_bf16_update(f"dp_world2_H256_{mode}", r[0]["p1"], p0, p_ref, p_f32, lay)
    dg, dr = r[0]["p1"] - p0, p_ref - p0
    assert dg @ dr / (np.linalg.norm(dg) * np.linalg.norm(dr)) > 0.99
