"""Data parallelism on the torch path (madrona_learn/generic.py): a
BackboneSeparate tree (actor_critic.py:247-303), which the fused kernels do
not implement, trained by two ranks sharing the box's GPU, collectives over
gloo (the product issues the same all-reduces over RCCL on a multi-GPU
node).  Global semantics as tests/test_gpu_dp.py: num_worlds = 2N and
minibatch_size = 32 sequences describe the whole job, each rank contributes
16 sequences to every global minibatch (ppo.py:366-488 under the reference's
data-parallel update).  Both ranks must hold identical parameters after every
update, and the first update must equal oracle/separate_ref.py's update over
the union of both ranks' minibatches (union advantage statistics, gradients
summed over ranks at loss scale 1/2), at the f32 tolerances of
tests/test_gpu_generic.py's single-rank update."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]
D, T, N, H, L, MBL = 64, 32, 64, 64, 2, 16


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _named(ps):
    return {n: ps.params[o:o + int(np.prod(s))].cpu().numpy().astype(np.float64).reshape(s)
            for n, o, s in ps.layout["params"]}


def worker(rank, world, port, outdir):
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
        dt = torch.float32
        env = DummyVecEnv(N, D, 6, seed=2, env_offset=rank * N, device=dev)
        cfg = ml.TrainConfig(
            num_worlds=world * N, num_agents_per_world=1, num_updates=3,
            actions={"actions": ml.DiscreteActionsConfig(BUCKETS)}, steps_per_update=T,
            lr=3e-4, algo=ml.PPOConfig(num_epochs=2, minibatch_size=MBL * world, clip_coef=0.2,
                                       value_loss_coef=0.5, entropy_coef={"actions": 0.01},
                                       max_grad_norm=0.5),
            num_bptt_chunks=1, gamma=0.99, gae_lambda=0.95, seed=5, metrics_buffer_size=4,
            dreamer_v3_critic=False, compute_dtype=dt)
        ac = ml.ActorCritic(
            backbone=ml.BackboneSeparate(actor_encoder=ml.BackboneEncoder(net=MLP(H, L, dt)),
                                         critic_encoder=ml.BackboneEncoder(net=MLP(H, L, dt))),
            actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dt),
            critic=DenseLayerCritic(dt))
        mgr = ml.init_training(dev, cfg, env.sim_fns(), ml.Policy(actor_critic=ac),
                               use_graph=True)
        ps, ts = mgr.state.policy_states, mgr.state.train_states
        assert getattr(ps, "generic", False), "BackboneSeparate must take the torch path"
        assert mgr.rollout_mgr.N == N and mgr.algo.mb == MBL, "global config must split per rank"
        p0 = ps.params.cpu().numpy()
        mgr.update_iter()
        torch.cuda.synchronize()
        s = mgr.rollout_mgr.store
        store = {k: (v.float() if v.dtype == torch.bfloat16 else v).cpu().numpy()
                 for k, v in s.as_dict().items()}
        p1 = ps.params.cpu().numpy()
        names = np.array([n for n, _, _ in ps.layout["params"]])
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), p0=p0, p1=p1, names=names,
                 key=np.array(ts.update_prng_key), step=np.array(int(ts.step.item())),
                 **{f"s_{k}": v for k, v in store.items()})
        for _ in range(2):
            mgr.update_iter()
        torch.cuda.synchronize()
        np.save(os.path.join(outdir, f"rank{rank}_p3.npy"), ps.params.cpu().numpy())
        with open(os.path.join(outdir, f"rank{rank}_layout.txt"), "w") as f:
            for n, o, shp in ps.layout["params"]:
                f.write(f"{n} {o} {' '.join(str(x) for x in shp)}\n")
    finally:
        dist.destroy_process_group()


def _unflat(vec, layout_file):
    out = {}
    with open(layout_file) as f:
        for line in f:
            parts = line.split()
            n, o, shp = parts[0], int(parts[1]), tuple(int(x) for x in parts[2:])
            out[n] = vec[o:o + int(np.prod(shp))].astype(np.float64).reshape(shp)
    return out


def test_dp_backbone_separate_two_ranks(tmp_path):
    from oracle import separate_ref as sref
    mp.spawn(worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [np.load(os.path.join(tmp_path, f"rank{i}.npz")) for i in range(2)]
    p3 = [np.load(os.path.join(tmp_path, f"rank{i}_p3.npy")) for i in range(2)]
    assert np.array_equal(r[0]["p0"], r[1]["p0"]), "initial params differ across ranks"
    assert np.array_equal(r[0]["p1"], r[1]["p1"]), "ranks diverged after the first update"
    assert np.array_equal(p3[0], p3[1]), "ranks diverged over later updates"
    assert np.isfinite(p3[0]).all() and not np.array_equal(p3[0], r[0]["p1"])
    assert not np.array_equal(r[0]["s_obs"], r[1]["s_obs"]), "env shards must differ"
    assert int(r[0]["step"]) == 2 * (N // MBL)
    lay = os.path.join(tmp_path, "rank0_layout.txt")
    order = [str(n) for n in r[0]["names"]]
    p0 = _unflat(r[0]["p0"], lay)
    init_norms = {k: float(np.sqrt((v * v).sum())) for k, v in p0.items()
                  if k.endswith("kernel") and k.startswith("backbone.")}
    assert len(init_norms) == 2 * L
    stores = [{k[2:]: ri[k] for k in ri.files if k.startswith("s_")} for ri in r]
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
          "normalize_advantages": True}
    want, _ = sref.ppo_update(dict(p0), order, stores, hp, BUCKETS, L, init_norms,
                              num_epochs=2, minibatch_size=MBL, bptt=T,
                              key=tuple(int(x) for x in r[0]["key"]), epoch_base=0,
                              mode="f32", lr=3e-4, max_grad_norm=0.5)
    got = _unflat(r[0]["p1"], lay)
    g = np.concatenate([got[k].reshape(-1) for k in order])
    w = np.concatenate([want[k].reshape(-1) for k in order])
    z = np.concatenate([p0[k].reshape(-1) for k in order])
    # the tolerances of tests/test_gpu_generic.py's single-rank f32 update
    np.testing.assert_allclose(g, w, rtol=0, atol=1e-4)
    close = np.abs(g - w) <= 2e-5 + 1e-4 * np.abs(w)
    assert close.mean() >= 0.999, close.mean()
    dg, dw = g - z, w - z
    assert dg @ dw / (np.linalg.norm(dg) * np.linalg.norm(dw)) > 0.999
    # a single-rank oracle update over rank 0's store alone must NOT match:
    # the test sees the union semantics, not one rank's
    solo, _ = sref.ppo_update(dict(p0), order, stores[0], hp, BUCKETS, L, init_norms,
                              num_epochs=2, minibatch_size=MBL, bptt=T,
                              key=tuple(int(x) for x in r[0]["key"]), epoch_base=0,
                              mode="f32", lr=3e-4, max_grad_norm=0.5)
    s = np.concatenate([solo[k].reshape(-1) for k in order])
    assert np.abs(g - s).max() > 10 * np.abs(g - w).max()
