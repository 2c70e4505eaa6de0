"""The product's data-parallel collective path inside the update's HIP graph
(``DataParallel.comm``: the C ABI's RCCL communicator on the compute stream,
madrona_learn/ppo.py update_program) against the host-collective path
(torch.distributed between captured graph segments, train.py _capture /
_replay), on one GPU: rank 0 of an emulated 2-rank job
(dist.set_emulated_world) whose collectives run on a one-rank RCCL
communicator.  A one-rank all-reduce is the identity, so the two paths must
give the same store, parameters and optimizer state bit for bit over eager,
capture and replay updates; the in-graph path is ONE captured graph, the
host path one segment per collective (the advantage sums once per update,
the gradient once per minibatch).  What this leaves unexercised is only the
multi-rank transport (the ring over xGMI), which tests/test_gpu_dp.py covers
semantically over gloo."""

import pytest
import torch

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]


def _manager(gpu, W, N, H, mbl, native):
    import madrona_learn as ml
    from madrona_learn import dist as mdist
    from madrona_learn.envs import DummyVecEnv
    from tests.test_gpu_train import make_policy
    env = DummyVecEnv(N, 64, 6, seed=3, device=gpu)
    cfg = ml.TrainConfig(
        num_worlds=W * N, num_agents_per_world=1, num_updates=3,
        actions={"actions": ml.DiscreteActionsConfig(BUCKETS)}, steps_per_update=32, lr=3e-4,
        algo=ml.PPOConfig(num_epochs=2, minibatch_size=W * mbl, clip_coef=0.2,
                          value_loss_coef=0.5, entropy_coef={"actions": 0.01},
                          max_grad_norm=0.5),
        num_bptt_chunks=1, gamma=0.99, gae_lambda=0.95, seed=7, metrics_buffer_size=4,
        dreamer_v3_critic=False, compute_dtype=torch.bfloat16)
    mdist.set_emulated_world(W)
    try:
        mgr = ml.init_training(gpu, cfg, env.sim_fns(), make_policy(torch.bfloat16, H),
                               use_graph=True)
    finally:
        mdist.set_emulated_world(1)
    assert mgr.dp.world_size == W and mgr.dp.comm is not None
    if not native:
        # the host-collective path: every collective yields out of the update
        # program and runs between graph segments (identity on one rank)
        mgr.dp.comm = None
        mgr.dp.all_reduce_sum_ = lambda t: t
    return mgr


def test_rccl_in_graph_matches_segmented_host_collectives(gpu):
    W, N, H, mbl = 2, 1024, 256, 128
    a = _manager(gpu, W, N, H, mbl, native=True)
    b = _manager(gpu, W, N, H, mbl, native=False)
    assert a.dp.collectives.startswith("rccl_in_graph")
    assert a.rollout_mgr.N == N and a.algo.mb == mbl
    for _ in range(3):  # eager, capture, replay
        a.update_iter()
        b.update_iter()
    torch.cuda.synchronize()
    nmb = 2 * N // mbl  # optimizer steps per update (2 epochs)
    assert len(a._segments) == 1
    assert len(b._segments) == 1 + 1 + nmb  # advantage sums + one gradient per minibatch
    sa, sb = a.rollout_mgr.store, b.rollout_mgr.store
    for k, v in sa.as_dict().items():
        assert torch.equal(v, sb.as_dict()[k]), k
    pa, pb = a.state.policy_states, b.state.policy_states
    ta, tb = a.state.train_states, b.state.train_states
    assert torch.equal(pa.params, pb.params)
    assert not torch.equal(pa.params, torch.zeros_like(pa.params))
    for x, y in ((ta.adam_m, tb.adam_m), (ta.adam_v, tb.adam_v), (ta.step, tb.step)):
        assert torch.equal(x, y)
    assert int(ta.step.item()) == 3 * nmb
