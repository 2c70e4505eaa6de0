"""The built-in synthetic sim's step fused into the rollout policy launch
(mlearn_policy_rollout_step_env, envs.DummyVecEnv.native_step) is
bit-identical to calling the sim's own step between the launches
(mlearn_dummy_env_step), and so is the whole rollout as one launch
(mlearn_policy_rollout_env): same store, env state, observations, rewards,
dones and parameters after whole update iterations, eager and graph-captured,
for MLP / population / LSTM policies, including a partial last workgroup of
envs.  The oracle parity of the fused path itself is tests/test_gpu_train.py
(the store against the oracle env, bit for bit), which runs fused by default."""

import pytest
import torch

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]


def _manager(gpu, fused, dtype, N, H, mb, P=1, lstm=False, use_graph=False):
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from tests.test_gpu_train import make_policy
    env = DummyVecEnv(N, 64, 6, seed=4, device=gpu)
    pbt = None
    if P > 1:
        pbt = ml.PBTConfig(num_teams=1, team_size=1, num_train_policies=P, num_past_policies=0,
                           self_play_portion=1.0, cross_play_portion=0.0, past_play_portion=0.0)
    cfg = ml.TrainConfig(
        num_worlds=N, num_agents_per_world=1, num_updates=2,
        actions={"actions": ml.DiscreteActionsConfig(BUCKETS)}, steps_per_update=32,
        lr=3e-4, algo=ml.PPOConfig(num_epochs=2, minibatch_size=mb, clip_coef=0.2,
                                   value_loss_coef=0.5, entropy_coef={"actions": 0.01},
                                   max_grad_norm=0.5),
        num_bptt_chunks=1, gamma=0.99, gae_lambda=0.95, seed=11, metrics_buffer_size=4,
        dreamer_v3_critic=False, compute_dtype=dtype, pbt=pbt)
    if lstm:
        from tests.test_gpu_lstm import make_actor_critic
        pol = ml.Policy(actor_critic=make_actor_critic(H, 2, dtype, 1),
                        obs_preprocess=ml.ObservationsCaster.create(dtype))
    else:
        pol = make_policy(dtype, H)
    fns = env.sim_fns(fused=fused)
    assert ("native_step" in fns) == fused
    return env, ml.init_training(gpu, cfg, fns, pol, use_graph=use_graph)


@pytest.mark.parametrize("mode", ["one_launch", "multi_tile", "c_per_step", "py_per_step"])
@pytest.mark.parametrize("dtype,N,H,mb,P,lstm,graph", [
    (torch.float32, 80, 64, 16, 1, False, False),    # partial last workgroup (80 = 2.5 x 32)
    (torch.bfloat16, 1024, 256, 256, 1, False, True),
    (torch.float32, 128, 64, 16, 2, False, True),     # population: one launch for both policies
    (torch.bfloat16, 384, 256, 32, 3, False, True),   # 3 policies x 4 tiles in one launch
    (torch.float32, 128, 64, 32, 2, True, True),      # population of LSTM policies
    (torch.bfloat16, 128, 256, 32, 1, True, False),   # LSTM H = 256: carry, start states, clears
    (torch.float32, 64, 64, 32, 1, True, False)])     # LSTM carry + done clears
def test_fused_env_step_is_bit_identical(gpu, mode, dtype, N, H, mb, P, lstm, graph):
    """one_launch: the whole rollout + bootstrap in one launch
    (mlearn_policy_rollout_env, one workgroup per env tile here; a
    population: mlearn_policy_rollout_env_pop over every policy's tiles);
    multi_tile: the same launch capped at 2 workgroups (1 for a 2-tile
    policy; mlearn_rollout_out.max_workgroups), so every workgroup runs several
    env tiles in series with the parameters it staged in LDS once (the
    headline's 2048 tiles on 768 resident workgroups take this branch); a
    population's launch under the same cap deals tiles of every policy to
    each workgroup, which restages the parameters when its next tile belongs
    to another policy (config P's 2048 tiles on 768 slots take that branch);
    c_per_step: the same entry's per-step launches (max_workgroups = -1);
    py_per_step: one rollout_step_env call per step from the host."""
    from madrona_learn import _native as nat
    from madrona_learn.rollouts import RolloutManager
    env_a, a = _manager(gpu, True, dtype, N, H, mb, P, lstm, graph)
    env_b, b = _manager(gpu, False, dtype, N, H, mb, P, lstm, graph)
    rm = a.rollout_mgr
    rm.whole_rollout = mode != "py_per_step"
    tiles = (rm.B + 31) // 32
    cap = 2 if tiles > 2 else 1
    rm.rollout_workgroups = {"multi_tile": cap, "c_per_step": -1}.get(mode, 0)
    ps = rm.policies[0]
    grid = nat.lib().mlearn_policy_rollout_workgroups(ps.desc, ps.lstm_desc, rm.B,
                                                      rm.rollout_workgroups)
    if mode == "multi_tile":
        assert grid == cap and tiles > grid, (grid, tiles)
        if P > 1:
            pg = nat.lib().mlearn_policy_rollout_pop_workgroups(ps.desc, ps.lstm_desc, rm.B, P,
                                                                cap)
            assert pg == cap
            # workgroup 0's tiles 0, cap, 2 cap, ... span more than one policy
            assert len({g // tiles for g in range(0, P * tiles, pg)}) > 1
    elif mode == "c_per_step":
        assert grid == -1
    elif mode == "one_launch":
        assert grid == tiles
    if P > 1 and mode in ("one_launch", "multi_tile"):
        # the population launch ran (its arguments were prepared)
        a.update_iter()
        assert getattr(rm, "_pop_sig", None) is not None
        b.update_iter()
    assert RolloutManager.rollout_workgroups == 0  # instance setting only
    for _ in range(2):
        a.update_iter()
        b.update_iter()
    torch.cuda.synchronize()
    sa, sb = a.rollout_mgr.store, b.rollout_mgr.store
    for k, v in sa.as_dict().items():
        assert torch.equal(v, sb.as_dict()[k]), k
    assert torch.equal(sa.env_returns_trace, sb.env_returns_trace)
    assert torch.equal(sa.bootstrap, sb.bootstrap)
    for x, y in ((env_a.state, env_b.state), (env_a.obs, env_b.obs),
                 (env_a.rewards, env_b.rewards), (env_a.dones, env_b.dones)):
        assert torch.equal(x, y)
    pa = a.state.policy_list if P > 1 else [a.state.policy_states]
    pb = b.state.policy_list if P > 1 else [b.state.policy_states]
    for x, y in zip(pa, pb):
        assert torch.equal(x.params, y.params)
    # the fused run issued no sim launch: its env buffers moved anyway
    iters = 3 if (mode in ("one_launch", "multi_tile") and P > 1) else 2
    assert int(env_a.state[:, 1].min().item()) == 32 * iters


def test_fused_env_rejects_foreign_obs(gpu):
    """env->obs must be the launch's own obs input (the next observations
    overwrite it in place)."""
    import madrona_learn as ml  # noqa: F401
    from madrona_learn import _native as nat
    from madrona_learn.envs import DummyVecEnv
    _, mgr = _manager(gpu, True, torch.float32, 64, 64, 16)
    ps = mgr.state.policy_states
    env = DummyVecEnv(64, 64, 6, seed=1, device=gpu)
    env.init()
    other = torch.zeros_like(env.obs)
    s = mgr.rollout_mgr.store
    with pytest.raises(RuntimeError, match="env->obs"):
        ps.rollout_step(other, s.obs[0], s.actions[0], s.log_probs[0], s.values[0],
                        (1, 2), mgr.rollout.counters[0:1], 0, env=env.native_step())
    assert nat.lib().mlearn_abi_version() == nat.ABI_VERSION
