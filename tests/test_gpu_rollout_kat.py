"""The integer known-answer design of the reference's tests/test_rollouts.py
(fake net `o + bias` 201-215, fake sim `obs = a + 1, reward = a + 2, done
every L` 264-288, closed-form checks of verify_rollout_data 380-460) run
through the HIP rollout path instead of the oracle (tests/test_rollout_kat.py
is the oracle's twin):

  * the post-step bookkeeping of env step t - 1 (store rewards / dones,
    env_returns = r + gamma env_returns traced and zeroed on done,
    rollouts.py:933-973) runs fused into the policy launch of step t and into
    the bootstrap critic launch after the last step, exactly as
    RolloutManager.collect issues it (mlearn_policy_rollout_step's `post`);
  * GAE (mlearn_gae_f32) with and without materialised returns, and the
    'Est Returns' / 'Rewards' metric kernel, on the resulting store.

The fake policy's integer actions drive the fake sim (they are what the
store's closed forms are about); the policy kernel the post-step rides on is
a random MLP whose own samples go to a scratch store."""

import numpy as np
import pytest
import torch

from oracle import ppo_ref as ref
from tests.test_gpu_policy import make_policy_state

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,L,N", [(32, 8, 64), (32, 5, 96), (12, 12, 32), (20, 32, 64)])
def test_rollout_integer_kat_hip_path(gpu, T, L, N):
    from madrona_learn import _native as nat
    from madrona_learn.algo_common import compute_advantages
    rng = np.random.default_rng(T * 100 + L)
    bias, gamma = 3, 0.5
    D = 16
    o0 = rng.integers(0, 1000, N).astype(np.float32)
    # the fake sim / fake policy, on device
    obs = torch.from_numpy(o0).to(gpu)
    counter = torch.zeros(N, dtype=torch.int64, device=gpu)
    st_rew = torch.full((T, N), -7.0, device=gpu)
    st_done = torch.full((T, N), 9, dtype=torch.uint8, device=gpu)
    env_ret = torch.zeros(N, device=gpu)
    trace = torch.zeros((T, N), device=gpu)
    values = torch.zeros((T, N), device=gpu)
    obs_hist = torch.zeros((T, N), device=gpu)
    # the policy kernel that carries the post-step (its samples: scratch)
    ps = make_policy_state(gpu, D, 64, 2, torch.float32, seed=1)
    sc_obs = torch.zeros((N, D), device=gpu)
    sc_act = torch.zeros((N, 6), dtype=torch.int32, device=gpu)
    sc_lp = torch.zeros((N, 6), device=gpu)
    sc_val = torch.zeros(N, device=gpu)
    step_ctr = torch.zeros(1, dtype=torch.int64, device=gpu)
    keep = []
    post = None
    for t in range(T):
        feat = torch.zeros((N, D), device=gpu)
        feat[:, 0] = obs / 1000.0
        ps.rollout_step(feat, sc_obs, sc_act, sc_lp, sc_val, (1, 2), step_ctr, t, 0,
                        sample=True, post=post)
        a = obs.to(torch.int32) + bias                      # FakeNet
        obs_hist[t] = obs
        values[t] = 2 * obs + 1                             # critic `+1`
        counter += 1                                        # fake_sim_step
        done = (counter == L).to(torch.uint8)
        counter %= L
        rew = (a + 2).to(torch.float32)
        obs = (a + 1).to(torch.float32)
        post = nat.PostStep()
        post.rewards, post.dones = nat.ptr(rew), nat.ptr(done)
        post.store_rewards, post.store_dones = nat.ptr(st_rew[t]), nat.ptr(st_done[t])
        post.env_returns, post.env_returns_trace = nat.ptr(env_ret), nat.ptr(trace[t])
        post.gamma = gamma
        keep.append((rew, done))
    boot_scratch = torch.zeros(N, device=gpu)
    feat = torch.zeros((N, D), device=gpu)
    ps.critic_only(feat, boot_scratch, post=post)           # the last step's post-step
    torch.cuda.synchronize()

    tt = np.arange(T)[:, None]
    o = o0[None, :] + tt * (bias + 1)
    assert np.array_equal(obs_hist.cpu().numpy(), o)
    assert np.array_equal(st_rew.cpu().numpy(), o + bias + 2)
    assert np.array_equal(st_done.cpu().numpy(),
                          np.broadcast_to(((tt + 1) % L == 0), (T, N)).astype(np.uint8))
    # env returns: r + gamma * running, traced, reset after each episode end
    want = np.zeros((T, N), np.float32)
    run = np.zeros(N, np.float32)
    r = (o + bias + 2).astype(np.float32)
    for i in range(T):
        run = (r[i] + np.float32(gamma) * run).astype(np.float32)
        want[i] = run
        if (i + 1) % L == 0:
            run = np.zeros(N, np.float32)
    assert np.array_equal(trace.cpu().numpy(), want)
    assert np.array_equal(env_ret.cpu().numpy(), run)

    # GAE on the store: gamma = lambda = 1 closed form, and the f32 restatement bit for bit
    boot = torch.from_numpy(2 * (o0 + T * (bias + 1)) + 1).to(gpu)

    class C:
        steps_per_update = T
        gamma = 1.0
        gae_lambda = 1.0

    adv, ret = compute_advantages(C, st_rew, values, st_done, boot)
    adv2, none = compute_advantages(C, st_rew, values, st_done, boot, out_ret=False)
    ea, er = ref.gae_f32(st_rew.cpu().numpy(), values.cpu().numpy(), st_done.cpu().numpy(),
                         boot.cpu().numpy(), 1.0, 1.0)
    assert np.array_equal(adv.cpu().numpy(), ea) and np.array_equal(ret.cpu().numpy(), er)
    assert none is None and np.array_equal(adv2.cpu().numpy(), ea)
    closed = np.zeros((T, N))
    for i in range(T):
        end = (i // L + 1) * L
        closed[i] = r[i:end].astype(np.float64).sum(0) if end <= T else \
            r[i:].astype(np.float64).sum(0) + boot.cpu().numpy()
    closed -= values.cpu().numpy()
    np.testing.assert_allclose(ea, closed, rtol=1e-6, atol=1e-3)

    # the rollout metrics kernel: 'Rewards' and 'Est Returns' (values + advantages, x2 form)
    jobs = (nat.MetricJob * 2)()
    jobs[0].x, jobs[0].n = nat.ptr(st_rew), T * N
    jobs[1].x, jobs[1].x2, jobs[1].n = nat.ptr(values), nat.ptr(adv2), T * N
    out = torch.zeros(10, device=gpu)
    ws = torch.zeros(int(nat.lib().mlearn_metrics_workspace_bytes(2)), dtype=torch.uint8,
                     device=gpu)
    nat.check(nat.lib().mlearn_metrics_f32(jobs, 2, nat.ptr(out), nat.ptr(ws),
                                           nat.stream_handle()))
    torch.cuda.synchronize()
    m = out.cpu().numpy()
    for j, x in enumerate((r, er)):
        x = x.astype(np.float64)
        np.testing.assert_allclose(m[5 * j], x.mean(), rtol=1e-6)
        np.testing.assert_allclose(m[5 * j + 2], x.min(), rtol=0)
        np.testing.assert_allclose(m[5 * j + 3], x.max(), rtol=0)
        assert m[5 * j + 4] == T * N
