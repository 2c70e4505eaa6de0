"""GPU parity of the value normaliser (TrainConfig.normalize_values,
ppo.py:190-211, rollouts.py:726-738, moving_avg.py:48-196) through the C ABI:
GAE over inverted values is bit-exact with the oracle's f32 recurrence on the
inverted values; one full PPO iteration (f32, scalar critic) matches the
oracle's update with the estimates chained minibatch by minibatch, and the
estimates after the update match within 1e-5."""

import dataclasses

import numpy as np
import pytest
import torch

from oracle import native as onat
from oracle import ppo_ref as ref
from tests.test_gpu_train import BUCKETS, make_cfg, make_policy

pytestmark = pytest.mark.gpu


def test_gae_inverts_normalised_values(gpu):
    from madrona_learn import _native as nat
    rng = np.random.default_rng(3)
    T, P, B = 32, 2, 96
    N = P * B
    r = rng.standard_normal((T, N)).astype(np.float32)
    v = rng.standard_normal((T, N)).astype(np.float32)
    d = (rng.random((T, N)) < 0.1).astype(np.uint8)
    b = rng.standard_normal(N).astype(np.float32)
    est = np.zeros((P, 8), np.float32)
    est[:, 0] = [0.7, -1.3]
    est[:, 2] = [2.5, 0.4]
    est[:, 1] = 1 / est[:, 2]
    # device copies kept alive across the launch
    tr, tv, td, tb, te = (torch.from_numpy(x).to(gpu) for x in (r, v, d, b, est))
    adv = torch.empty((T, N), dtype=torch.float32, device=gpu)
    ret = torch.empty_like(adv)
    nat.check(nat.lib().mlearn_gae_vnorm_f32(
        nat.ptr(tr), nat.ptr(tv), nat.ptr(td), nat.ptr(tb), nat.ptr(te), B,
        nat.ptr(adv), nat.ptr(ret), T, N, 0.99, 0.99 * 0.95, nat.stream_handle()), "gae_vnorm")
    torch.cuda.synchronize()
    cols = np.repeat(np.arange(P), B)
    vi = np.empty_like(v)
    bi = np.empty_like(b)
    for p in range(P):
        e = {"mu": est[p, 0:1], "sigma": est[p, 2:3]}
        vi[:, cols == p] = ref.ema_invert(e, v[:, cols == p])
        bi[cols == p] = ref.ema_invert(e, b[cols == p])
    a_ref, r_ref = ref.gae_f32(r, vi, d, bi, 0.99, 0.95)
    assert np.array_equal(adv.cpu().numpy(), a_ref)
    assert np.array_equal(ret.cpu().numpy(), r_ref)


def test_full_update_with_value_norm_matches_oracle(gpu):
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    dtype = torch.float32
    env = DummyVecEnv(64, 64, 6, seed=2, device=gpu)
    cfg = dataclasses.replace(make_cfg(dtype), normalize_values=True,
                              value_normalizer_decay=0.99)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), make_policy(dtype, 64), use_graph=False)
    ps, ts = mgr.state.policy_states, mgr.state.train_states
    p0 = ps.params.cpu().numpy().astype(np.float64)
    mgr.update_iter()
    torch.cuda.synchronize()
    s = mgr.rollout_mgr.store
    # the initial estimates (mu 0, sigma 1) invert to the stored values exactly
    adv, ret = ref.gae_f32(s.rewards.cpu().numpy(), s.values.cpu().numpy(),
                           s.dones.cpu().numpy(), s.bootstrap.cpu().numpy(), cfg.gamma,
                           cfg.gae_lambda)
    assert np.array_equal(s.advantages.cpu().numpy(), adv)
    store = {k: v.cpu().numpy() for k, v in s.as_dict().items()}
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
          "normalize_advantages": True}
    zeros = np.zeros_like(p0)
    est = ref.ema_init(1)
    p1, _, met = ref.ppo_update(
        p0, (zeros, zeros.copy(), 0), [store], hp, BUCKETS, ref.param_layout(64, 64, 2, 26),
        ps.init_norms.cpu().numpy().astype(np.float64), num_epochs=2, minibatch_size=16,
        bptt=cfg.steps_per_update, key=ts.update_prng_key, epoch_base=0, mode="f32",
        lr=3e-4, max_grad_norm=0.5, value_norm=est, value_norm_decay=0.99)
    assert est["N"] == 2 * (64 // 16)
    got = ps.params.cpu().numpy()
    np.testing.assert_allclose(got, p1, rtol=1e-4, atol=2e-5)
    vn = ts.value_norm_est.cpu().numpy()
    np.testing.assert_allclose(vn[0], est["mu"][0], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(vn[2], est["sigma"][0], rtol=1e-5)
    assert int(ts.value_norm_count.item()) == est["N"]
    # the last minibatch's value errors use the inverted critic
    last = mgr.metrics.last()
    np.testing.assert_allclose(last["Value Errors"].mean, np.mean(met["Value Errors"]),
                               rtol=1e-4)
