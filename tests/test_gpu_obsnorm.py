"""GPU parity of ObservationsEMANormalizer (observations.py:70-132,
EMANormalizer moving_avg.py:48-196) on the fused path against the oracle
(oracle/ppo_ref.py ema_*): the in-kernel normalisation of the observations,
the per-step statistics written by the rollout launches, and their fold into
the estimates (rollouts.py:670-678, train.py:193-204).

Tolerances: estimates within 1e-5 relative (f32 reductions in a different
order than the two-pass numpy restatement); the normalised observations in
the store are bit-exact given the estimates the kernel used.
"""

import numpy as np
import pytest
import torch

from oracle import native as onat
from oracle import ppo_ref as ref
from tests.test_gpu_train import BUCKETS, make_cfg

pytestmark = pytest.mark.gpu

SCALE, SHIFT = 3.0, 1.5  # the wrapped env's observations: affine of N(0, 1)


class AffineEnv:
    """DummyVecEnv with observations SCALE * x + SHIFT (so the normaliser has
    something to learn)."""

    def __init__(self, env):
        self.env = env
        self.obs = torch.zeros_like(env.obs)

    def _wrap(self, out):
        torch.mul(out["obs"], SCALE, out=self.obs)
        self.obs.add_(SHIFT)
        return dict(out, obs=self.obs)

    def sim_fns(self):
        return {"init": lambda: self._wrap(self.env.init()),
                "step": lambda inp: self._wrap(self.env.step(inp))}


def _setup(gpu, dtype, decay, N=64, H=64, D=64):
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from tests.test_gpu_train import make_policy
    env = DummyVecEnv(N, D, 6, seed=4, device=gpu)
    cfg = make_cfg(dtype, N=N, H=H)
    pol = make_policy(dtype, H)
    pol = ml.Policy(actor_critic=pol.actor_critic,
                    obs_preprocess=ml.ObservationsEMANormalizer.create(decay, dtype))
    mgr = ml.init_training(gpu, cfg, AffineEnv(env).sim_fns(), pol, use_graph=False)
    return cfg, env, mgr


def _est_np(ps):
    e = ps.obs_est.cpu().numpy()
    return {"mu": e[0], "inv_sigma": e[1], "sigma": e[2], "mu_biased": e[3],
            "sigma_sq_biased": e[4], "N": int(ps.obs_count.item())}


@pytest.mark.parametrize("mode,dtype", [("f32", torch.float32), ("bf16", torch.bfloat16)])
def test_obs_normalizer_two_updates_match_oracle(gpu, mode, dtype):
    decay = 0.99
    cfg, env, mgr = _setup(gpu, dtype, decay)
    ps = mgr.state.policy_states
    lay = ref.param_layout(64, 64, 2, 26)
    oenv = onat.Env(env.N, env.D, env.k0, env.k1, 0)
    oenv.reset()
    oenv.obs = (oenv.obs * np.float32(SCALE) + np.float32(SHIFT)).astype(np.float32)
    est = ref.ema_init(64)
    for it in range(2):
        est_before = _est_np(ps)
        p0 = ps.params.cpu().numpy().astype(np.float64)
        mgr.update_iter()
        torch.cuda.synchronize()
        s = mgr.rollout_mgr.store
        # replay the GPU trajectory on the oracle env with the estimates the GPU used
        step = oenv.step

        def affine_step(a, _step=step):
            o, r, d = _step(a)
            o = (o * np.float32(SCALE) + np.float32(SHIFT)).astype(np.float32)
            oenv.obs = o
            return o, r, d
        oenv.step = affine_step
        ro, _ = ref.rollout(p0, lay, oenv, cfg.steps_per_update, BUCKETS, mgr.rollout.prng_key,
                            it * cfg.steps_per_update, mode=mode, gamma=cfg.gamma,
                            actions_override=s.actions.cpu().numpy(),
                            obs_norm=(est_before, decay, 1e-5))
        oenv.step = step
        # the kernel's normalisation, bit-exact given its estimates
        assert np.array_equal(s.obs.float().cpu().numpy(), ro["obs"]), f"update {it}"
        tol = 1e-4 if mode == "f32" else 3e-2
        np.testing.assert_allclose(s.values.cpu().numpy(), ro["values"], rtol=tol, atol=tol)
        # the statistics folded into the estimates
        got = _est_np(ps)
        exp = ro["obs_est"]
        assert got["N"] == exp["N"] == it + 1
        for k in ("mu", "mu_biased", "sigma_sq_biased", "inv_sigma", "sigma"):
            np.testing.assert_allclose(got[k], exp[k], rtol=1e-5, atol=1e-6, err_msg=k)
        est = exp
    # after one update with decay 0.99 the bias-corrected estimate is the rollout's
    # own mean / variance: mu ~ SHIFT, sigma ~ SCALE
    assert abs(float(np.mean(est["mu"])) - SHIFT) < 0.2
    assert abs(float(np.mean(est["sigma"])) - SCALE) < 0.3


def test_obs_stats_kernel_partial_tiles(gpu):
    """Rollout-step statistics with a partial last tile (N = 1000) folded by
    mlearn_obs_norm_update over 5 steps, against the two-pass restatement."""
    import madrona_learn as ml
    from madrona_learn import _native as nat
    from tests.test_gpu_policy import make_policy_state
    ps = make_policy_state(gpu, 32, 64, 2, torch.float32, seed=2)
    ps.obs_preprocess = ml.ObservationsEMANormalizer.create(0.95, torch.float32)
    D, N, T = 32, 1000, 5
    est = torch.zeros((5, D), dtype=torch.float32, device=gpu)
    est[1:3] = 1.0
    count = torch.zeros(1, dtype=torch.int32, device=gpu)
    tiles = (N + 31) // 32
    stats = torch.zeros((T, tiles, D, 2), dtype=torch.float32, device=gpu)
    ps.desc.obs_mu, ps.desc.obs_inv_sigma = est.data_ptr(), est.data_ptr() + 4 * D
    ps.desc.obs_stats, ps.desc.obs_stats_tiles, ps.desc.obs_stats_steps = stats.data_ptr(), tiles, T
    rng = np.random.default_rng(7)
    xs = [(rng.standard_normal((N, D)) * rng.uniform(0.5, 4, D) + rng.uniform(-3, 3, D))
          .astype(np.float32) for _ in range(T)]
    store = torch.zeros((N, D), dtype=torch.float32, device=gpu)
    acts = torch.zeros((N, 6), dtype=torch.int32, device=gpu)
    logp = torch.zeros((N, 6), dtype=torch.float32, device=gpu)
    vals = torch.zeros(N, dtype=torch.float32, device=gpu)
    ctr = torch.zeros(4, dtype=torch.int64, device=gpu)
    for t in range(T):
        ps.rollout_step(torch.from_numpy(xs[t]).to(gpu), store, acts, logp, vals, (1, 2),
                        ctr[0:1], t)
    nat.check(nat.lib().mlearn_obs_norm_update(nat.ptr(stats), T, tiles, N, D, 0.95, 1e-5,
                                               nat.ptr(est), nat.ptr(count),
                                               nat.stream_handle()))
    torch.cuda.synchronize()
    # the kernel normalised with the initial estimates (identity)
    assert torch.equal(store.cpu(), torch.from_numpy(xs[-1]))
    o = ref.ema_init(D)
    st = (np.zeros(D, np.float32), np.zeros(D, np.float32))
    for t in range(T):
        st = ref.ema_update_input_stats(st, t, xs[t])
    exp = ref.ema_update_estimates(o, st, 0.95, 1e-5)
    e = est.cpu().numpy()
    for i, k in enumerate(("mu", "inv_sigma", "sigma", "mu_biased", "sigma_sq_biased")):
        np.testing.assert_allclose(e[i], exp[k], rtol=2e-5, atol=1e-6, err_msg=k)
    assert int(count.item()) == 1


def test_obs_normalizer_before_prefix_on_torch_path(gpu):
    """ObservationsEMANormalizer with a BackboneShared prefix: the reference
    normalises the raw observations and runs the prefix on the result
    (rollouts.py:838-840, actor_critic.py:226-229).  The fused rollout kernel
    normalises what it multiplies (the prefix's output), so init_training
    routes this policy to the torch path, which keeps the reference's order.
    Two updates against the oracle: the stored observations are the
    normalised RAW observations (bit-exact given the estimates), the
    estimates follow ppo_ref.ema_* (1e-5 relative; the observations normalised
    with updated estimates then agree to 1e-5 as well), and the stored values
    are the critic of prefix(normalised observations) (oracle forward)."""
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
    from tests.test_gpu_generic import _shared_mlp_flat
    decay, N, H, T = 0.99, 64, 64, 32
    dt = torch.float32
    env = DummyVecEnv(N, 64, 6, seed=14, device=gpu)
    halve = lambda x, train=False: x * 0.5  # noqa: E731
    ac = ml.ActorCritic(
        backbone=ml.BackboneShared(prefix=halve, encoder=ml.BackboneEncoder(net=MLP(H, 2, dt))),
        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dt),
        critic=DenseLayerCritic(dt))
    pol = ml.Policy(actor_critic=ac, obs_preprocess=ml.ObservationsEMANormalizer.create(decay, dt))
    cfg = make_cfg(dt, N=N, H=H)
    mgr = ml.init_training(gpu, cfg, AffineEnv(env).sim_fns(), pol, use_graph=False)
    ps = mgr.state.policy_states
    assert getattr(ps, "generic", False)
    oenv = onat.Env(env.N, env.D, env.k0, env.k1, 0)
    oenv.reset()
    oenv.obs = (oenv.obs * np.float32(SCALE) + np.float32(SHIFT)).astype(np.float32)
    est = ref.ema_init(64)
    for it in range(2):
        p0, lay = _shared_mlp_flat(ps, 64, H, 2)
        mgr.update_iter()
        torch.cuda.synchronize()
        s = mgr.rollout_mgr.store
        step = oenv.step

        def affine_step(a, _step=step):
            o, r, d = _step(a)
            o = (o * np.float32(SCALE) + np.float32(SHIFT)).astype(np.float32)
            oenv.obs = o
            return o, r, d
        oenv.step = affine_step
        ro, _ = ref.rollout(p0, lay, oenv, T, BUCKETS, mgr.rollout.prng_key, it * T, mode="f32",
                            gamma=cfg.gamma, actions_override=s.actions.cpu().numpy(),
                            obs_norm=(est, decay, 1e-5))
        oenv.step = step
        # bit-exact with the initial estimates; afterwards the torch path's
        # estimate update (moving_avg.py in torch) differs from the oracle's by
        # f32 rounding (checked at 1e-5 below), which the normalised
        # observations inherit
        if it == 0:
            assert np.array_equal(s.obs.float().cpu().numpy(), ro["obs"]), f"update {it}"
        else:
            np.testing.assert_allclose(s.obs.float().cpu().numpy(), ro["obs"], rtol=1e-5,
                                       atol=1e-5, err_msg=f"update {it}")
        _, V, _ = ref.forward(ref.unflatten(p0, lay), ro["obs"].reshape(T * N, 64) * 0.5, "f32")
        np.testing.assert_allclose(s.values.cpu().numpy().reshape(-1), V, rtol=1e-4, atol=1e-4)
        est = ro["obs_est"]
        got = ps.obs_pre_state
        for k in ("mu", "sigma"):
            np.testing.assert_allclose(got[k].cpu().numpy(), est[k], rtol=1e-5, atol=1e-6)


def test_bare_obs_normalizer_state_survives_checkpoint(gpu, tmp_path):
    """A bare (unnamed) observation tensor under ObservationsEMANormalizer on
    the torch path keeps its normaliser state _Bare-marked; a checkpoint
    stores plain dicts, so the restore must re-mark it: after
    save -> load into a fresh manager the state is the same estimates, still
    read as the bare observation's, and training continues from it (the
    estimates move on from the restored ones)."""
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
    from madrona_learn.observations import _Bare
    decay, N, H = 0.99, 64, 64
    dt = torch.float32

    def build():
        env = DummyVecEnv(N, 64, 6, seed=21, device=gpu)
        halve = lambda x, train=False: x * 0.5  # noqa: E731  (routes to the torch path)
        ac = ml.ActorCritic(
            backbone=ml.BackboneShared(prefix=halve,
                                       encoder=ml.BackboneEncoder(net=MLP(H, 2, dt))),
            actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dt),
            critic=DenseLayerCritic(dt))
        pol = ml.Policy(actor_critic=ac,
                        obs_preprocess=ml.ObservationsEMANormalizer.create(decay, dt))
        return ml.init_training(gpu, make_cfg(dt, N=N, H=H), AffineEnv(env).sim_fns(), pol,
                                use_graph=False)

    a = build()
    assert getattr(a.state.policy_states, "generic", False)
    a.update_iter()
    torch.cuda.synchronize()
    a.save_ckpt(str(tmp_path))
    b = build()
    b.load_ckpt(str(tmp_path))
    sa, sb = a.state.policy_states.obs_pre_state, b.state.policy_states.obs_pre_state
    assert isinstance(sa, _Bare) and isinstance(sb, _Bare)
    assert set(sa) == set(sb)
    for k in sa:
        assert torch.equal(sa[k].cpu(), sb[k].cpu()), k
    loaded = {k: v.clone() for k, v in sb.items()}
    b.update_iter()  # (a crash here was the ADVICE r05 failure: the state read as named obs)
    torch.cuda.synchronize()
    sb = b.state.policy_states.obs_pre_state
    assert isinstance(sb, _Bare) and set(sb) == set(loaded)
    for k in sb:
        assert torch.isfinite(sb[k]).all(), k
    assert not torch.equal(sb["mu"], loaded["mu"])  # the estimates moved on from the restore
