"""Training a policy tree the fused kernels do not implement (the torch path
of init_training, madrona_learn/generic.py): the reference trains whatever
module the Policy holds (ppo.py:119-127, 276-281).

* BackboneSeparate (actor_critic.py:247-303: separate MLP encoders for the
  actor and the critic), f32: the rollout store against the oracle env and
  the oracle forward, GAE bit-exact, and one full PPO update (2 epochs x 4
  minibatches) against oracle/separate_ref.py from the same store and
  parameters (the tolerances of tests/test_gpu_train.py's f32 update).
* A user ObservationsPreprocess subclass (observations.py:13-68 plugin
  interface, _preprocess overridden) on a BackboneShared MLP: trained on
  the torch path, the store holds the preprocessed observations.
* action_stats' autograd form (HIP forward, softmax backward) against
  torch's own log_softmax / entropy gradients.
"""

import numpy as np
import pytest
import torch

from oracle import native as onat
from oracle import ppo_ref as ref
from oracle import separate_ref as sref

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]


def _cfg(N, mb, epochs=2, dtype=torch.float32):
    import madrona_learn as ml
    return ml.TrainConfig(
        num_worlds=N, num_agents_per_world=1, num_updates=1,
        actions={"actions": ml.DiscreteActionsConfig(BUCKETS)}, steps_per_update=32, lr=3e-4,
        algo=ml.PPOConfig(num_epochs=epochs, minibatch_size=mb, clip_coef=0.2,
                          value_loss_coef=0.5, entropy_coef={"actions": 0.01},
                          max_grad_norm=0.5),
        num_bptt_chunks=1, gamma=0.99, gae_lambda=0.95, seed=3, metrics_buffer_size=4,
        dreamer_v3_critic=False, compute_dtype=dtype)


def _named(ps):
    return {n: ps.params[o:o + int(np.prod(s))].cpu().numpy().astype(np.float64).reshape(s)
            for n, o, s in ps.layout["params"]}


def test_backbone_separate_update_matches_oracle(gpu):
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
    N, H, L, mb, T = 64, 64, 2, 16, 32
    dt = torch.float32
    env = DummyVecEnv(N, 64, 6, seed=2, device=gpu)
    ac = ml.ActorCritic(
        backbone=ml.BackboneSeparate(actor_encoder=ml.BackboneEncoder(net=MLP(H, L, dt)),
                                     critic_encoder=ml.BackboneEncoder(net=MLP(H, L, dt))),
        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dt),
        critic=DenseLayerCritic(dt))
    cfg = _cfg(N, mb)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), ml.Policy(actor_critic=ac), use_graph=True)
    ps, ts = mgr.state.policy_states, mgr.state.train_states
    # (the torch path captures its updates in HIP graphs from update 2 on)
    assert getattr(ps, "generic", False) and mgr.use_graph and mgr._torch_path
    order = [n for n, _, _ in ps.layout["params"]]
    p0 = _named(ps)
    init_norms = {k: float(np.sqrt((v * v).sum())) for k, v in p0.items() if k.endswith("kernel")
                  and k.startswith("backbone.")}
    assert len(init_norms) == 2 * L and ts.num_groups == 4 * L
    oenv = onat.Env(N, 64, env.k0, env.k1, 0)
    oenv.reset()
    mgr.update_iter()
    torch.cuda.synchronize()
    s = mgr.rollout_mgr.store
    acts = s.actions.cpu().numpy()
    obs = s.obs.float().cpu().numpy()
    for t in range(T):
        assert np.array_equal(obs[t], oenv.obs), t
        o, r, d = oenv.step(acts[t])
        assert np.array_equal(s.rewards[t].cpu().numpy(), r)
        assert np.array_equal(s.dones[t].cpu().numpy(), d)
    logits, V, _ = sref.forward(p0, obs.reshape(T * N, 64), L, "f32")
    lp, _ = ref.action_stats(logits, BUCKETS, acts.reshape(T * N, 6))
    np.testing.assert_allclose(s.values.cpu().numpy().reshape(-1), V, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(s.log_probs.cpu().numpy().reshape(-1, 6), lp, rtol=1e-4,
                               atol=1e-4)
    adv, _ = ref.gae_f32(s.rewards.cpu().numpy(), s.values.cpu().numpy(), s.dones.cpu().numpy(),
                         s.bootstrap.cpu().numpy(), cfg.gamma, cfg.gae_lambda)
    assert np.array_equal(s.advantages.cpu().numpy(), adv)
    store = {k: v.float().cpu().numpy() if v.dtype == torch.bfloat16 else v.cpu().numpy()
             for k, v in s.as_dict().items()}
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
          "normalize_advantages": True}
    want, _ = sref.ppo_update(dict(p0), order, store, hp, BUCKETS, L, init_norms, num_epochs=2,
                              minibatch_size=mb, bptt=T, key=ts.update_prng_key, epoch_base=0,
                              mode="f32", lr=3e-4, max_grad_norm=0.5)
    got = _named(ps)
    g = np.concatenate([got[k].reshape(-1) for k in order])
    w = np.concatenate([want[k].reshape(-1) for k in order])
    z = np.concatenate([p0[k].reshape(-1) for k in order])
    # as tests/test_gpu_train.py f32: Adam takes noise-sized steps where the
    # gradient is at the f32 summation-noise level, in both implementations
    np.testing.assert_allclose(g, w, rtol=0, atol=1e-4)
    close = np.abs(g - w) <= 2e-5 + 1e-4 * np.abs(w)
    assert close.mean() >= 0.999, close.mean()
    dg, dw = g - z, w - z
    assert dg @ dw / (np.linalg.norm(dg) * np.linalg.norm(dw)) > 0.999
    assert int(ts.step.item()) == 2 * (N // mb)
    # the projections held: every trunk kernel at its initial norm
    for k, n0 in init_norms.items():
        np.testing.assert_allclose(np.sqrt((got[k] ** 2).sum()), n0, rtol=1e-5)
    last = mgr.metrics.last()
    assert np.isfinite(last["Loss"].mean)


def test_user_preprocess_trains_on_torch_path(gpu):
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from madrona_learn.observations import ObservationsPreprocess
    from tests.test_gpu_train import make_policy

    class Halve(ObservationsPreprocess):
        def _preprocess(self, ob_name, state, ob):
            return ob * 0.5

    N = 64
    env = DummyVecEnv(N, 64, 6, seed=4, device=gpu)
    pol = make_policy(torch.float32, 64)
    pol = ml.Policy(actor_critic=pol.actor_critic, obs_preprocess=Halve())
    mgr = ml.init_training(gpu, _cfg(N, 16, epochs=1), env.sim_fns(), pol)
    ps = mgr.state.policy_states
    assert getattr(ps, "generic", False)
    oenv = onat.Env(N, 64, env.k0, env.k1, 0)
    oenv.reset()
    p0 = ps.params.clone()
    mgr.update_iter()
    torch.cuda.synchronize()
    s = mgr.rollout_mgr.store
    np.testing.assert_array_equal(s.obs[0].cpu().numpy(), oenv.obs * np.float32(0.5))
    assert torch.isfinite(ps.params).all() and not torch.equal(ps.params, p0)


def test_action_stats_autograd_matches_torch(gpu):
    from madrona_learn.dists import DiscreteActionDistributions
    torch.manual_seed(0)
    lg = torch.randn((300, sum(BUCKETS)), device=gpu, dtype=torch.float32) * 3
    acts = torch.stack([torch.randint(0, b, (300,), device=gpu) for b in BUCKETS], -1)
    wl = torch.randn((300, 6), device=gpu)
    we = torch.randn((300, 6), device=gpu)
    x = lg.clone().requires_grad_(True)
    logp, ent = DiscreteActionDistributions(BUCKETS, x).action_stats(acts)
    ((logp * wl).sum() + (ent * we).sum()).backward()
    y = lg.clone().requires_grad_(True)
    lps, ents, off = [], [], 0
    for k, b in enumerate(BUCKETS):
        ls = torch.log_softmax(y[:, off:off + b], -1)
        lps.append(ls.gather(1, acts[:, k:k + 1]).squeeze(1))
        ents.append(-(ls.exp() * ls).sum(-1))
        off += b
    lp2, ent2 = torch.stack(lps, -1), torch.stack(ents, -1)
    ((lp2 * wl).sum() + (ent2 * we).sum()).backward()
    torch.testing.assert_close(logp, lp2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ent, ent2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad, y.grad, rtol=1e-4, atol=1e-5)


def test_fp16_trains_with_dynamic_scale(gpu):
    """compute_dtype fp16 (train_state.py:402-403, ppo.py:276-291): the
    fused kernels are bf16 / f32, so the tree trains on the torch path with
    DynamicScale.  A finite update moves the parameters and counts
    fin_steps; a forced overflow (scale 2^126: the fp16 backward overflows)
    leaves params (up to the projections), Adam moments and step unchanged
    and halves the scale, as flax's where_finite + backoff."""
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from tests.test_gpu_train import make_policy
    N, mb = 64, 16
    env = DummyVecEnv(N, 64, 6, seed=5, device=gpu)
    cfg = _cfg(N, mb, epochs=1, dtype=torch.float16)
    assert "fp16" in repr(cfg)
    pol = make_policy(torch.float16, 64)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), pol)
    ps, ts = mgr.state.policy_states, mgr.state.train_states
    assert getattr(ps, "generic", False) and ts.scaler is not None
    assert mgr.rollout_mgr.store.obs.dtype == torch.float16
    p0 = ps.params.clone()
    mgr.update_iter()
    torch.cuda.synchronize()
    nmb = N // mb
    assert torch.isfinite(ps.params).all() and not torch.equal(ps.params, p0)
    assert int(ts.step.item()) == nmb
    assert float(ts.scaler.scale.item()) == 65536.0 and int(ts.scaler.fin_steps.item()) == nmb
    # overflow every minibatch of the next update
    ts.scaler.scale.fill_(2.0 ** 126)
    p1, m1, v1 = ps.params.clone(), ts.adam_m.clone(), ts.adam_v.clone()
    mgr.update_iter()
    torch.cuda.synchronize()
    assert int(ts.step.item()) == nmb
    assert torch.equal(ts.adam_m, m1) and torch.equal(ts.adam_v, v1)
    torch.testing.assert_close(ps.params, p1, rtol=2e-6, atol=1e-7)  # re-projection only
    assert float(ts.scaler.scale.item()) == 2.0 ** (126 - nmb)
    assert int(ts.scaler.fin_steps.item()) == 0


def test_mlp_width_outside_kernels_trains(gpu):
    """models.py:99-119's MLP takes any width and depth; the kernels are
    instantiated for 64 / 128 / 256 x 1..4, so a 96-wide 5-layer trunk trains
    on the torch path: rollout store against the oracle env, GAE bit-exact,
    parameters moved and finite."""
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from tests.test_gpu_train import make_policy
    N, T = 64, 32
    env = DummyVecEnv(N, 64, 6, seed=6, device=gpu)
    cfg = _cfg(N, 16, epochs=1)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), make_policy(torch.float32, 96, L=5))
    ps = mgr.state.policy_states
    assert getattr(ps, "generic", False)
    oenv = onat.Env(N, 64, env.k0, env.k1, 0)
    oenv.reset()
    p0 = ps.params.clone()
    mgr.update_iter()
    torch.cuda.synchronize()
    s = mgr.rollout_mgr.store
    acts = s.actions.cpu().numpy()
    for t in range(T):
        assert np.array_equal(s.obs[t].float().cpu().numpy(), oenv.obs), t
        o, r, d = oenv.step(acts[t])
        assert np.array_equal(s.rewards[t].cpu().numpy(), r)
    adv, _ = ref.gae_f32(s.rewards.cpu().numpy(), s.values.cpu().numpy(), s.dones.cpu().numpy(),
                         s.bootstrap.cpu().numpy(), cfg.gamma, cfg.gae_lambda)
    assert np.array_equal(s.advantages.cpu().numpy(), adv)
    assert torch.isfinite(ps.params).all() and not torch.equal(ps.params, p0)


def test_multilayer_lstm_trains_on_torch_path(gpu):
    """rnn.LSTM with num_layers = 2 (MultiLayerLSTMCell, rnn.py:10-45; the
    fused kernels take one layer) trains on the torch path: the rollout
    carries rollout_state.rnn_states, clears it where an episode ended
    (rollouts.py:941-942) and saves the carry entering every BPTT chunk
    (rnn_start_states, rollouts.py:528-537); the update runs LSTM.sequence from
    those start states.  Self-consistency (parity unpinned: the oracle's LSTM
    is one layer): replaying LSTM.sequence over each chunk's stored
    observations from its stored start state with the rollout-time parameters
    reproduces the stored log-probs and values."""
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
    from madrona_learn.rnn import LSTM
    N, T, C = 32, 32, 2
    dt = torch.float32
    env = DummyVecEnv(N, 64, 6, seed=8, device=gpu)
    ac = ml.ActorCritic(
        backbone=ml.BackboneShared(encoder=ml.RecurrentBackboneEncoder(
            net=MLP(64, 1, dt), rnn=LSTM(64, 2, dt))),
        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dt),
        critic=DenseLayerCritic(dt))
    cfg = ml.TrainConfig(
        num_worlds=N, num_agents_per_world=1, num_updates=2,
        actions={"actions": ml.DiscreteActionsConfig(BUCKETS)}, steps_per_update=T, lr=3e-4,
        algo=ml.PPOConfig(num_epochs=1, minibatch_size=16, clip_coef=0.2, value_loss_coef=0.5,
                          entropy_coef={"actions": 0.01}, max_grad_norm=0.5),
        num_bptt_chunks=C, gamma=0.99, gae_lambda=0.95, seed=9, metrics_buffer_size=4,
        dreamer_v3_critic=False, compute_dtype=dt)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), ml.Policy(actor_critic=ac))
    ps = mgr.state.policy_states
    assert getattr(ps, "generic", False) and ps.recurrent
    cell0 = ac.backbone.encoder.rnn.cell
    wi0 = [w.detach().clone() for w in cell0.wi]
    wh0 = [w.detach().clone() for w in cell0.wh]
    assert mgr.state.train_states.num_groups == 2 * 8 + 2  # 8 gate kernels per layer + W0, LN0
    for it in range(2):
        p_roll = ps.params.clone()
        mgr.update_iter()
        torch.cuda.synchronize()
        s = mgr.rollout_mgr.store
        if it == 0:  # the first chunk starts from the zero carry
            for x in s.torch_start[0] + s.torch_start[1]:
                assert not torch.any(x[0])
        assert torch.isfinite(ps.params).all() and not torch.equal(ps.params, p_roll)
        dones = s.dones
        assert int(dones.sum()) > 0  # episodes end inside the rollout (carry clears exercised)
        p_now = ps.params.clone()
        ps.params.copy_(p_roll)
        bp = T // C
        with torch.no_grad():
            for c in range(C):
                start = ([x[c] for x in s.torch_start[0]], [x[c] for x in s.torch_start[1]])
                obs = s.obs[c * bp:(c + 1) * bp].float()
                fa, fc = ac.backbone.sequence(start, dones[c * bp:(c + 1) * bp, :, None], obs)
                dists = ac.actor(fa)
                lp, _ = dists.action_stats(s.actions[c * bp:(c + 1) * bp].reshape(bp * N, -1))
                v = ac.critic(fc).reshape(bp, N)
                torch.testing.assert_close(lp.reshape(bp, N, -1),
                                           s.log_probs[c * bp:(c + 1) * bp], rtol=1e-4, atol=1e-5)
                torch.testing.assert_close(v, s.values[c * bp:(c + 1) * bp], rtol=1e-4, atol=1e-5)
        ps.params.copy_(p_now)
        # every gate kernel of every layer stayed at its initial norm (flax's
        # separate per-gate Dense leaves, each projected, ppo.py:303-310)
        cell = ac.backbone.encoder.rnn.cell
        for l in range(2):
            for w, w0 in ((cell.wi[l], wi0[l]), (cell.wh[l], wh0[l])):
                for g in range(4):
                    blk = w.detach()[:, g * 64:(g + 1) * 64]
                    torch.testing.assert_close(torch.linalg.vector_norm(blk),
                                               torch.linalg.vector_norm(w0[:, g * 64:(g + 1) * 64]),
                                               rtol=1e-5, atol=0)


def _shared_mlp_flat(ps, D, H, L):
    """The torch arena of a BackboneShared(BackboneEncoder(MLP)) tree with
    DenseLayerDiscreteActor / DenseLayerCritic as oracle/ppo_ref's flat
    layout (trunk W / LayerNorm per layer, head W = [actor | critic] columns)."""
    named = _named(ps)
    pre = "backbone.encoder.net"
    lay = ref.param_layout(D, H, L, sum(BUCKETS))
    P = {"W": [named[f"{pre}.dense.{l}.kernel"] for l in range(L)],
         "s": [named[f"{pre}.norms.{l}.scale"] for l in range(L)],
         "b": [named[f"{pre}.norms.{l}.bias"] for l in range(L)],
         "Wh": np.concatenate([named["actor.impl.kernel"], named["critic.impl.kernel"]], 1),
         "bh": np.concatenate([named["actor.impl.bias"], named["critic.impl.bias"]])}
    return ref.flatten(P, lay), lay


def test_fp16_update_matches_oracle(gpu):
    """compute_dtype fp16 (train_state.py:402-403) on the torch path, one
    update of 2 epochs x 4 minibatches under DynamicScale (ppo.py:276-291),
    against the oracle's fp16 mode (oracle/ppo_ref.py rnd 'fp16': the fp16
    significand at every compute-dtype rounding point) under the per-tensor
    bound of tests/bf16_bound.py: the GPU's distance to the fp16 oracle
    within the oracle's own fp16-vs-f32 distance per tensor.  Rollout: the
    stored fp16 observations bit-exact, values / log-probs within fp16
    tolerance of the oracle forward."""
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from tests.bf16_bound import check_bf16_update
    from tests.test_gpu_train import make_policy
    N, H, L, mb, T = 64, 64, 2, 16, 32
    env = DummyVecEnv(N, 64, 6, seed=12, device=gpu)
    cfg = _cfg(N, mb, epochs=2, dtype=torch.float16)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), make_policy(torch.float16, H))
    ps, ts = mgr.state.policy_states, mgr.state.train_states
    assert getattr(ps, "generic", False) and ts.scaler is not None
    p0, lay = _shared_mlp_flat(ps, 64, H, L)
    oenv = onat.Env(N, 64, env.k0, env.k1, 0)
    oenv.reset()
    mgr.update_iter()
    torch.cuda.synchronize()
    assert int(ts.scaler.fin_steps.item()) == 2 * (N // mb)  # no skipped step
    s = mgr.rollout_mgr.store
    acts = s.actions.cpu().numpy()
    obs = s.obs.float().cpu().numpy()
    for t in range(T):
        assert np.array_equal(obs[t], oenv.obs.astype(np.float16).astype(np.float32)), t
        oenv.step(acts[t])
    logits, V, _ = ref.forward(ref.unflatten(p0, lay), obs.reshape(T * N, 64), "fp16")
    lp, _ = ref.action_stats(logits, BUCKETS, acts.reshape(T * N, 6))
    np.testing.assert_allclose(s.values.cpu().numpy().reshape(-1), V, rtol=1e-2, atol=1e-2)
    np.testing.assert_allclose(s.log_probs.cpu().numpy().reshape(-1, 6), lp, rtol=1e-2,
                               atol=1e-2)
    store = {k: v.float().cpu().numpy() if v.dtype != torch.uint8 and v.is_floating_point()
             else v.cpu().numpy() for k, v in s.as_dict().items()}
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
          "normalize_advantages": True}
    norms = np.array([np.sqrt((w ** 2).sum()) for w in ref.unflatten(p0, lay)["W"]])
    z = np.zeros_like(p0)
    upd = dict(num_epochs=2, minibatch_size=mb, bptt=T, key=ts.update_prng_key, epoch_base=0,
               lr=3e-4, max_grad_norm=0.5)
    ph, _, _ = ref.ppo_update(p0, (z, z.copy(), 0), [store], hp, BUCKETS, lay, norms,
                              mode="fp16", **upd)
    pf, _, _ = ref.ppo_update(p0, (z, z.copy(), 0), [store], hp, BUCKETS, lay, norms,
                              mode="f32", **upd)
    got, _ = _shared_mlp_flat(ps, 64, H, L)
    check_bf16_update("torch_fp16_update", got, p0, ph, pf, lay)


def test_value_norm_on_torch_path_matches_oracle(gpu):
    """normalize_values (ppo.py:190-211) with a tree outside the fused
    kernels (BackboneSeparate, f32): the GAE inverts the stored values, the
    per-minibatch return statistics move the estimates minibatch by
    minibatch (mlearn_return_stats / mlearn_value_norm_chain, as the fused
    path), the value loss targets the normalised returns; one update against
    oracle/separate_ref.py with the value normaliser (ppo_ref's rule)."""
    import dataclasses
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
    N, H, L, mb, T = 64, 64, 2, 16, 32
    dt = torch.float32
    env = DummyVecEnv(N, 64, 6, seed=13, device=gpu)
    ac = ml.ActorCritic(
        backbone=ml.BackboneSeparate(actor_encoder=ml.BackboneEncoder(net=MLP(H, L, dt)),
                                     critic_encoder=ml.BackboneEncoder(net=MLP(H, L, dt))),
        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dt),
        critic=DenseLayerCritic(dt))
    cfg = dataclasses.replace(_cfg(N, mb), normalize_values=True, value_normalizer_decay=0.99)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), ml.Policy(actor_critic=ac))
    ps, ts = mgr.state.policy_states, mgr.state.train_states
    assert getattr(ps, "generic", False) and ts.value_norm_est is not None
    order = [n for n, _, _ in ps.layout["params"]]
    p0 = _named(ps)
    init_norms = {k: float(np.sqrt((v * v).sum())) for k, v in p0.items() if k.endswith("kernel")
                  and k.startswith("backbone.")}
    mgr.update_iter()
    torch.cuda.synchronize()
    s = mgr.rollout_mgr.store
    # the initial estimates (mu 0, sigma 1) invert to the stored values exactly
    adv, _ = ref.gae_f32(s.rewards.cpu().numpy(), s.values.cpu().numpy(), s.dones.cpu().numpy(),
                         s.bootstrap.cpu().numpy(), cfg.gamma, cfg.gae_lambda)
    assert np.array_equal(s.advantages.cpu().numpy(), adv)
    store = {k: v.cpu().numpy() for k, v in s.as_dict().items()}
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
          "normalize_advantages": True}
    est = ref.ema_init(1)
    want, met = sref.ppo_update(dict(p0), order, store, hp, BUCKETS, L, init_norms, num_epochs=2,
                                minibatch_size=mb, bptt=T, key=ts.update_prng_key, epoch_base=0,
                                mode="f32", lr=3e-4, max_grad_norm=0.5, value_norm=est,
                                value_norm_decay=0.99)
    assert est["N"] == 2 * (N // mb)
    vn = ts.value_norm_est.cpu().numpy()
    np.testing.assert_allclose(vn[0], est["mu"][0], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(vn[2], est["sigma"][0], rtol=1e-5)
    assert int(ts.value_norm_count.item()) == est["N"]
    got = _named(ps)
    g = np.concatenate([got[k].reshape(-1) for k in order])
    w = np.concatenate([want[k].reshape(-1) for k in order])
    np.testing.assert_allclose(g, w, rtol=0, atol=1e-4)
    close = np.abs(g - w) <= 2e-5 + 1e-4 * np.abs(w)
    assert close.mean() >= 0.999, close.mean()
    # the last minibatch's value errors use the critic inverted with the
    # estimates before that minibatch
    last = mgr.metrics.last()
    np.testing.assert_allclose(last["Value Errors"].mean, np.mean(met["Value Errors"]), rtol=1e-4)


def test_wide_head_routes_to_torch_path(gpu):
    """A head wider than the fused kernels' 96 columns (DreamerV3Critic with
    255 bins, the dreamerv3 default the reference's models.py mentions) is a
    valid tree: init_training trains it on the torch path instead of failing
    (_native.head_cols raises NotImplementedError)."""
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from madrona_learn.models import MLP, DenseLayerDiscreteActor, DreamerV3Critic
    N, H = 64, 64
    dt = torch.float32
    env = DummyVecEnv(N, 64, 6, seed=5, device=gpu)
    ac = ml.ActorCritic(
        backbone=ml.BackboneShared(encoder=ml.BackboneEncoder(net=MLP(H, 2, dt))),
        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dt),
        critic=DreamerV3Critic(dt, num_bins=255))
    cfg = _cfg(N, 16, epochs=1)
    import dataclasses
    cfg = dataclasses.replace(cfg, dreamer_v3_critic=True)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), ml.Policy(actor_critic=ac))
    ps = mgr.state.policy_states
    assert getattr(ps, "generic", False) and ps.critic_bins == 255
    p0 = ps.params.clone()
    mgr.update_iter()
    torch.cuda.synchronize()
    assert torch.isfinite(ps.params).all() and not torch.equal(ps.params, p0)
    assert np.isfinite(mgr.metrics.last()["Loss"].mean)


def test_population_of_separate_backbones_matches_oracle(gpu):
    """A population (cfg.pbt, self-play split) of a tree outside the fused
    kernels: 2 train policies of BackboneSeparate on the torch path, each its
    own copy of the modules, init, optimizer and update RNG (the reference
    vmaps algo.update over the policy axis, train.py:165-174).  Policy p acts
    for env columns [p B, (p + 1) B); each policy's stored values / log-probs
    against the oracle forward with ITS parameters, GAE bit-exact, and each
    policy's whole update (2 epochs x 4 minibatches of its own columns)
    against oracle/separate_ref.py (test_backbone_separate_update_matches_oracle's
    tolerances)."""
    import dataclasses
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
    P, B, H, L, mb, T = 2, 64, 64, 2, 16, 32
    N = P * B
    dt = torch.float32
    env = DummyVecEnv(N, 64, 6, seed=8, device=gpu)
    ac = ml.ActorCritic(
        backbone=ml.BackboneSeparate(actor_encoder=ml.BackboneEncoder(net=MLP(H, L, dt)),
                                     critic_encoder=ml.BackboneEncoder(net=MLP(H, L, dt))),
        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dt),
        critic=DenseLayerCritic(dt))
    pbt = ml.PBTConfig(num_teams=1, team_size=1, num_train_policies=P, num_past_policies=0,
                       self_play_portion=1.0, cross_play_portion=0.0, past_play_portion=0.0)
    cfg = dataclasses.replace(_cfg(N, mb), pbt=pbt)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), ml.Policy(actor_critic=ac))
    pss, tss = mgr.state.policy_list, mgr.state.train_list
    assert len(pss) == P and all(getattr(ps, "generic", False) for ps in pss)
    assert pss[0].actor_critic is not pss[1].actor_critic
    p0s = [_named(ps) for ps in pss]
    order = [n for n, _, _ in pss[0].layout["params"]]
    assert any(not np.array_equal(p0s[0][k], p0s[1][k]) for k in order)  # own inits
    oenv = onat.Env(N, 64, env.k0, env.k1, 0)
    oenv.reset()
    mgr.update_iter()
    torch.cuda.synchronize()
    s = mgr.rollout_mgr.store
    acts = s.actions.cpu().numpy()
    obs = s.obs.float().cpu().numpy()
    for t in range(T):
        assert np.array_equal(obs[t], oenv.obs), t
        o, r, d = oenv.step(acts[t])
        assert np.array_equal(s.rewards[t].cpu().numpy(), r)
        assert np.array_equal(s.dones[t].cpu().numpy(), d)
    full = {k: v.float().cpu().numpy() if v.dtype == torch.bfloat16 else v.cpu().numpy()
            for k, v in s.as_dict().items()}
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
          "normalize_advantages": True}
    for p in range(P):
        c = slice(p * B, (p + 1) * B)
        p0 = p0s[p]
        logits, V, _ = sref.forward(p0, obs[:, c].reshape(T * B, 64), L, "f32")
        lp, _ = ref.action_stats(logits, BUCKETS, acts[:, c].reshape(T * B, 6))
        np.testing.assert_allclose(s.values[:, c].cpu().numpy().reshape(-1), V, rtol=1e-4,
                                   atol=1e-4)
        np.testing.assert_allclose(s.log_probs[:, c].cpu().numpy().reshape(-1, 6), lp,
                                   rtol=1e-4, atol=1e-4)
        store = {k: (v[:, c] if v.ndim >= 2 else v[c]) for k, v in full.items()}
        adv, _ = ref.gae_f32(store["rewards"], store["values"], store["dones"],
                             s.bootstrap[c].cpu().numpy(), cfg.gamma, cfg.gae_lambda)
        assert np.array_equal(store["advantages"], adv)
        init_norms = {k: float(np.sqrt((v * v).sum())) for k, v in p0.items()
                      if k.endswith("kernel") and k.startswith("backbone.")}
        want, _ = sref.ppo_update(dict(p0), order, store, hp, BUCKETS, L, init_norms,
                                  num_epochs=2, minibatch_size=mb, bptt=T,
                                  key=tss[p].update_prng_key, epoch_base=0, mode="f32", lr=3e-4,
                                  max_grad_norm=0.5)
        got = _named(pss[p])
        g = np.concatenate([got[k].reshape(-1) for k in order])
        w = np.concatenate([want[k].reshape(-1) for k in order])
        z = np.concatenate([p0[k].reshape(-1) for k in order])
        np.testing.assert_allclose(g, w, rtol=0, atol=1e-4, err_msg=f"policy {p}")
        close = np.abs(g - w) <= 2e-5 + 1e-4 * np.abs(w)
        assert close.mean() >= 0.999, (p, close.mean())
        dg, dw = g - z, w - z
        assert dg @ dw / (np.linalg.norm(dg) * np.linalg.norm(dw)) > 0.999
        assert int(tss[p].step.item()) == 2 * (B // mb)


def _torch_tree(kind, dt):
    import madrona_learn as ml
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
    from madrona_learn.rnn import LSTM
    if kind == "lstm2":
        bb = ml.BackboneShared(encoder=ml.RecurrentBackboneEncoder(net=MLP(64, 1, dt),
                                                                   rnn=LSTM(64, 2, dt)))
    else:
        bb = ml.BackboneSeparate(actor_encoder=ml.BackboneEncoder(net=MLP(64, 2, dt)),
                                 critic_encoder=ml.BackboneEncoder(net=MLP(64, 2, dt)))
    return ml.ActorCritic(backbone=bb,
                          actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dt),
                          critic=DenseLayerCritic(dt))


@pytest.mark.parametrize("kind", ["separate", "lstm2", "pop2"])
def test_torch_path_graph_replay_matches_eager(gpu, kind):
    """The torch path's whole update (rollout with the user's modules and
    the sim, GAE, the PPO update under autograd) captured in HIP graphs
    (TrainingManager._update_torch: update 1 eager on the capture stream,
    update 2 captured, update 3 replayed) against the same tree trained
    eagerly (use_graph=False): parameters, Adam state, the rollout store and
    the loss metrics bit-identical after every update -- BackboneSeparate, a
    two-layer LSTM (per-chunk start states, C = 2) and a 2-policy population."""
    import dataclasses
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    dt = torch.float32
    P = 2 if kind == "pop2" else 1
    N = 64 * P
    cfg = _cfg(N, 16)
    if kind == "lstm2":
        cfg = dataclasses.replace(cfg, num_bptt_chunks=2)
    if kind == "pop2":
        cfg = dataclasses.replace(cfg, pbt=ml.PBTConfig(
            num_teams=1, team_size=1, num_train_policies=P, num_past_policies=0,
            self_play_portion=1.0, cross_play_portion=0.0, past_play_portion=0.0))
    mgrs = []
    for use_graph in (False, True):
        env = DummyVecEnv(N, 64, 6, seed=12, device=gpu)
        mgrs.append(ml.init_training(gpu, cfg, env.sim_fns(),
                                     ml.Policy(actor_critic=_torch_tree(kind, dt)),
                                     use_graph=use_graph))
    eager, graph = mgrs
    assert not eager.use_graph and graph.use_graph and graph._torch_path
    for it in range(3):
        for m in mgrs:
            m.update_iter()
        torch.cuda.synchronize()
        assert graph.use_graph, "the update fell back to eager"
        assert (graph._segments is not None) == (it >= 1)
        for pe, pg in zip(eager.state.policy_list, graph.state.policy_list):
            assert torch.equal(pe.params, pg.params), (it, kind)
        for te, tg in zip(eager.state.train_list, graph.state.train_list):
            assert torch.equal(te.adam_m, tg.adam_m) and torch.equal(te.adam_v, tg.adam_v)
            assert torch.equal(te.step, tg.step)
        se, sg = eager.rollout_mgr.store, graph.rollout_mgr.store
        for k, v in se.as_dict().items():
            assert torch.equal(v, sg.as_dict()[k]), (it, k)
        le, lg = eager.metrics.last(), graph.metrics.last()
        for k in ("Loss", "Value Loss", "Entropy"):
            assert le[k].mean == lg[k].mean, (it, k)
    assert graph.graph_scope == "all"  # the rollout was captured too
    assert int(graph.state.train_list[0].step.item()) == 3 * 2 * (cfg.num_bptt_chunks * 64 // 16)


@pytest.mark.parametrize("where", ["rollout", "update"])
def test_torch_path_uncapturable_tree_falls_back(gpu, capsys, where):
    """A user module that reads a device value on the host (not capturable in
    a HIP graph) keeps training.  In its rollout forward: the whole-update
    capture at update 2 fails, the host references it moved are restored and
    only the PPO update is captured (graph_scope "learn").  In its training
    forward: that capture fails too and updates run eagerly.  Either way
    bit-identical to a use_graph=False run."""
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor

    class SyncingMLP(MLP):
        def forward(self, inputs, train=False):
            if train == (where == "update"):
                _ = float(inputs.float().abs().max().item())  # a host read
            return super().forward(inputs, train)

    dt = torch.float32

    def tree():
        return ml.ActorCritic(
            backbone=ml.BackboneSeparate(actor_encoder=ml.BackboneEncoder(net=SyncingMLP(64, 2, dt)),
                                         critic_encoder=ml.BackboneEncoder(net=MLP(64, 2, dt))),
            actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dt),
            critic=DenseLayerCritic(dt))

    mgrs = []
    for use_graph in (False, True):
        env = DummyVecEnv(64, 64, 6, seed=13, device=gpu)
        mgrs.append(ml.init_training(gpu, _cfg(64, 16), env.sim_fns(),
                                     ml.Policy(actor_critic=tree()), use_graph=use_graph))
    eager, graph = mgrs
    for it in range(3):
        for m in mgrs:
            m.update_iter()
        torch.cuda.synchronize()
        assert torch.equal(eager.state.policy_states.params, graph.state.policy_states.params), it
    if where == "update":
        assert not graph.use_graph and graph._segments is None
    else:
        assert graph.use_graph and graph.graph_scope == "learn" and graph._segments is not None
    assert "not capturable" in capsys.readouterr().err
