"""GPU parity of the fused MLP actor-critic kernels (rollout step, PPO
minibatch gradient, optimizer step) against the NumPy oracle.

Tolerances: compute_dtype float32 — loss within 1e-5 relative (north star),
values/log-probs/gradients within 1e-4 relative of the fp64 oracle; bfloat16
— the oracle emulates the reference's bf16 rounding points, and results are
compared within 2e-2 relative (one bf16 ulp is 2^-8 = 3.9e-3).  Sampled
actions must equal the oracle's wherever the oracle's Gumbel-perturbed top-2
margin exceeds 1e-3 (bit-exact sampler: see test_gpu_kernels).
"""

import numpy as np
import pytest
import torch

from oracle import native as onat
from oracle import ppo_ref as ref

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]


def make_critic(critic_bins, dtype):
    from madrona_learn.models import DenseLayerCritic, DreamerV3Critic
    return DenseLayerCritic(dtype) if critic_bins == 1 else DreamerV3Critic(dtype,
                                                                            num_bins=critic_bins)


def make_policy_state(gpu, obs_dim, hidden, layers, dtype, seed=0, critic_bins=1):
    import madrona_learn as ml
    from madrona_learn.models import MLP, DenseLayerDiscreteActor
    from madrona_learn.train_state import PolicyState, compile_arch
    ac = ml.ActorCritic(
        backbone=ml.BackboneShared(encoder=ml.BackboneEncoder(net=MLP(hidden, layers, dtype))),
        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dtype),
        critic=make_critic(critic_bins, dtype))
    arch = compile_arch(ac, obs_dim, dtype)
    return PolicyState(ac, arch, None, gpu, np.random.default_rng(seed))


def perturb(ps, seed, scale=0.05, critic_scale=0.3):
    """Non-trivial LayerNorm / bias parameters (init is scale 1, bias 0) and,
    for a two-hot critic, non-trivial (zero-initialised) bin weights."""
    rng = np.random.default_rng(seed)
    p = ps.params.cpu().numpy()
    for key in ("s", "b"):
        for o, shp in ps.layout[key]:
            p[o:o + shp[0]] += rng.standard_normal(shp[0]).astype(np.float32) * 0.3
    o, shp = ps.layout["hw"]
    p[o:o + shp[0] * shp[1]] += rng.standard_normal(shp[0] * shp[1]).astype(np.float32) * scale
    if ps.arch.critic_bins > 1:
        hw = p[o:o + shp[0] * shp[1]].reshape(shp)
        A = ps.arch.num_logits
        hw[:, A:] += rng.standard_normal(hw[:, A:].shape).astype(np.float32) * critic_scale
    o, shp = ps.layout["hb"]
    p[o:o + shp[0]] += rng.standard_normal(shp[0]).astype(np.float32) * 0.1
    ps.params.copy_(torch.from_numpy(p))
    ps.sync_weights()


def oracle_layout(ps):
    a = ps.arch
    return ref.param_layout(a.obs_dim, a.hidden, a.num_layers, a.num_logits, a.critic_bins)


CASES = [("f32", torch.float32, 64, 256, 2), ("bf16", torch.bfloat16, 64, 256, 2),
         ("f32", torch.float32, 32, 64, 2), ("bf16", torch.bfloat16, 48, 128, 3),
         ("f32", torch.float32, 16, 128, 1)]
# DreamerV3Critic (two-hot, 63 bins: head width 96) on a subset of the shapes
CRITIC_CASES = [c + (1,) for c in CASES] + [
    ("f32", torch.float32, 64, 256, 2, 63), ("bf16", torch.bfloat16, 64, 256, 2, 63),
    ("f32", torch.float32, 32, 64, 2, 63), ("f32", torch.float32, 16, 128, 1, 5)]


@pytest.mark.parametrize("mode,dtype,D,H,L,CB", CRITIC_CASES)
def test_rollout_step(gpu, mode, dtype, D, H, L, CB):
    ps = make_policy_state(gpu, D, H, L, dtype, seed=D + H, critic_bins=CB)
    perturb(ps, 1)
    N = 1000
    rng = np.random.default_rng(2)
    obs = rng.standard_normal((N, D)).astype(np.float32)
    o = torch.from_numpy(obs).to(gpu)
    store = torch.zeros((N, D), dtype=dtype, device=gpu)
    acts = torch.zeros((N, 6), dtype=torch.int32, device=gpu)
    logp = torch.zeros((N, 6), dtype=torch.float32, device=gpu)
    vals = torch.zeros(N, dtype=torch.float32, device=gpu)
    ctr = torch.tensor([100, 0, 0, 0], dtype=torch.int64, device=gpu)
    ps.rollout_step(o, store, acts, logp, vals, (5, 6), ctr[0:1], 7, env_offset=3)
    torch.cuda.synchronize()
    P = ref.unflatten(ps.params.cpu().numpy(), oracle_layout(ps))
    logits, V, _ = ref.forward(P, obs, mode)
    assert np.array_equal(store.float().cpu().numpy(), ref.rnd(obs, mode).astype(np.float32))
    tol = 1e-4 if mode == "f32" else 2e-2
    vtol = tol * (1.0 if CB == 1 else max(1.0, float(np.abs(V).max())))
    np.testing.assert_allclose(vals.cpu().numpy(), V, rtol=tol, atol=vtol)
    if CB > 1:
        assert np.abs(V).max() > 1e-2, "two-hot values should be non-trivial"
    gum = onat.gumbel_table(5, 6, 107, 3, N, 26)
    noisy = logits.astype(np.float32) + gum
    exp_acts, _ = ref.sample_actions(logits.astype(np.float32), BUCKETS, gum)
    got = acts.cpu().numpy()
    off = 0
    for g, nb in enumerate(BUCKETS):
        srt = np.sort(noisy[:, off:off + nb], axis=-1)
        clear = (srt[:, -1] - srt[:, -2]) > 1e-3
        assert np.array_equal(got[clear, g], exp_acts[clear, g]), f"group {g}"
        off += nb
    elogp, _ = ref.action_stats(logits, BUCKETS, got)
    np.testing.assert_allclose(logp.cpu().numpy(), elogp, rtol=tol, atol=tol)
    # critic only (bootstrap path)
    v2 = torch.zeros(N, dtype=torch.float32, device=gpu)
    ps.critic_only(o, v2)
    assert torch.equal(v2, vals)


def _random_store(rng, T, N, D, ps, mode):
    obs = ref.rnd(rng.standard_normal((T, N, D)), mode).astype(np.float32)
    P = ref.unflatten(ps.params.cpu().numpy(), oracle_layout(ps))
    logits, V, _ = ref.forward(P, obs.reshape(T * N, D), mode)
    acts = np.stack([rng.integers(0, b, T * N) for b in BUCKETS], -1).astype(np.int32)
    lp, _ = ref.action_stats(logits, BUCKETS, acts)
    lp = (lp + rng.standard_normal(lp.shape) * 0.1).astype(np.float32)  # old policy != new
    return {
        "obs": obs,
        "actions": acts.reshape(T, N, 6),
        "log_probs": lp.reshape(T, N, 6),
        "values": V.astype(np.float32).reshape(T, N),
        "advantages": (rng.standard_normal((T, N)) * 2 + 0.3).astype(np.float32),
        "returns": (V.reshape(T, N) + rng.standard_normal((T, N))).astype(np.float32),
        "rewards": np.zeros((T, N), np.float32),
    }


def _device_store(gpu, st, dtype):
    from madrona_learn.rollouts import RolloutStore
    T, N, D = st["obs"].shape
    s = RolloutStore(T, N, D, 6, dtype, gpu)
    s.obs.copy_(torch.from_numpy(st["obs"]).to(dtype))
    s.actions.copy_(torch.from_numpy(st["actions"]))
    s.log_probs.copy_(torch.from_numpy(st["log_probs"]))
    s.values.copy_(torch.from_numpy(st["values"]))
    s.advantages.copy_(torch.from_numpy(st["advantages"]))
    s.returns.copy_(torch.from_numpy(st["returns"]))
    return s


HP = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
      "normalize_advantages": True}


@pytest.mark.parametrize("mode,dtype,D,H,L,CB", CRITIC_CASES)
@pytest.mark.parametrize("bptt", [32, 16])
@pytest.mark.parametrize("mb", [40, 37])
def test_minibatch_grad(gpu, mode, dtype, D, H, L, CB, bptt, mb):
    """mb = 37 leaves padding rows in the last 64-row block (37 x 32 = 1184
    of 1216)."""
    from madrona_learn import _native as nat
    ps = make_policy_state(gpu, D, H, L, dtype, seed=H, critic_bins=CB)
    perturb(ps, 9, scale=0.2)
    T, N = 32, 96
    rng = np.random.default_rng(11)
    st = _random_store(rng, T, N, D, ps, mode)
    if CB > 1:  # returns spread over many bins
        st["returns"] = (st["returns"] * 20.0).astype(np.float32)
    s = _device_store(gpu, st, dtype)
    nseq = (T // bptt) * N
    seqs = rng.permutation(nseq)[:mb].astype(np.int32)
    rows = ref.minibatch_rows(seqs, N, bptt)
    batch = ref.gather_minibatch(st, rows)
    adv = batch["advantages"].astype(np.float64)
    P = ref.unflatten(ps.params.cpu().numpy(), oracle_layout(ps))
    loss, G, met, _ = ref.ppo_loss_grads(P, batch, HP, BUCKETS, mode)
    gflat = ref.flatten(G, oracle_layout(ps))

    view = s.view(bptt)
    hp = nat.PPOHparams()
    hp.clip_coef, hp.value_loss_coef = 0.2, 0.5
    for k in range(6):
        hp.entropy_coef[k] = 0.01
    hp.normalize_advantages, hp.loss_scale = 1, 1.0
    stats = torch.tensor([adv.mean(), 1.0 / np.sqrt(max(adv.var(), 1e-5))], dtype=torch.float32,
                         device=gpu)
    M = mb * bptt
    ws = torch.zeros(int(nat.lib().mlearn_ppo_workspace_bytes(ps.desc, M)), dtype=torch.uint8,
                     device=gpu)
    grad = torch.zeros(ps.layout["total"], dtype=torch.float32, device=gpu)
    out = torch.zeros(25, dtype=torch.float32, device=gpu)
    sq = torch.from_numpy(seqs).to(gpu)
    nat.check(nat.lib().mlearn_ppo_minibatch_grad(ps.desc, view, nat.ptr(sq), mb, nat.ptr(stats),
                                                  hp, nat.ptr(grad), nat.ptr(out), nat.ptr(ws),
                                                  nat.stream_handle()))
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    g = grad.cpu().numpy()
    if mode == "f32":
        np.testing.assert_allclose(o[0], loss, rtol=1e-5, atol=1e-7)
        scale = np.abs(gflat).max()
        np.testing.assert_allclose(g, gflat, rtol=1e-3, atol=1e-4 * scale)
    else:
        np.testing.assert_allclose(o[0], loss, rtol=2e-2, atol=2e-3)
        scale = np.abs(gflat).max()
        err = np.abs(g - gflat).max() / scale
        assert err < 3e-2, err
        cos = g @ gflat / (np.linalg.norm(g) * np.linalg.norm(gflat))
        assert cos > 0.999
    # metrics vectors: 'Value Loss' mean and 'Entropy' mean
    np.testing.assert_allclose(o[10], met["Value Loss"].mean(), rtol=2e-2 if mode == "bf16" else 1e-5)
    np.testing.assert_allclose(o[20], met["Entropy"].mean(), rtol=2e-2 if mode == "bf16" else 1e-5)
    assert o[14] == mb * bptt and o[24] == mb * bptt * 6


def test_optimizer_step(gpu):
    from madrona_learn.train_state import PolicyTrainState
    from madrona_learn.ppo import PPOHyperParams
    ps = make_policy_state(gpu, 64, 256, 2, torch.float32, seed=4)
    perturb(ps, 5)
    hp = PPOHyperParams(lr=3e-4, gamma=0.99, gae_lambda=0.95, normalize_values=False,
                        value_normalizer_decay=0.0, max_advantage_est_decay=0.0, clip_coef=0.2,
                        value_loss_coef=0.5, entropy_coef=0.01, max_grad_norm=0.5)
    ts = PolicyTrainState(None, hp, ps, (1, 2))
    lay = oracle_layout(ps)
    rng = np.random.default_rng(6)
    p = ps.params.cpu().numpy().astype(np.float64)
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    init_norms = ps.init_norms.cpu().numpy().astype(np.float64)
    for step in range(3):
        g = (rng.standard_normal(p.size) * (0.01 if step != 1 else 1.0)).astype(np.float32)
        ts.grads.copy_(torch.from_numpy(g))
        ts.optimizer_step(ps)
        p, m, v, gn = ref.optimizer_step(p, g.astype(np.float64), m, v, step, lay, init_norms,
                                         3e-4, 0.5)
    torch.cuda.synchronize()
    got = ps.params.cpu().numpy()
    np.testing.assert_allclose(got, p, rtol=2e-5, atol=2e-6)
    assert int(ts.step.item()) == 3
    # compute-dtype operand images follow the master weights (frag.py)
    from madrona_learn.frag import from_image
    for l in range(2):
        wl = ps.view("w", l)
        fin, H = wl.shape
        assert torch.equal(from_image(ps.w_t[l], H, fin, l > 0), wl.t())
        if l > 0:
            assert torch.equal(from_image(ps.w[l], fin, H, True), wl)
    hw = ps.view("hw")
    A1 = hw.shape[1]
    assert torch.equal(from_image(ps.head_t, 32, 256, True)[:A1], hw.t())
    assert torch.equal(from_image(ps.head, 256, 32, False)[:, :A1], hw)
    assert not from_image(ps.head, 256, 32, False)[:, A1:].any()
