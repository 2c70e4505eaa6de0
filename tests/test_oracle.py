"""CPU pins of the parity oracle: external known-answer vectors
(Random123 Philox4x32-10), closed-form cases derived from the reference's
equations, invariants of the replaced RNG constructs, and the committed
golden fixtures (tests/golden, made by tests/golden/make_golden.py).

No reference code is imported (JAX is absent: parity beyond these cases is
"parity unpinned", DESIGN.md "Oracle")."""

import os

import numpy as np
import pytest

from oracle import native
from oracle import ppo_ref as ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BUCKETS = [4, 8, 5, 5, 2, 2]


# ---------------------------------------------------------------------------
# Philox4x32-10: Random123 known-answer vectors (kat_vectors, philox4x32 10)
# ---------------------------------------------------------------------------
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_random123_kat(ctr, key, want):
    out = native.philox(np.array([ctr], np.uint32), key[0], key[1])
    assert tuple(int(x) for x in out[0]) == want


def test_det_log2_accuracy():
    x = np.concatenate([np.geomspace(1e-30, 1e30, 20001), np.linspace(0.5, 2.0, 4001)])
    x = x.astype(np.float32)
    got = np.array([native.lib().oracle_log2(float(v)) for v in x[::7]], np.float64)
    want = np.log2(x[::7].astype(np.float64))
    err = np.abs(got - want) / np.maximum(np.abs(want), 1.0)
    assert err.max() < 4e-7


def test_gumbel_sampler_distribution():
    """Gumbel-max with the counter RNG samples softmax(logits) (the property
    jax.random.categorical guarantees, dists.py:33-38)."""
    logits = np.array([[0.3, -1.2, 2.0, 0.0, 0.5]], np.float32)
    N = 40000
    lg = np.repeat(logits, N, 0)
    acts = native.sample(lg, [5], 7, 9, step=3)[:, 0]
    freq = np.bincount(acts, minlength=5) / N
    p = np.exp(logits[0] - logits[0].max())
    p /= p.sum()
    # 5 sigma binomial band
    assert np.all(np.abs(freq - p) < 5 * np.sqrt(p * (1 - p) / N))


def test_sampler_argmax_and_logprob():
    rng = np.random.default_rng(0)
    logits = rng.standard_normal((257, 26)).astype(np.float32)
    acts = native.sample(logits, BUCKETS, 1, 2, step=5)
    gum = native.gumbel_table(1, 2, 5, 0, 257, 26)
    want, lp = ref.sample_actions(logits, BUCKETS, gum)
    assert np.array_equal(acts, want)
    elp, _ = ref.action_stats(logits, BUCKETS, want)
    np.testing.assert_allclose(lp, elp, rtol=1e-6, atol=1e-6)
    # sample=False: argmax (DiscreteActionDistributions.best, dists.py:46-52)
    best = native.sample(logits, BUCKETS, 1, 2, step=5, sample=False)
    off = 0
    for g, nb in enumerate(BUCKETS):
        assert np.array_equal(best[:, g], np.argmax(logits[:, off:off + nb], -1))
        off += nb


# ---------------------------------------------------------------------------
# GAE / returns closed forms (algo_common.py:45-130)
# ---------------------------------------------------------------------------
def _rvd(T=32, N=64, seed=0, pdone=0.1):
    rng = np.random.default_rng(seed)
    r = rng.standard_normal((T, N)).astype(np.float32)
    v = rng.standard_normal((T, N)).astype(np.float32)
    d = (rng.random((T, N)) < pdone).astype(np.uint8)
    b = rng.standard_normal(N).astype(np.float32)
    return r, v, d, b


@pytest.mark.parametrize("fn", [ref.gae_f32, ref.gae])
def test_gae_gamma1_lambda1_no_dones(fn):
    r, v, d, b = _rvd(pdone=0.0)
    adv, ret = fn(r, v, d, b, 1.0, 1.0)
    want = np.cumsum(r[::-1].astype(np.float64), 0)[::-1] + b[None].astype(np.float64) - v
    np.testing.assert_allclose(adv, want, rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(ret, adv.astype(np.float64) + v, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("fn", [ref.gae_f32, ref.gae])
def test_gae_all_done(fn):
    r, v, d, b = _rvd()
    adv, _ = fn(r, v, np.ones_like(d), b, 0.99, 0.95)
    np.testing.assert_allclose(adv, r.astype(np.float64) - v, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("fn", [ref.gae_f32, ref.gae])
def test_gae_lambda0_is_td_error(fn):
    r, v, d, b = _rvd()
    g = 0.97
    adv, _ = fn(r, v, d, b, g, 0.0)
    nv = np.concatenate([v[1:], b[None]], 0).astype(np.float64)
    nv = np.where(d.astype(bool), 0.0, nv)
    np.testing.assert_allclose(adv, r + g * nv - v, rtol=1e-5, atol=1e-5)


def test_gae_f32_matches_f64():
    r, v, d, b = _rvd(seed=3)
    a32, r32 = ref.gae_f32(r, v, d, b, 0.99, 0.95)
    a64, r64 = ref.gae(r, v, d, b, 0.99, 0.95)
    np.testing.assert_allclose(a32, a64, rtol=1e-5, atol=1e-5)


def test_gae_gamma_lambda_single_rounding():
    """algo_common.py:120 forms cfg.gamma * cfg.gae_lambda from Python floats
    (one f64 product, rounded to f32 once by JAX's weak typing).  The oracle
    must use that constant: with no dones, lambda = 1 recursion check on one
    step isolates it (A_T-1 = r + g * boot - v; A_T-2 = td + gl * A_T-1)."""
    g, lam = 0.998, 0.95
    gl_ref = np.float32(g * lam)
    assert gl_ref != np.float32(np.float32(g) * np.float32(lam))  # the two roundings differ
    r = np.array([[0.0], [0.0]], np.float32)
    v = np.array([[0.0], [0.0]], np.float32)
    d = np.zeros((2, 1), bool)
    b = np.array([1.0], np.float32)
    adv, _ = ref.gae_f32(r, v, d, b, g, lam)
    assert adv[1, 0] == np.float32(g)
    assert adv[0, 0] == np.float32(gl_ref * np.float32(g))


def test_discounted_returns():
    r, v, d, b = _rvd(pdone=0.0)
    out = ref.discounted_returns_f32(r, d, b, 1.0)
    want = np.cumsum(r[::-1].astype(np.float64), 0)[::-1] + b[None]
    np.testing.assert_allclose(out, want, rtol=1e-5, atol=2e-5)
    out = ref.discounted_returns_f32(r, np.ones_like(d), b, 0.9)
    np.testing.assert_allclose(out, r, rtol=0, atol=0)


def test_zscore_population_variance_and_floor():
    x = np.array([1.0, 2.0, 3.0, 4.0])
    z, mean, var = ref.zscore(x)
    assert mean == 2.5 and var == 1.25
    np.testing.assert_allclose(z, (x - 2.5) / np.sqrt(1.25))
    z, _, var = ref.zscore(np.full(8, 3.0))
    assert var == 0.0 and np.all(z == 0.0)  # rsqrt(max(var, 1e-5)) keeps it finite


# ---------------------------------------------------------------------------
# optimizer (ppo.py:84-90, 283-338; optax 0.1.9 defaults)
# ---------------------------------------------------------------------------
def test_adam_first_step_closed_form():
    rng = np.random.default_rng(1)
    p = rng.standard_normal(1000)
    g = rng.standard_normal(1000)
    z = np.zeros_like(p)
    p1, m1, v1 = ref.adam_step(p, g, z, z.copy(), 0, 3e-4)
    # m_hat = g, v_hat = g^2  ->  step = -lr * g / (|g| + eps)
    np.testing.assert_allclose(p1, p - 3e-4 * g / (np.abs(g) + ref.ADAM_EPS), rtol=1e-12)
    np.testing.assert_allclose(m1, 0.1 * g)
    np.testing.assert_allclose(v1, 0.001 * g * g)


def test_clip_by_global_norm():
    g = np.array([3.0, 4.0])
    c, n = ref.clip_by_global_norm(g, 0.5)
    assert n == 5.0
    np.testing.assert_allclose(c, g / 5.0 * 0.5)
    c, _ = ref.clip_by_global_norm(g, 10.0)
    np.testing.assert_allclose(c, g)


def test_projections_restore_norms():
    lay = ref.param_layout(16, 64, 2, 26)
    rng = np.random.default_rng(2)
    flat = rng.standard_normal(lay["total"])
    P = ref.unflatten(flat, lay)
    init = np.array([1.5, 2.5])
    Q = ref.project(ref.unflatten(flat.copy(), lay), init)
    for l in range(2):
        assert np.isclose(np.linalg.norm(Q["W"][l]), init[l])
        assert np.isclose((Q["s"][l] ** 2).sum() + (Q["b"][l] ** 2).sum(), 64.0)
    # actor/critic head untouched (ppo.py:303-310 skips actor/critic kernels)
    assert np.array_equal(Q["Wh"], P["Wh"]) and np.array_equal(Q["bh"], P["bh"])


# ---------------------------------------------------------------------------
# minibatching (ppo.py:437-458, rollouts.py:319-329, 786-804)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1, 2, 3, 5, 64, 1000, 8192, 10007])
def test_epoch_permutation_is_bijection(n):
    p = ref.epoch_permutation(11, 22, 7, 3, n)
    assert p.dtype == np.int32 and np.array_equal(np.sort(p), np.arange(n))
    assert np.array_equal(p, ref.epoch_permutation(11, 22, 7, 3, n))


def test_epoch_permutation_depends_on_epoch_rank_key():
    a = ref.epoch_permutation(11, 22, 7, 0, 4096)
    assert not np.array_equal(a, ref.epoch_permutation(11, 22, 8, 0, 4096))
    assert not np.array_equal(a, ref.epoch_permutation(11, 22, 7, 1, 4096))
    assert not np.array_equal(a, ref.epoch_permutation(12, 22, 7, 0, 4096))
    # roughly uniform displacement: a shuffle, not a near-identity
    assert np.mean(a == np.arange(4096)) < 0.01


def _reference_reorder(x, C):
    """_finalize_rollouts transpose (rollouts.py:786-804) restated for P = 1:
    store [C, T/C, B, ...] -> [C*B, T/C, ...] (sequence-major)."""
    T, B = x.shape[:2]
    y = x.reshape(C, T // C, B, *x.shape[2:])
    y = np.swapaxes(y, 1, 2)  # [C, B, T/C, ...]
    return y.reshape(C * B, T // C, *x.shape[2:])


@pytest.mark.parametrize("C", [1, 2, 4])
def test_minibatch_rows_match_reference_reorder(C):
    """RolloutData.minibatch (take over sequences, swapaxes to [T/C, mb])
    on the reference's reordered store equals our direct row gather."""
    T, N = 32, 24
    store = (np.arange(T * N, dtype=np.int64) * 7 + 3).reshape(T, N)  # integer KAT data
    seqs = ref.epoch_permutation(5, 6, 1, 0, C * N)[:10]
    want = np.swapaxes(_reference_reorder(store, C)[seqs], 0, 1)  # [T/C, mb]
    got = store.reshape(-1)[ref.minibatch_rows(seqs, N, T // C)].reshape(T // C, len(seqs))
    assert np.array_equal(got, want)


# ---------------------------------------------------------------------------
# golden fixtures (regression pin of the oracle; tests/golden/make_golden.py)
# ---------------------------------------------------------------------------
def _golden(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        pytest.fail(f"missing golden fixture {name}: run tests/golden/make_golden.py")
    return np.load(path, allow_pickle=False)


def test_golden_gae():
    g = _golden("gae_32x64.npz")
    adv, ret = ref.gae_f32(g["rewards"], g["values"], g["dones"], g["bootstrap"],
                           float(g["gamma"]), float(g["lam"]))
    assert np.array_equal(adv, g["advantages"]) and np.array_equal(ret, g["returns"])


def test_golden_ppo_loss_grads():
    g = _golden("ppo_4x16.npz")
    lay = ref.param_layout(int(g["D"]), int(g["H"]), int(g["L"]), int(sum(g["buckets"])))
    P = ref.unflatten(g["params"], lay)
    batch = {k: g[k] for k in ("obs", "actions", "log_probs", "advantages", "returns", "values")}
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
          "normalize_advantages": True}
    loss, G, _, _ = ref.ppo_loss_grads(P, batch, hp, list(g["buckets"]), "f64")
    np.testing.assert_allclose(loss, g["loss"], rtol=1e-12)
    np.testing.assert_allclose(ref.flatten(G, lay), g["grads"], rtol=1e-10, atol=1e-14)


def test_golden_optimizer_step():
    g = _golden("optim_step.npz")
    lay = ref.param_layout(int(g["D"]), int(g["H"]), int(g["L"]), int(g["A"]))
    p, m, v, gn = ref.optimizer_step(g["p0"], g["grad"], g["m0"], g["v0"], int(g["count"]), lay,
                                     g["init_norms"], float(g["lr"]), float(g["max_norm"]))
    np.testing.assert_allclose(p, g["p1"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(m, g["m1"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(v, g["v1"], rtol=1e-12, atol=1e-15)


# ---------------------------------------------------------------------------
# SymExpTwoHotDistribution (DreamerV3Critic, dists.py:119-208): closed-form
# properties of the restatement (parity with executed reference output is
# unpinned: no JAX here and no reference fixture for this distribution)
# ---------------------------------------------------------------------------
def test_twohot_bins_and_mean():
    b = ref.twohot_bins(63)
    assert b.dtype == np.float32 and b.shape == (63,)
    assert b[31] == 0 and np.array_equal(b[32:], -b[:31][::-1])
    assert np.all(np.diff(b) > 0)
    np.testing.assert_allclose(b[0], -np.expm1(14.0), rtol=1e-6)
    # the symmetric sum is exactly 0 at initialisation (zero-init critic)
    assert ref.twohot_mean(np.zeros((3, 63), np.float32)).tolist() == [0.0, 0.0, 0.0]
    lg = np.full((1, 63), -1e4)
    lg[0, 40] = 0.0
    np.testing.assert_allclose(ref.twohot_mean(lg), b[40], rtol=1e-6)


def test_twohot_weights_follow_the_reference():
    """two_hot_cross_entropy_loss weighs the lower bin by |b_lo - t| / gap
    (dists.py:193-196, as written)."""
    b = ref.twohot_bins(63).astype(np.float64)
    t = 0.25 * b[40] + 0.75 * b[41]
    W = ref.twohot_weights(63, [t])
    np.testing.assert_allclose(W[0, 40], 0.75, rtol=1e-9)
    np.testing.assert_allclose(W[0, 41], 0.25, rtol=1e-9)
    W = ref.twohot_weights(63, [b[40]])           # on a bin: dist_to_lower = 0
    assert W[0, 41] == 1.0 and W[0].sum() == 1.0
    W = ref.twohot_weights(63, [1e9, -1e9])      # clipped indices coincide: 1/2 + 1/2
    assert W[0, 62] == 1.0 and W[1, 0] == 1.0
    loss, grad = ref.twohot_ce(np.zeros((2, 63)), np.array([1e9, 0.3]))
    np.testing.assert_allclose(loss, np.log(63.0), rtol=1e-12)
    np.testing.assert_allclose(grad.sum(-1), 0.0, atol=1e-15)


# ---------------------------------------------------------------------------
# EMANormalizer (moving_avg.py:48-196): closed forms of the restatement
# ---------------------------------------------------------------------------
def test_ema_normalizer_closed_forms():
    rng = np.random.default_rng(3)
    xs = [(rng.standard_normal((50, 4)) * 2 + 1).astype(np.float32) for _ in range(6)]
    st = (np.zeros(4, np.float32), np.zeros(4, np.float32))
    for t, x in enumerate(xs):
        st = ref.ema_update_input_stats(st, t, x)
    # equal-size batches: the running fold is the pooled mean / population variance
    allx = np.concatenate(xs).astype(np.float64)
    np.testing.assert_allclose(st[0], allx.mean(0), rtol=1e-5)
    np.testing.assert_allclose(st[1], allx.var(0), rtol=1e-5)
    # first update: the bias correction makes the estimate the batch statistics
    e = ref.ema_update_estimates(ref.ema_init(4), st, 0.999, 1e-5)
    np.testing.assert_allclose(e["mu"], st[0], rtol=1e-3)
    np.testing.assert_allclose(e["sigma"] ** 2, st[1], rtol=2e-3)
    assert e["N"] == 1
    # a constant feature: variance floored at eps (rsqrt(max(var, eps)))
    c = ref.ema_update_input_stats((np.zeros(1, np.float32), np.zeros(1, np.float32)), 0,
                                   np.full((8, 1), 3.0, np.float32))
    e = ref.ema_update_estimates(ref.ema_init(1), c, 0.9, 1e-5)
    np.testing.assert_allclose(e["inv_sigma"], 1 / np.sqrt(1e-5), rtol=1e-6)
    y = ref.ema_normalize(e, np.full((2, 1), 3.0, np.float32), "f32")
    np.testing.assert_allclose(y, 0.0, atol=1e-3)


# ---------------------------------------------------------------------------
# Value normaliser (normalize_values, ppo.py:190-211): closed forms
# ---------------------------------------------------------------------------
def test_value_normaliser_first_update_and_loss_target():
    """The first update's estimates are the minibatch's own mean / population
    variance (bias correction, moving_avg.py:163-167); the value target is the
    return normalised with the updated estimates and the value error inverts
    the critic with the previous ones (ppo.py:190-211)."""
    rng = np.random.default_rng(7)
    M, buckets = 64, [4, 8, 5, 5, 2, 2]
    R = (rng.standard_normal(M) * 3 + 2).astype(np.float32)
    z = np.zeros(1, np.float32)
    est = ref.ema_init(1)
    new = ref.ema_update_estimates(est, ref.ema_update_input_stats((z, z), 0, R[:, None]),
                                   0.99999, 1e-5)
    np.testing.assert_allclose(new["mu"][0], R.astype(np.float64).mean(), rtol=1e-4)
    np.testing.assert_allclose(new["sigma"][0] ** 2, R.astype(np.float64).var(), rtol=1e-3)
    assert new["N"] == 1
    # invert is the inverse of normalize
    x = rng.standard_normal(5).astype(np.float32)
    np.testing.assert_allclose(ref.ema_invert(new, ref.ema_normalize(new, x, "f32")), x,
                               rtol=1e-5, atol=1e-5)
    V = rng.standard_normal(M)
    batch = {"actions": np.zeros((M, 6), np.int32), "log_probs": np.zeros((M, 6)),
             "advantages": rng.standard_normal(M), "returns": R, "values": np.zeros(M)}
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
          "value_norm": (new["mu"][0], new["inv_sigma"][0], 0.5, 2.0)}
    _, dhead, met = ref.ppo_loss_dhead(np.zeros((M, 26)), V, batch, hp, buckets)
    tgt = (R - np.float32(new["mu"][0])) * np.float32(new["inv_sigma"][0])
    np.testing.assert_allclose(dhead[:, -1], 0.5 / M * (V - tgt), rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(met["Value Errors"], np.abs(V * 2.0 + 0.5 - R), rtol=1e-12)
