"""GPU parity of the PPO minibatch gradient at the sizes the benchmarks run
(SURVEY §8(d) B1 / headline: 8192-env store, minibatch 2048 sequences x
bptt 32 = 65,536 rows, MLP[256,256], 2048 workgroups of the step kernel)
and of the value-loss variants of PPOConfig (clip_value_loss,
huber_value_loss; ppo.py:197-218) including rows sitting exactly on the
clip bounds and on the huber kink, where JAX's balanced min / max / abs
derivatives give 0.5 (oracle ppo_ref.ppo_loss_dhead restates them).

Tolerances as test_gpu_policy: f32 loss within 1e-5 relative, gradients
within 1e-3 relative + 1e-4 x max|g|; bf16 gradients within 3e-2 x max|g|,
cosine > 0.999."""

import numpy as np
import pytest
import torch

from oracle import ppo_ref as ref
from tests.test_gpu_policy import BUCKETS, make_policy_state, oracle_layout, perturb

pytestmark = pytest.mark.gpu


def _minibatch_store(rng, ps, T, N, D, mode, seqs, bptt):
    """[T][N] store whose minibatch rows carry old log-probs / values from the
    oracle forward of the current parameters (+ noise, so ratios != 1);
    every other row is random (never read)."""
    obs = ref.rnd(rng.standard_normal((T, N, D), dtype=np.float32), mode).astype(np.float32)
    acts = np.stack([rng.integers(0, b, (T, N)) for b in BUCKETS], -1).astype(np.int32)
    st = {"obs": obs, "actions": acts,
          "log_probs": (rng.standard_normal((T, N, 6)) - 2.0).astype(np.float32),
          "values": rng.standard_normal((T, N)).astype(np.float32),
          "advantages": (rng.standard_normal((T, N)) * 2 + 0.3).astype(np.float32),
          "returns": rng.standard_normal((T, N)).astype(np.float32),
          "rewards": np.zeros((T, N), np.float32)}
    rows = ref.minibatch_rows(seqs, N, bptt)
    P = ref.unflatten(ps.params.cpu().numpy(), oracle_layout(ps))
    logits, V, _ = ref.forward(P, obs.reshape(T * N, D)[rows], mode)
    lp, _ = ref.action_stats(logits, BUCKETS, acts.reshape(T * N, 6)[rows])
    lpf = st["log_probs"].reshape(T * N, 6)
    # ratio noise kept clear of the clip bounds 1 -/+ 0.2 (|ratio - bound| > 1e-3):
    # the clipped objective's derivative jumps there, and a 1-ulp difference in
    # the new log-prob would move a row across (an O(1/M) jump per row)
    d = rng.standard_normal(lp.shape) * 0.1
    near = (np.abs(np.exp(d) - 0.8) < 1e-3) | (np.abs(np.exp(d) - 1.2) < 1e-3)
    d[near] = 0.0
    lpf[rows] = (lp - d).astype(np.float32)
    vf = st["values"].reshape(T * N)
    vf[rows] = V.astype(np.float32)
    rf = st["returns"].reshape(T * N)
    rf[rows] = (V + rng.standard_normal(V.shape)).astype(np.float32)
    return st, rows


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


def _run_grad(gpu, ps, s, seqs, mb, bptt, hpd, stats, step_kernel=0, wgrad_form=0):
    from madrona_learn import _native as nat
    hp = nat.PPOHparams()
    hp.step_kernel = step_kernel
    hp.wgrad_form = wgrad_form
    hp.clip_coef, hp.value_loss_coef = hpd["clip_coef"], hpd["value_loss_coef"]
    for k in range(6):
        hp.entropy_coef[k] = hpd["entropy_coef"]
    hp.normalize_advantages, hp.loss_scale = 1, 1.0
    hp.clip_value_loss = 1 if hpd.get("clip_value_loss") else 0
    hp.huber_value_loss = 1 if hpd.get("huber_value_loss") else 0
    st = torch.tensor([stats[0], 1.0 / np.sqrt(max(stats[1], 1e-5))], dtype=torch.float32,
                      device=gpu)
    M = mb * bptt
    ws = torch.zeros(int(nat.lib().mlearn_ppo_workspace_bytes(ps.desc, M)), dtype=torch.uint8,
                     device=gpu)
    grad = torch.zeros(ps.layout["total"], dtype=torch.float32, device=gpu)
    out = torch.zeros(25, dtype=torch.float32, device=gpu)
    sq = torch.from_numpy(np.asarray(seqs, np.int32)).to(gpu)
    nat.check(nat.lib().mlearn_ppo_minibatch_grad(ps.desc, s.view(bptt), nat.ptr(sq), mb,
                                                  nat.ptr(st), hp, nat.ptr(grad), nat.ptr(out),
                                                  nat.ptr(ws), nat.stream_handle()))
    torch.cuda.synchronize()
    return grad.cpu().numpy(), out.cpu().numpy()


def _check(mode, g, o, loss, gflat, met, M, full_size=False, verr_atol=0.0):
    scale = np.abs(gflat).max()
    if mode == "f32" and full_size:
        # 65,536 rows x 512 ReLUs: tens of pre-activations sit within an f32
        # rounding of 0, where ReLU' jumps (the oracle and the kernel round the
        # LayerNorm in different orders), each moving O(1/M) of gradient; so
        # the elementwise bound is taken relative to the gradient's scale and
        # the bulk is checked in norm
        np.testing.assert_allclose(o[0], loss, rtol=1e-5, atol=1e-7)
        err = np.abs(g - gflat).max() / scale
        assert err < 2e-3, err
        rel = np.linalg.norm(g - gflat) / np.linalg.norm(gflat)
        assert rel < 1e-3, rel
        cos = g @ gflat / (np.linalg.norm(g) * np.linalg.norm(gflat))
        assert cos > 0.99999, cos
        mtol = 1e-5
    elif mode == "f32":
        np.testing.assert_allclose(o[0], loss, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(g, gflat, rtol=1e-3, atol=1e-4 * scale)
        mtol = 1e-5
    else:
        np.testing.assert_allclose(o[0], loss, rtol=2e-2, atol=2e-3)
        err = np.abs(g - gflat).max() / scale
        assert err < 3e-2, err
        cos = g @ gflat / (np.linalg.norm(g) * np.linalg.norm(gflat))
        assert cos > 0.999, cos
        mtol = 2e-2
    np.testing.assert_allclose(o[10], met["Value Loss"].mean(), rtol=mtol)
    np.testing.assert_allclose(o[15], np.abs(met["Value Errors"]).mean(), rtol=mtol,
                               atol=verr_atol)
    np.testing.assert_allclose(o[20], met["Entropy"].mean(), rtol=mtol)
    assert o[14] == M and o[24] == M * 6


def _twohot_value_scale(P, obs):
    """Mean over rows of E_p|b| of the oracle's two-hot bin distributions: the
    scale of mean()."""
    _, _, cache = ref.forward(P, obs, "bf16")
    lg = np.asarray(cache["crit"], np.float64)
    p = np.exp(lg - lg.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    return float((p * np.abs(ref.twohot_bins(lg.shape[-1]))).sum(-1).mean())


HP = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
      "normalize_advantages": True}


@pytest.mark.parametrize("mode,dtype", [("f32", torch.float32), ("bf16", torch.bfloat16)])
def test_minibatch_grad_b1_size(gpu, mode, dtype):
    """One B1 / headline minibatch: 2048 sequences of 32 steps gathered from
    an 8192-env store (65,536 rows, 2048 step-kernel workgroups)."""
    T, N, D, H, L, mb, bptt = 32, 8192, 64, 256, 2, 2048, 32
    ps = make_policy_state(gpu, D, H, L, dtype, seed=21)
    perturb(ps, 22, scale=0.2)
    rng = np.random.default_rng(23)
    seqs = rng.permutation(N)[:mb].astype(np.int32)
    st, rows = _minibatch_store(rng, ps, T, N, D, mode, seqs, bptt)
    s = _device_store(gpu, st, dtype)
    batch = ref.gather_minibatch(st, rows)
    adv = batch["advantages"].astype(np.float64)
    stats = (adv.mean(), adv.var())
    P = ref.unflatten(ps.params.cpu().numpy(), oracle_layout(ps))
    loss, G, met, _ = ref.ppo_loss_grads(P, batch, HP, BUCKETS, mode, adv_stats=stats)
    gflat = ref.flatten(G, oracle_layout(ps))
    g, o = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats)
    _check(mode, g, o, loss, gflat, met, mb * bptt, full_size=True)


def _set_constant_critic(ps, value):
    """Critic column of the head zeroed and its bias set so that every row's
    value is exactly `value` in both dtypes (ties are then exact)."""
    p = ps.params.cpu().numpy()
    o, shp = ps.layout["hw"]
    hw = p[o:o + shp[0] * shp[1]].reshape(shp)
    A = ps.arch.num_logits
    hw[:, A] = 0.0
    o, _ = ps.layout["hb"]
    p[o + A] = value
    ps.params.copy_(torch.from_numpy(p))
    ps.sync_weights()


@pytest.mark.parametrize("mode,dtype", [("f32", torch.float32), ("bf16", torch.bfloat16)])
@pytest.mark.parametrize("clip_vl,huber", [(True, False), (False, True), (True, True)])
@pytest.mark.parametrize("ties", [False, True])
def test_value_loss_variants(gpu, mode, dtype, clip_vl, huber, ties):
    T, N, D, H, L, mb, bptt = 32, 96, 64, 128, 2, 40, 16
    ps = make_policy_state(gpu, D, H, L, dtype, seed=31)
    perturb(ps, 32, scale=0.2)
    hpd = dict(HP, clip_coef=0.25, clip_value_loss=clip_vl, huber_value_loss=huber)
    if ties:
        _set_constant_critic(ps, 0.5)  # V == 0.5 exactly on every row
    rng = np.random.default_rng(33)
    nseq = (T // bptt) * N
    seqs = rng.permutation(nseq)[:mb].astype(np.int32)
    st, rows = _minibatch_store(rng, ps, T, N, D, mode, seqs, bptt)
    if ties:
        # old values on the clip bounds (V == ov -/+ clip), inside, and
        # clipped on either side; returns on the huber kink (|vpred - R| == 1)
        n = len(rows)
        vf = st["values"].reshape(-1)
        vf[rows] = np.array([0.75, 0.25, 0.5, 2.0, -1.0], np.float32)[np.arange(n) % 5]
        rf = st["returns"].reshape(-1)
        rf[rows] = np.array([1.5, -0.5, 0.5, 3.0, -2.5, 0.75, 0.1], np.float32)[np.arange(n) % 7]
    else:
        st["values"].reshape(-1)[rows] += (rng.standard_normal(len(rows)) * 0.3).astype(
            np.float32)
        st["returns"].reshape(-1)[rows] *= 2.0
    s = _device_store(gpu, st, dtype)
    batch = ref.gather_minibatch(st, rows)
    adv = batch["advantages"].astype(np.float64)
    stats = (adv.mean(), adv.var())
    P = ref.unflatten(ps.params.cpu().numpy(), oracle_layout(ps))
    loss, G, met, aux = ref.ppo_loss_grads(P, batch, hpd, BUCKETS, mode, adv_stats=stats)
    if ties:
        assert np.all(aux["value"] == 0.5), "the oracle's values must sit on the ties too"
    gflat = ref.flatten(G, oracle_layout(ps))
    g, o = _run_grad(gpu, ps, s, seqs, mb, bptt, hpd, stats)
    _check(mode, g, o, loss, gflat, met, mb * bptt)
    if ties:
        # the critic bias gradient is the sum of d loss / d V: pins the 0.5 tie weights
        A = ps.arch.num_logits
        ob, _ = ps.layout["hb"]
        np.testing.assert_allclose(g[ob + A], gflat[ob + A], rtol=1e-5 if mode == "f32" else 2e-2,
                                   atol=1e-7)


@pytest.mark.parametrize("mb,bptt", [(2048, 32), (4095, 16), (1024, 32), (1023, 32)])
def test_row_split_step_kernel(gpu, mb, bptt):
    """The row-split step kernel (the bf16 default: W1 held in LDS, one wave
    per 16-row tile, 16x16x32 MFMAs) against the oracle and against the
    feature-split kernel (step_kernel 1) on the same minibatch, in both of
    its shapes: 8 waves x 2 tiles per workgroup at 65,536 rows, 8 x 1 at
    32,768 (a two-rank data-parallel slice); (4095, 16) and (1023, 32) leave
    padding rows.  The two kernels
    sum in different orders (f32 accumulation of the same bf16 products), so
    they agree to the bf16 bound, not bitwise."""
    T, N, D, H, L = 32, 8192, 64, 256, 2
    ps = make_policy_state(gpu, D, H, L, torch.bfloat16, seed=41)
    perturb(ps, 42, scale=0.2)
    rng = np.random.default_rng(43)
    nseq = (T // bptt) * N
    seqs = rng.permutation(nseq)[:mb].astype(np.int32)
    st, rows = _minibatch_store(rng, ps, T, N, D, "bf16", seqs, bptt)
    s = _device_store(gpu, st, torch.bfloat16)
    batch = ref.gather_minibatch(st, rows)
    adv = batch["advantages"].astype(np.float64)
    stats = (adv.mean(), adv.var())
    g2, o2 = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats, step_kernel=2)
    g1, o1 = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats, step_kernel=1)
    g0, o0 = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats)
    assert np.array_equal(g0, g2) and np.array_equal(o0, o2), "auto must pick the row split"
    scale = np.abs(g1).max()
    assert np.abs(g2 - g1).max() / scale < 1e-2
    assert g2 @ g1 / (np.linalg.norm(g2) * np.linalg.norm(g1)) > 0.9999
    np.testing.assert_allclose(o2[[0, 10, 15, 20]], o1[[0, 10, 15, 20]], rtol=2e-3)
    assert o2[14] == mb * bptt and o2[24] == mb * bptt * 6
    P = ref.unflatten(ps.params.cpu().numpy(), oracle_layout(ps))
    loss, G, met, _ = ref.ppo_loss_grads(P, batch, HP, BUCKETS, "bf16", adv_stats=stats)
    _check("bf16", g2, o2, loss, ref.flatten(G, oracle_layout(ps)), met, mb * bptt)


@pytest.mark.parametrize("mb,bptt", [(2048, 32), (1023, 32)])
def test_row_split_step_kernel_twohot(gpu, mb, bptt):
    """The row-split step kernel with the reference's default critic, a
    DreamerV3 two-hot critic of 63 bins (round 6: head width 96, both head
    products streaming the head image from L2, the two-hot cross entropy by
    each row's four lanes) against the oracle and the feature-split kernel on
    the same minibatch (65,536 rows: 8 waves x 2 tiles; 32,736 rows: 8 x 1
    with padding rows)."""
    T, N, D, H, L = 32, 8192, 64, 256, 2
    ps = make_policy_state(gpu, D, H, L, torch.bfloat16, seed=61, critic_bins=63)
    perturb(ps, 62, scale=0.2)
    rng = np.random.default_rng(63)
    nseq = (T // bptt) * N
    seqs = rng.permutation(nseq)[:mb].astype(np.int32)
    st, rows = _minibatch_store(rng, ps, T, N, D, "bf16", seqs, bptt)
    s = _device_store(gpu, st, torch.bfloat16)
    batch = ref.gather_minibatch(st, rows)
    adv = batch["advantages"].astype(np.float64)
    stats = (adv.mean(), adv.var())
    g2, o2 = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats, step_kernel=2)
    g1, o1 = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats, step_kernel=1)
    g0, o0 = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats)
    assert np.array_equal(g0, g2) and np.array_equal(o0, o2), "auto must pick the row split"
    scale = np.abs(g1).max()
    assert np.abs(g2 - g1).max() / scale < 1e-2
    assert g2 @ g1 / (np.linalg.norm(g2) * np.linalg.norm(g1)) > 0.9999
    np.testing.assert_allclose(o2[[0, 10, 20]], o1[[0, 10, 20]], rtol=2e-3)
    assert o2[14] == mb * bptt and o2[24] == mb * bptt * 6
    P = ref.unflatten(ps.params.cpu().numpy(), oracle_layout(ps))
    loss, G, met, _ = ref.ppo_loss_grads(P, batch, HP, BUCKETS, "bf16", adv_stats=stats)
    # 'Value Errors' = mean |mean() - R|: mean() weighs the bins' symexp values
    # (up to 1.2e6) by the bin probabilities, so one bf16 ulp of a bin logit
    # (the kernels and the oracle accumulate the head in different orders)
    # moves a row's mean by p_j |b_j - mean| ulp(l_j), far more than it moves
    # the loss; and the store's returns are the oracle's own means + N(0, 1),
    # so the oracle's metric is E|N(0,1)| = 0.8 while a kernel's adds its ulp
    # noise.  With these perturbed bin weights mean() is ~1.2e5 (E_p|b| ~1.5e5)
    # and the kernels' metric sits ~1.7 (1e-5 of that scale) off the oracle's:
    # both comparisons are held to 1e-4 of the value scale
    verr_atol = 1e-4 * _twohot_value_scale(P, batch["obs"])
    assert abs(o2[15] - o1[15]) <= 2 * verr_atol, (o2[15], o1[15], verr_atol)
    _check("bf16", g2, o2, loss, ref.flatten(G, oracle_layout(ps)), met, mb * bptt,
           verr_atol=verr_atol)


def test_row_split_rejects_ineligible(gpu):
    """step_kernel 2 on a minibatch the row split cannot take is EINVAL."""
    from madrona_learn import _native as nat
    T, N, D, H, L, mb, bptt = 16, 96, 64, 128, 2, 40, 16
    ps = make_policy_state(gpu, D, H, L, torch.bfloat16, seed=51)
    rng = np.random.default_rng(52)
    seqs = rng.permutation(N)[:mb].astype(np.int32)
    st, _ = _minibatch_store(rng, ps, T, N, D, "bf16", seqs, bptt)
    s = _device_store(gpu, st, torch.bfloat16)
    with pytest.raises(RuntimeError, match="step_kernel"):
        _run_grad(gpu, ps, s, seqs, mb, bptt, HP, (0.0, 1.0), step_kernel=2)


@pytest.mark.parametrize("D,H,L,CB,mb,bptt", [
    (64, 256, 2, 1, 2048, 32),   # the headline minibatch (row-split step, 65,536 rows)
    (64, 256, 2, 63, 1023, 32),  # two-hot critic: head width 96, padding rows
    (64, 128, 3, 1, 200, 16),    # feature-split step, 128-column tiles
    (32, 64, 1, 1, 77, 16),      # obs 32 / hidden 64: 64-byte and 128-byte operand rows
])
def test_wgrad_staging_forms_bit_identical(gpu, D, H, L, CB, mb, bptt):
    """mlearn_ppo_hparams.wgrad_form (ABI 22): the LDS-DMA weight-gradient
    pipeline (2, the default) and the register-staged form (1) feed the same
    fragments to the same MFMAs in the same order -- the flat gradient and
    the loss metrics must be bit-identical, and the default must be form 2's."""
    T, N = 32, 8192 if mb >= 1023 else 256
    ps = make_policy_state(gpu, D, H, L, torch.bfloat16, seed=51, critic_bins=CB)
    perturb(ps, 52, scale=0.2)
    rng = np.random.default_rng(53)
    nseq = (T // bptt) * N
    seqs = rng.permutation(nseq)[:mb].astype(np.int32)
    st, rows = _minibatch_store(rng, ps, T, N, D, "bf16", seqs, bptt)
    s = _device_store(gpu, st, torch.bfloat16)
    adv = ref.gather_minibatch(st, rows)["advantages"].astype(np.float64)
    stats = (adv.mean(), adv.var())
    g1, o1 = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats, wgrad_form=1)
    g2, o2 = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats, wgrad_form=2)
    g0, o0 = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats)
    assert np.all(np.isfinite(g2)) and np.abs(g2).max() > 0
    assert np.array_equal(g1, g2), np.abs(g1 - g2).max()
    assert np.array_equal(o1, o2)
    assert np.array_equal(g0, g2) and np.array_equal(o0, o2)
    with pytest.raises(Exception, match="wgrad_form"):
        _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats, wgrad_form=3)
