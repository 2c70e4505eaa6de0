"""EMANormalizer on the native kernels (madrona_learn/moving_avg.py,
mlearn_ema_input_stats / mlearn_ema_update_estimates) with the design of the
reference's tests/test_ema.py: 100 batches of 1024 x 2 values with extreme
means (uniform [-5, 95)) and standard deviations (uniform [2, 2002)), the
last batch at mean -20 / std 0.01, each batch fed as 32 sub-chunks through
update_input_stats and then one update_estimates, decay 0.999.

The reference only prints its three comparisons; the bounds here are ours:
  * against the oracle restatement (oracle/ppo_ref.py ema_*, the same
    per-sub-chunk sequence with f64 batch moments rounded to f32): mu and
    sigma within 2e-6 x the final sigma (f32 Welford vs f64 moments per
    sub-chunk, 3200 merges);
  * against the naive float64 bias-corrected EMA of E[x] and E[x^2] of every
    batch (the reference's check): mu within 1e-5 x sigma, sigma within 1e-5
    relative — the Schubert-Gertz merge is the same estimator, so only f32
    rounding separates them."""

import numpy as np
import pytest
import torch

from oracle import ppo_ref as ref

pytestmark = pytest.mark.gpu

DECAY, BATCH, SUB, ITERS, DIMS = 0.999, 1024, 32, 100, 2


def _values():
    rng = np.random.default_rng(5)
    means = rng.random((ITERS, DIMS)) * 100 - 5
    stds = rng.random((ITERS, DIMS)) * 2000 + 2
    means[-1] = -20
    stds[-1] = 0.01
    return (rng.standard_normal((ITERS, BATCH, DIMS)) * stds[:, None] + means[:, None]).astype(
        np.float32)


def test_ema_normalizer_matches_naive_ema_and_oracle(gpu):
    from madrona_learn.moving_avg import EMANormalizer
    vals = _values()
    norm = EMANormalizer(decay=DECAY, norm_dtype=torch.float32, inv_dtype=torch.float32)
    xs = torch.from_numpy(vals).to(gpu)
    est = norm.init_estimates(xs[0])
    oest = ref.ema_init(DIMS)
    naive_x = np.zeros(DIMS)
    naive_xx = np.zeros(DIMS)
    for i in range(ITERS):
        stats = norm.init_input_stats(est)
        ost = (np.zeros(DIMS, np.float32), np.zeros(DIMS, np.float32))
        chunks = xs[i].reshape(SUB, BATCH // SUB, DIMS)
        for j in range(SUB):
            stats = norm.update_input_stats(stats, j, chunks[j])
            ost = ref.ema_update_input_stats(ost, j, vals[i].reshape(SUB, -1, DIMS)[j])
        est = norm.update_estimates(est, stats)
        oest = ref.ema_update_estimates(oest, ost, DECAY, 1e-5)
        v = vals[i].astype(np.float64)
        naive_x = DECAY * naive_x + (1 - DECAY) * v.mean(0)
        naive_xx = DECAY * naive_xx + (1 - DECAY) * (v * v).mean(0)
    bc = -np.expm1(ITERS * np.log(DECAY))
    naive_mu = naive_x / bc
    naive_sigma = np.sqrt(naive_xx / bc - naive_mu * naive_mu)
    mu = est["mu"].cpu().numpy().astype(np.float64)
    sigma = est["sigma"].cpu().numpy().astype(np.float64)
    assert int(est["N"].item()) == ITERS
    # the oracle restatement
    np.testing.assert_allclose(mu, oest["mu"], atol=2e-6 * sigma.max())
    np.testing.assert_allclose(sigma, oest["sigma"], rtol=2e-6)
    np.testing.assert_allclose(est["inv_sigma"].cpu().numpy(), oest["inv_sigma"], rtol=2e-6)
    # the reference test's naive float64 EMA
    np.testing.assert_allclose(mu, naive_mu, atol=1e-5 * naive_sigma.max())
    np.testing.assert_allclose(sigma, naive_sigma, rtol=1e-5)
    # normalize / invert round trip and the functional interface (est unchanged)
    x = xs[-1]
    y = norm.normalize(est, x)
    back = norm.invert(est, y)
    np.testing.assert_allclose(back.cpu().numpy(), x.cpu().numpy(), rtol=1e-5,
                               atol=1e-4 * sigma.max())
    e2, _ = norm.normalize_and_update_estimates(est, x)
    assert int(e2["N"].item()) == ITERS + 1 and int(est["N"].item()) == ITERS


def test_ema_estimate_matches_closed_form(gpu):
    """EMAEstimate (moving_avg.py:7-45): bias-corrected EMA of the batch mean."""
    from madrona_learn.moving_avg import EMAEstimate
    rng = np.random.default_rng(3)
    e = EMAEstimate(decay=0.99)
    xs = [rng.standard_normal((64, 3)).astype(np.float32) * 3 + k for k in range(20)]
    est = e.init_estimates(torch.from_numpy(xs[0]).to(gpu))
    mb = np.float32(0)
    for n, x in enumerate(xs, 1):
        est = e.update_estimates(est, torch.from_numpy(x).to(gpu))
        mb = np.float32(0.99) * mb + np.float32(0.01) * np.float32(x.mean(dtype=np.float64))
        want = mb / -np.expm1(np.float64(n) * np.log(np.float32(0.99)))
        np.testing.assert_allclose(est["mu"].cpu().numpy(), np.full(3, want), rtol=1e-5)
    assert int(est["N"].item()) == 20
