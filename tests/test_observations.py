"""ObservationsPreprocess hooks (the torch path's calls; the statistics run
through the HIP EMA kernels, so on the GPU) (observations.py:13-132): a bare
observation tensor and a dict of named observations run through
init_state -> init_obs_stats -> update_obs_stats x T -> update_state ->
preprocess and match the oracle's EMA restatement (ppo_ref.ema_*); a name in
skip_normalization keeps no state and is only passed through."""

import numpy as np
import torch

import pytest

from oracle import ppo_ref as ref

pytestmark = pytest.mark.gpu


def _run(pre, obs_seq):
    st = pre.init_state(obs_seq[0])
    stats = pre.init_obs_stats(st)
    for t, ob in enumerate(obs_seq):
        stats = pre.update_obs_stats(st, stats, t, ob)
    st = pre.update_state(st, stats)
    return st, pre.preprocess(st, obs_seq[-1])


def _oracle(xs, decay, eps):
    est = ref.ema_init(xs[0].shape[-1])
    stats = (np.zeros(xs[0].shape[-1], np.float32), np.zeros(xs[0].shape[-1], np.float32))
    for t, x in enumerate(xs):
        stats = ref.ema_update_input_stats(stats, t, x)
    est = ref.ema_update_estimates(est, stats, decay, eps)
    return est, ref.ema_normalize(est, xs[-1], "f32")


def test_bare_and_named_observations(gpu):
    import madrona_learn as ml
    rng = np.random.default_rng(3)
    decay, eps = 0.99, 1e-5
    xs = [(rng.standard_normal((16, 8)) * 3 + 1).astype(np.float32) for _ in range(4)]
    ys = [rng.standard_normal((16, 5)).astype(np.float32) for _ in range(4)]
    est, want = _oracle(xs, decay, eps)

    pre = ml.ObservationsEMANormalizer.create(decay, torch.float32, eps=eps)
    st, out = _run(pre, [torch.from_numpy(x).to(gpu) for x in xs])
    for k in ("mu", "sigma", "inv_sigma"):
        np.testing.assert_allclose(st[k].cpu().numpy(), est[k], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out.cpu().numpy(), want, rtol=1e-5, atol=1e-5)

    pre = ml.ObservationsEMANormalizer.create(decay, torch.float32, eps=eps,
                                              skip_normalization={"b"})
    seq = [{"a": torch.from_numpy(x).to(gpu), "b": torch.from_numpy(y).to(gpu)} for x, y in zip(xs, ys)]
    st, out = _run(pre, seq)
    assert set(st) == {"a", "b"} and st["b"] is None
    for k in ("mu", "sigma"):
        np.testing.assert_allclose(st["a"][k].cpu().numpy(), est[k], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out["a"].cpu().numpy(), want, rtol=1e-5, atol=1e-5)
    assert torch.equal(out["b"], seq[-1]["b"])


def test_stateless_preprocess_passes_through(gpu):
    import madrona_learn as ml
    x = torch.randn(4, 3, device=gpu)
    pre = ml.ObservationsPreprocessNoop.create()
    assert torch.equal(pre.preprocess(None, x), x)
    d = pre.preprocess(None, {"p": x, "q": x * 2})
    assert torch.equal(d["q"], x * 2)
