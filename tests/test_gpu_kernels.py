"""GPU parity of the individual HIP kernels against the CPU oracle.

Integer / byte work (Philox, sampling, permutation, env, dones) is checked
bit-exact; fp32 recurrences with a fixed operation order (GAE, returns) are
checked bit-exact against the oracle's float32 restatement; reductions and
transcendental math within stated tolerances.
"""

import numpy as np
import pytest
import torch

from oracle import native as onat
from oracle import ppo_ref as ref

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]  # tests/ac_test.py:206-209


def _nat():
    from madrona_learn import _native as nat
    return nat


def test_philox_bitexact(gpu):
    nat = _nat()
    rng = np.random.default_rng(0)
    ctr = rng.integers(0, 2**32, size=(4096, 4), dtype=np.uint64).astype(np.uint32)
    ctr[0] = 0
    ctr[1] = 0xFFFFFFFF
    exp = onat.philox(ctr, 0x12345678, 0x9ABCDEF0)
    c = torch.from_numpy(ctr.view(np.int32)).to(gpu)
    out = torch.empty_like(c)
    nat.check(nat.lib().mlearn_philox4x32(nat.ptr(c), 0x12345678, 0x9ABCDEF0, nat.ptr(out),
                                          4096, nat.stream_handle()))
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("T,N", [(32, 64), (32, 8192), (7, 1001), (1, 4), (32, 0)])
def test_gae_bitexact(gpu, T, N):
    from madrona_learn.algo_common import compute_advantages

    class C:
        steps_per_update = T
        gamma = 0.99
        gae_lambda = 0.95

    rng = np.random.default_rng(T * 1000 + N)
    r = rng.standard_normal((T, N)).astype(np.float32)
    v = rng.standard_normal((T, N)).astype(np.float32)
    d = rng.random((T, N)) < 0.1
    b = rng.standard_normal(N).astype(np.float32)
    if N == 0:
        return
    adv, ret = compute_advantages(C, torch.from_numpy(r).to(gpu), torch.from_numpy(v).to(gpu),
                                  torch.from_numpy(d).to(gpu), torch.from_numpy(b).to(gpu))
    ea, er = ref.gae_f32(r, v, d, b, 0.99, 0.95)
    assert np.array_equal(adv.cpu().numpy(), ea)
    assert np.array_equal(ret.cpu().numpy(), er)
    # and within 1e-5 rel of the fp64 restatement
    fa, _ = ref.gae(r, v, d, b, 0.99, 0.95)
    np.testing.assert_allclose(adv.cpu().numpy(), fa, rtol=1e-5, atol=1e-5)
    # returns not materialised (the product path): identical advantages, and
    # the consumers' advantages + values equal the materialised returns bit for bit
    adv2, none = compute_advantages(C, torch.from_numpy(r).to(gpu), torch.from_numpy(v).to(gpu),
                                    torch.from_numpy(d).to(gpu), torch.from_numpy(b).to(gpu),
                                    out_ret=False)
    assert none is None
    assert np.array_equal(adv2.cpu().numpy(), ea)
    assert np.array_equal((adv2 + torch.from_numpy(v).to(gpu)).cpu().numpy(), er)


@pytest.mark.parametrize("gamma,lam", [(0.998, 0.95), (0.9, 0.8), (0.9999, 0.97), (0.95, 1.0)])
def test_gae_gamma_lambda_constant(gpu, gamma, lam):
    """The gamma * lambda constant is the reference's single rounding
    (algo_common.py:120 multiplies the Python floats, rollouts.py:406): at
    0.998 / 0.95 it differs by one ulp from f32(gamma) * f32(lambda), and the
    advantages must follow the reference's, bit for bit."""
    from madrona_learn.algo_common import compute_advantages

    class C:
        steps_per_update = 32
        gae_lambda = lam

    C.gamma = gamma
    rng = np.random.default_rng(17)
    T, N = 32, 4096
    r = rng.standard_normal((T, N)).astype(np.float32)
    v = rng.standard_normal((T, N)).astype(np.float32)
    d = rng.random((T, N)) < 0.03
    b = rng.standard_normal(N).astype(np.float32)
    adv, ret = compute_advantages(C, torch.from_numpy(r).to(gpu), torch.from_numpy(v).to(gpu),
                                  torch.from_numpy(d).to(gpu), torch.from_numpy(b).to(gpu))
    ea, er = ref.gae_f32(r, v, d, b, gamma, lam)
    assert np.array_equal(adv.cpu().numpy(), ea)
    assert np.array_equal(ret.cpu().numpy(), er)


def test_returns_bitexact(gpu):
    from madrona_learn.algo_common import compute_returns

    class C:
        steps_per_update = 16
        gamma = 0.97

    rng = np.random.default_rng(3)
    r = rng.standard_normal((16, 300)).astype(np.float32)
    d = rng.random((16, 300)) < 0.2
    b = rng.standard_normal(300).astype(np.float32)
    out = compute_returns(C, torch.from_numpy(r).to(gpu), torch.from_numpy(d).to(gpu),
                          torch.from_numpy(b).to(gpu))
    assert np.array_equal(out.cpu().numpy(), ref.discounted_returns_f32(r, d, b, 0.97))


def test_zscore(gpu):
    from madrona_learn.algo_common import zscore_data
    rng = np.random.default_rng(4)
    x = (rng.standard_normal(100003) * 3 + 7).astype(np.float32)
    got = zscore_data(torch.from_numpy(x).to(gpu)).cpu().numpy()
    exp, _, _ = ref.zscore(x)
    np.testing.assert_allclose(got, exp, rtol=1e-5, atol=1e-5)
    # constant input: variance clamps at 1e-5 (algo_common.py:140)
    c = np.full(1000, 2.5, np.float32)
    got = zscore_data(torch.from_numpy(c).to(gpu)).cpu().numpy()
    assert np.all(got == 0)


@pytest.mark.parametrize("sample", [1, 0])
def test_discrete_sample_bitexact(gpu, sample):
    from madrona_learn.dists import DiscreteActionDistributions, PhiloxKey
    rng = np.random.default_rng(5)
    N = 5000
    lg = (rng.standard_normal((N, 26)) * 2).astype(np.float32)
    lg[:10] = 0.0  # exact ties: first-index argmax when not sampling
    dist = DiscreteActionDistributions(BUCKETS, torch.from_numpy(lg).to(gpu))
    key = PhiloxKey(77, 99, step=12345678901, env_offset=17)
    if sample:
        acts, logp = dist.sample(key)
    else:
        acts, logp = dist.best(), None
    exp = onat.sample(lg, BUCKETS, 77, 99, 12345678901, 17, sample=bool(sample))
    assert np.array_equal(acts.cpu().numpy(), exp)
    if sample:
        elogp, _ = ref.action_stats(lg, BUCKETS, exp)
        np.testing.assert_allclose(logp.cpu().numpy(), elogp, rtol=1e-5, atol=2e-6)


def test_sampling_distribution(gpu):
    """Gumbel-max with the deterministic log matches softmax frequencies."""
    from madrona_learn.dists import DiscreteActionDistributions, PhiloxKey
    p = np.array([0.1, 0.2, 0.3, 0.4])
    N = 200000
    lg = np.tile(np.log(p).astype(np.float32), (N, 1))
    dist = DiscreteActionDistributions([4], torch.from_numpy(lg).to(gpu))
    acts, _ = dist.sample(PhiloxKey(1, 2, 3))
    freq = np.bincount(acts.cpu().numpy()[:, 0], minlength=4) / N
    np.testing.assert_allclose(freq, p, atol=4e-3)


def test_action_stats(gpu):
    from madrona_learn.dists import DiscreteActionDistributions
    rng = np.random.default_rng(6)
    lg = (rng.standard_normal((777, 26)) * 3).astype(np.float32)
    acts = np.stack([rng.integers(0, b, 777) for b in BUCKETS], -1).astype(np.int32)
    dist = DiscreteActionDistributions(BUCKETS, torch.from_numpy(lg).to(gpu))
    lp, ent = dist.action_stats(torch.from_numpy(acts).to(gpu))
    elp, eent = ref.action_stats(lg, BUCKETS, acts)
    np.testing.assert_allclose(lp.cpu().numpy(), elp, rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(ent.cpu().numpy(), eent, rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("n", [1, 16, 1000, 8192, 16384, 100003])
def test_minibatch_perm_bitexact(gpu, n):
    nat = _nat()
    out = torch.empty(n, dtype=torch.int32, device=gpu)
    ctr = torch.tensor([5, 0, 0, 0, 0, 0, 0, 0], dtype=torch.int64, device=gpu)
    nat.check(nat.lib().mlearn_minibatch_perm(11, 22, nat.ptr(ctr), 2, 3, n, nat.ptr(out),
                                              nat.stream_handle()))
    got = out.cpu().numpy()
    assert np.array_equal(np.sort(got), np.arange(n))
    assert np.array_equal(got, ref.epoch_permutation(11, 22, 7, 3, n))


@pytest.mark.parametrize("D", [64, 48, 18, 1100])
def test_env_bitexact(gpu, D):
    """Q = ceil(D / 4) quads per env: 16 (16 envs per workgroup), 12 (21, not
    dividing 256), 5 (a ragged last quad) and 275 (the one-env-per-workgroup
    kernel for D > 256)."""
    from madrona_learn.envs import DummyVecEnv
    N = 300
    env = DummyVecEnv(N, D, 6, seed=3, env_offset=1000, device=gpu)
    oenv = onat.Env(N, D, env.k0, env.k1, 1000)
    o = env.init()["obs"].cpu().numpy()
    assert np.array_equal(o, oenv.reset())
    rng = np.random.default_rng(7)
    for t in range(40):
        a = np.stack([rng.integers(0, b, N) for b in BUCKETS], -1).astype(np.int32)
        out = env.step({"actions": torch.from_numpy(a).to(gpu)})
        eo, er, ed = oenv.step(a)
        assert np.array_equal(out["obs"].cpu().numpy(), eo)
        assert np.array_equal(out["rewards"].cpu().numpy().reshape(-1), er)
        assert np.array_equal(out["dones"].cpu().numpy().reshape(-1).astype(np.uint8), ed)
    assert np.array_equal(env.state.cpu().numpy(), oenv.state)


def test_metrics(gpu):
    nat = _nat()
    rng = np.random.default_rng(8)
    xs = [rng.standard_normal(n).astype(np.float32) * 5 + 1 for n in (1, 1000, 262144)]
    ts = [torch.from_numpy(x).to(gpu) for x in xs]
    # a [32][48] window (columns 16..63) of a [32][80] array: one policy's env
    # columns of a population store
    big = rng.standard_normal((32, 80)).astype(np.float32)
    tb = torch.from_numpy(big).to(gpu)
    jobs = (nat.MetricJob * 4)()
    for i, t in enumerate(ts):
        jobs[i].x = t.data_ptr()
        jobs[i].n = t.numel()
        jobs[i].abs_value = 1 if i == 2 else 0
    jobs[3].x = tb.data_ptr() + 16 * 4
    jobs[3].n = 32 * 48
    jobs[3].cols = 48
    jobs[3].ld = 80
    out = torch.zeros((4, 5), device=gpu)
    ws = torch.zeros(int(nat.lib().mlearn_metrics_workspace_bytes(4)), dtype=torch.uint8,
                     device=gpu)
    nat.check(nat.lib().mlearn_metrics_f32(jobs, 4, nat.ptr(out), nat.ptr(ws),
                                           nat.stream_handle()))
    got = out.cpu().numpy()
    for i, x in enumerate(xs + [big[:, 16:64].reshape(-1)]):
        x = np.abs(x) if i == 2 else x
        x = x.astype(np.float64)
        np.testing.assert_allclose(got[i, 0], x.mean(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(got[i, 1], ((x - x.mean()) ** 2).sum(), rtol=1e-4, atol=1e-5)
        assert got[i, 2] == np.float32(x.min()) and got[i, 3] == np.float32(x.max())
        assert got[i, 4] == x.size


def test_errors_are_reported(gpu):
    nat = _nat()
    rc = nat.lib().mlearn_gae_f32(None, None, None, None, None, None, 4, 8, 0.9, 0.9,
                                  nat.stream_handle())
    assert rc == -1
    assert b"null" in nat.lib().mlearn_last_error()


def test_lstm_activation_accuracy(gpu):
    """The gate activations on v_exp_f32 / v_rcp_f32 (rowtile.h sigmoidf,
    tanh_fast) against libm over a dense sweep of [-20, 20], both sides of
    the |x| = 1/8 series cutover included: absolute error <= 2e-7 (below
    the bf16 rounding of every stored gate, 2^-9 relative) and relative
    error <= 4e-6 where |f(x)| >= 1e-3."""
    from madrona_learn import _native as nat
    xs = np.concatenate([np.linspace(-20, 20, 400001), np.linspace(-0.13, 0.13, 20001),
                         np.nextafter(np.float32([0.125, -0.125]), 0),
                         np.float32([0.125, -0.125, 0.0, 1e-30, -1e-30, 88.0, -88.0])])
    x = torch.tensor(xs, dtype=torch.float32, device=gpu)
    sg, th = torch.empty_like(x), torch.empty_like(x)
    nat.check(nat.lib().mlearn_lstm_activations_f32(nat.ptr(x), x.numel(), nat.ptr(sg), nat.ptr(th),
                                                   nat.stream_handle()), "activations")
    xd = x.cpu().double().numpy()
    ref_s = 1.0 / (1.0 + np.exp(-xd))
    ref_t = np.tanh(xd)
    for got, ref in ((sg.cpu().double().numpy(), ref_s), (th.cpu().double().numpy(), ref_t)):
        err = np.abs(got - ref)
        assert err.max() <= 2e-7, err.max()
        big = np.abs(ref) >= 1e-3
        assert (err[big] / np.abs(ref[big])).max() <= 4e-6
        assert np.all(np.isfinite(got))
    assert np.all(np.abs(th.cpu().numpy()) <= 1.0) and np.all((sg.cpu().numpy() >= 0) & (sg.cpu().numpy() <= 1))
