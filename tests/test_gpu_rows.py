"""ppo_rows_kernel (csrc/ppo_rows.h): the row-split fused minibatch step for the
headline shape (bf16, MLP[256, 256], head width 32; opt-in MLEARN_ROWS=1),
one wave per 32-row tile and W_1 shared in LDS.

It is pinned two ways:
  * against ppo_step_kernel (MLEARN_ROWS=0, the feature-split kernel every
    other shape runs): the flat gradient must be identical bit for bit (same
    MFMA k-step order per block, LayerNorm sums per block combined in block
    order, head partials in block order; the weight-gradient launch rebuilds
    A_0 = relu(LN_0(Z_0)) with ln_apply's operations), and the loss metrics
    equal within f32 summation order (1e-5 relative);
  * against the oracle (ppo_ref.ppo_loss_grads, bf16 rounding mode) with the
    bf16 tolerances of tests/test_gpu_fullsize.py.
Sizes cover every workgroup width of launch_rows (8 / 4 / 2 / 1 waves), a
ragged last tile (padding rows), and observation widths 32 / 64 / 128."""

import numpy as np
import pytest
import torch

from oracle import ppo_ref as ref
from tests.test_gpu_fullsize import HP, _check, _device_store, _minibatch_store, _run_grad
from tests.test_gpu_policy import BUCKETS, make_policy_state, oracle_layout, perturb

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,N,D,mb,bptt", [
    (32, 8192, 64, 2048, 32),  # headline minibatch: 65,536 rows, 2048 tiles, 8 waves / workgroup
    (32, 4096, 64, 1024, 32),  # 1024 tiles: 4 waves
    (32, 2048, 64, 512, 32),   # 512 tiles: 2 waves
    (32, 96, 32, 37, 16),      # 592 rows -> 640 (ragged tile), 1 wave, D = 32
    (32, 64, 128, 33, 2),      # 66 rows -> 128, D = 128
])
def test_rows_kernel_matches_step_kernel(gpu, monkeypatch, T, N, D, mb, bptt):
    ps = make_policy_state(gpu, D, 256, 2, torch.bfloat16, seed=51)
    perturb(ps, 52, scale=0.2)
    rng = np.random.default_rng(53)
    nseq = (T // bptt) * N
    seqs = rng.permutation(nseq)[:mb].astype(np.int32)
    st, rows = _minibatch_store(rng, ps, T, N, D, "bf16", seqs, bptt)
    s = _device_store(gpu, st, torch.bfloat16)
    batch = ref.gather_minibatch(st, rows)
    adv = batch["advantages"].astype(np.float64)
    stats = (adv.mean(), adv.var())
    monkeypatch.setenv("MLEARN_ROWS", "0")
    g0, o0 = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats)
    monkeypatch.setenv("MLEARN_ROWS", "1")
    g1, o1 = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, stats)
    assert np.all(np.isfinite(g1))
    bad = np.flatnonzero(g0 != g1)
    assert bad.size == 0, (bad.size, bad[:8], g0[bad[:8]], g1[bad[:8]])
    np.testing.assert_allclose(o1, o0, rtol=1e-5, atol=1e-7)
    P = ref.unflatten(ps.params.cpu().numpy(), oracle_layout(ps))
    loss, G, met, _ = ref.ppo_loss_grads(P, batch, HP, BUCKETS, "bf16", adv_stats=stats)
    gflat = ref.flatten(G, oracle_layout(ps))
    _check("bf16", g1, o1, loss, gflat, met, mb * bptt)


def test_rows_kernel_graph_replay_deterministic(gpu, monkeypatch):
    """Two launches (and a HIP-graph replay) of the row-split step give the same bits."""
    from madrona_learn import _native as nat
    monkeypatch.setenv("MLEARN_ROWS", "1")
    T, N, D, mb, bptt = 32, 1024, 64, 256, 32
    ps = make_policy_state(gpu, D, 256, 2, torch.bfloat16, seed=61)
    perturb(ps, 62, scale=0.2)
    rng = np.random.default_rng(63)
    seqs = rng.permutation(N)[:mb].astype(np.int32)
    st, rows = _minibatch_store(rng, ps, T, N, D, "bf16", seqs, bptt)
    s = _device_store(gpu, st, torch.bfloat16)
    a = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, (0.1, 2.0))
    b = _run_grad(gpu, ps, s, seqs, mb, bptt, HP, (0.1, 2.0))
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    hp = nat.PPOHparams()
    hp.clip_coef, hp.value_loss_coef = HP["clip_coef"], HP["value_loss_coef"]
    for k in range(6):
        hp.entropy_coef[k] = HP["entropy_coef"]
    hp.normalize_advantages, hp.loss_scale = 1, 1.0
    st_t = torch.tensor([0.1, 1.0 / np.sqrt(2.0)], dtype=torch.float32, device=gpu)
    M = mb * bptt
    ws = torch.zeros(int(nat.lib().mlearn_ppo_workspace_bytes(ps.desc, M)), dtype=torch.uint8,
                     device=gpu)
    grad = torch.zeros(ps.layout["total"], dtype=torch.float32, device=gpu)
    out = torch.zeros(25, dtype=torch.float32, device=gpu)
    sq = torch.from_numpy(seqs).to(gpu)
    view = s.view(bptt)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        nat.check(nat.lib().mlearn_ppo_minibatch_grad(ps.desc, view, nat.ptr(sq), mb, nat.ptr(st_t),
                                                      hp, nat.ptr(grad), nat.ptr(out), nat.ptr(ws),
                                                      nat.stream_handle()))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        nat.check(nat.lib().mlearn_ppo_minibatch_grad(ps.desc, view, nat.ptr(sq), mb, nat.ptr(st_t),
                                                      hp, nat.ptr(grad), nat.ptr(out), nat.ptr(ws),
                                                      nat.stream_handle()))
    grad.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(grad.cpu().numpy(), a[0])
