"""The optimizer chain as one launch (csrc/optim.hip optim_fused_kernel,
mlearn_optim_state.launch_form, ABI 21) against the split launches it
replaces: clip_by_global_norm + Adam (ppo.py:84-90, 283-286), the weight-norm
and LayerNorm projections (ppo.py:303-338) and the compute-image refresh.
Bit-identical by construction (the fused launch replays the split kernels'
summation orders), so every comparison here is torch.equal: master
parameters, Adam moments, the step counter and every compute image, over
several steps (one with a clipped norm), with the norm partials taken from
the gradient reduction (world 1) or formed in the launch (the all-reduced
gradient, world > 1), on MLP and LSTM layouts.  The oracle comparisons of
the optimizer (tests/test_gpu_policy.py, tests/test_gpu_lstm.py) and of
every full update run on the split launches, the library's default (the
fused launch measured no faster)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

IMAGES = ("head_t", "head", "head_bias", "lstm_wi_perm", "lstm_wi_nat", "lstm_wh_nat",
          "lstm_w_bwd", "head_t_nat")


def _images(ps):
    out = []
    for name in ("w_t", "w"):
        for t in getattr(ps, name, []) or []:
            if isinstance(t, torch.Tensor):
                out.append(t)
    for name in IMAGES:
        t = getattr(ps, name, None)
        if isinstance(t, torch.Tensor):
            out.append(t)
    return out


def _train_state(ps, form, partials):
    from madrona_learn import _native as nat
    from madrona_learn.ppo import PPOHyperParams
    from madrona_learn.train_state import PolicyTrainState
    hp = PPOHyperParams(lr=3e-4, gamma=0.99, gae_lambda=0.95, normalize_values=False,
                        value_normalizer_decay=0.0, max_advantage_est_decay=0.0, clip_coef=0.2,
                        value_loss_coef=0.5, entropy_coef=0.01, max_grad_norm=0.5)
    ts = PolicyTrainState(None, hp, ps, (1, 2))
    ts.optim_desc.launch_form = form
    if partials is not None:
        ts.optim_desc.grad_sumsq_part = partials.data_ptr()
        ts.optim_desc.grad_sumsq_nparts = partials.numel()
    _ = nat
    return ts


@pytest.mark.parametrize("kind,dtype,D,H,L,CB,with_partials", [
    ("mlp", torch.bfloat16, 64, 256, 2, 1, True),    # the headline policy at world 1
    ("mlp", torch.bfloat16, 64, 256, 2, 1, False),   # ... at world > 1 (norm in the launch)
    ("mlp", torch.float32, 32, 64, 2, 63, True),
    ("mlp", torch.float32, 48, 128, 3, 1, False),
    ("mlp", torch.bfloat16, 256, 256, 4, 63, True),  # 3 parameters per thread (PRE 8)
    ("lstm", torch.bfloat16, 64, 256, 2, 1, True),   # config L's layout (5 per thread)
    ("lstm", torch.float32, 64, 128, 2, 1, False),
])
def test_fused_optimizer_bit_identical(gpu, kind, dtype, D, H, L, CB, with_partials):
    from madrona_learn import _native as nat
    if kind == "mlp":
        from tests.test_gpu_policy import make_policy_state, perturb
    else:
        from tests.test_gpu_lstm import make_policy_state, perturb
    ps = [make_policy_state(gpu, D, H, L, dtype, seed=4, critic_bins=CB) for _ in range(2)]
    for p in ps:
        perturb(p, 5)
    assert torch.equal(ps[0].params, ps[1].params)
    n = ps[0].layout["total"]
    parts = None
    if with_partials:
        parts = torch.zeros(int(nat.lib().mlearn_grad_sumsq_parts(n)), dtype=torch.float64,
                            device=gpu)
    ts = [_train_state(ps[0], 1, parts), _train_state(ps[1], 2, parts)]
    rng = np.random.default_rng(6)
    for step in range(4):
        g = torch.from_numpy((rng.standard_normal(n) * (0.01 if step != 1 else 1.0))
                             .astype(np.float32)).to(gpu)
        if parts is not None:  # per-64-parameter partials of g^2, as the gradient reduction
            gp = torch.nn.functional.pad(g.double(), (0, parts.numel() * 64 - n))
            parts.copy_((gp * gp).view(-1, 64).sum(1))
        for t, p in zip(ts, ps):
            t.grads.copy_(g)
            t.optimizer_step(p)
        torch.cuda.synchronize()
        for a, b, what in ((ps[0].params, ps[1].params, "params"),
                           (ts[0].adam_m, ts[1].adam_m, "m"), (ts[0].adam_v, ts[1].adam_v, "v"),
                           (ts[0].step, ts[1].step, "step")):
            assert torch.equal(a, b), (what, step)
        for k, (a, b) in enumerate(zip(_images(ps[0]), _images(ps[1]))):
            assert torch.equal(a, b), ("image", k, step)
    assert int(ts[1].step.item()) == 4
    # the barrier words: no poll ran out (the fail word stays 0)
    ws = ts[1].optim_ws.view(torch.int64)
    assert int(ws[-8].item()) == 0
    assert not torch.equal(ps[1].params, make_policy_state(gpu, D, H, L, dtype, seed=4,
                                                           critic_bins=CB).params)


def test_fused_launch_form_rejects_bad_value(gpu):
    from madrona_learn import _native as nat
    from tests.test_gpu_policy import make_policy_state
    ps = make_policy_state(gpu, 64, 64, 1, torch.float32)
    ts = _train_state(ps, 3, None)
    with pytest.raises(RuntimeError):
        ts.optimizer_step(ps)
    _ = nat
