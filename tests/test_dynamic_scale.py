"""DynamicScale's scale / fin_steps rule (madrona_learn/dynamic_scale.py,
the fp16 torch path) against oracle/dynamic_scale_ref.py (flax 0.8.x's
published rule, ppo.py:276-291 / train_state.py:402-403), on CPU tensors:
growth at the interval, backoff on a non-finite gradient, the minimum-scale
floor and the f32-max cap."""

import numpy as np
import torch

from oracle import dynamic_scale_ref as ref


def _run(seq, **kw):
    from madrona_learn.dynamic_scale import DynamicScale
    sc = DynamicScale(torch.device("cpu"), **kw)
    want_s, want_f = float(sc.scale.item()), 0
    rule = {k: v for k, v in kw.items() if k != "scale"}
    for finite in seq:
        g = torch.ones(7) if finite else torch.tensor([1.0, float("inf"), 2.0])
        got = bool(sc.update(g))
        assert got == finite
        want_s, want_f = ref.step(want_s, want_f, finite, **rule)
        assert float(sc.scale.item()) == want_s and int(sc.fin_steps.item()) == want_f
    return float(sc.scale.item()), int(sc.fin_steps.item())


def test_defaults_growth_and_backoff():
    s, f = _run([True] * 5 + [False] + [True] * 3)
    assert s == 65536.0 * 0.5 and f == 3


def test_growth_interval():
    s, f = _run([True] * 7, growth_interval=3)  # grows when fin_steps == 3, then restarts
    assert s == 65536.0 * 2 and f == 3


def test_nan_and_floor_and_cap():
    _run([False] * 200, growth_interval=3)                        # floors at f32 tiny
    s, _ = _run([True] * 40, growth_interval=0, scale=2.0 ** 120)  # capped at f32 max
    assert s == float(np.finfo(np.float32).max)


def test_scale_and_unscale_roundtrip():
    from madrona_learn.dynamic_scale import DynamicScale
    sc = DynamicScale(torch.device("cpu"))
    g = torch.tensor([3.0, -1.5])
    assert torch.equal(sc.unscale_(g * 65536.0), g)
    assert float(sc.scale_loss(torch.tensor(2.0))) == 131072.0
