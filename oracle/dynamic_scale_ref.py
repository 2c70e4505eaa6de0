"""TEST INFRASTRUCTURE ONLY (tests/ may import it; the product never does).

flax.training.dynamic_scale.DynamicScale's scale / fin_steps rule (flax
0.8.x, flax/training/dynamic_scale.py; a third-party dependency of the
reference, absent here), restated in plain Python floats with f32 rounding
of the products, as the reference builds it for fp16 compute
(/root/reference/src/madrona_learn/train_state.py:402-403) and applies it in
ppo.py:276-291.  Parity unpinned against flax itself (not importable here);
the rule is the published one."""

import numpy as np


def step(scale, fin_steps, finite, growth_factor=2.0, backoff_factor=0.5,
         growth_interval=2000, minimum_scale=float(np.finfo(np.float32).tiny)):
    f32 = np.float32
    grow = fin_steps == growth_interval
    if grow and finite:
        fin_scale = min(f32(scale) * f32(growth_factor), np.finfo(np.float32).max)
    else:
        fin_scale = f32(scale)
    inf_scale = f32(scale) * f32(backoff_factor)
    if minimum_scale is not None:
        inf_scale = max(inf_scale, f32(minimum_scale))
    new_scale = fin_scale if finite else inf_scale
    new_fin = 0 if (grow or not finite) else fin_steps + 1
    return float(f32(new_scale)), int(new_fin)
