"""DynamicScale: loss scaling for fp16 compute (TrainConfig.compute_dtype =
fp16).  The reference creates flax.training.dynamic_scale.DynamicScale() with
its defaults when compute_dtype is float16 (train_state.py:402-403), trains
through scaler.value_and_grad and keeps params and optimizer state where the
gradient is not finite (ppo.py:276-291).  flax is a third-party dependency
absent here; this restates its published algorithm (flax 0.8.x
flax/training/dynamic_scale.py): the loss is multiplied by `scale`, the
gradient divided by it in f32, and

    finite     = all(isfinite(grad))
    grow       = fin_steps == growth_interval
    fin_scale  = min(scale * growth_factor, f32 max) if grow and finite else scale
    inf_scale  = max(scale * backoff_factor, minimum_scale)
    scale'     = fin_scale if finite else inf_scale
    fin_steps' = 0 if grow or not finite else fin_steps + 1

State lives on the device (no host synchronisation per minibatch); the skip
itself is the flat optimizer's skip_nonfinite (include/mlearn.h)."""

import numpy as np
import torch


class DynamicScale:
    def __init__(self, device, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 scale=65536.0, minimum_scale=float(np.finfo(np.float32).tiny)):
        self.growth_factor = float(growth_factor)
        self.backoff_factor = float(backoff_factor)
        self.growth_interval = int(growth_interval)
        self.minimum_scale = minimum_scale
        self.scale = torch.full((1,), float(scale), dtype=torch.float32, device=device)
        self.fin_steps = torch.zeros(1, dtype=torch.int32, device=device)

    def scale_loss(self, loss):
        return loss * self.scale[0]

    def unscale_(self, grads):
        grads.div_(self.scale)
        return grads

    def update(self, grads):
        """Advance the scale from this step's (unscaled, reduced) gradient;
        returns the device bool `finite`."""
        finite = torch.isfinite(grads).all()
        grow = self.fin_steps == self.growth_interval
        fmax = torch.tensor(np.finfo(np.float32).max, dtype=torch.float32, device=grads.device)
        up = torch.minimum(self.scale * self.growth_factor, fmax)
        fin_scale = torch.where(grow & finite, up, self.scale)
        inf_scale = self.scale * self.backoff_factor
        if self.minimum_scale is not None:
            inf_scale = torch.clamp(inf_scale, min=self.minimum_scale)
        new_scale = torch.where(finite, fin_scale, inf_scale)
        new_fin = torch.where(grow | ~finite, torch.zeros_like(self.fin_steps), self.fin_steps + 1)
        self.scale.copy_(new_scale)
        self.fin_steps.copy_(new_fin)
        return finite

    def state_dict(self):
        return {"scale": self.scale.cpu(), "fin_steps": self.fin_steps.cpu()}

    def load_state_dict(self, sd):
        self.scale.copy_(sd["scale"])
        self.fin_steps.copy_(sd["fin_steps"])
