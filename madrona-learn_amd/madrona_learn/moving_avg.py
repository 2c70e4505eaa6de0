"""EMA estimators (src/madrona_learn/moving_avg.py), on device tensors.

EMANormalizer keeps the reference's functional interface (every method
takes the estimates and returns new ones; moving_avg.py:48-198) with the
statistics on the native kernels: update_input_stats (moving_avg.py:107-130)
and update_estimates (moving_avg.py:132-180) are mlearn_ema_input_stats /
mlearn_ema_update_estimates (csrc/misc.hip; the same arithmetic the rollout
kernel's ObservationsEMANormalizer fold runs, mlearn_obs_norm_update), and
normalize / invert are the reference's elementwise expressions in the
reference's dtypes.  Estimates are a dict of device tensors: the five
[dim] f32 vectors are views of one [5][dim] buffer ('_buf', the layout the
kernels take) and 'N' is a one-element int32 tensor.  The oracle restatement
is oracle/ppo_ref.py ema_*; tests/test_gpu_ema.py ports the reference's
tests/test_ema.py design.
"""

from dataclasses import dataclass

import torch

from .cfg import canonical_dtype

_FIELDS = ("mu", "inv_sigma", "sigma", "mu_biased", "sigma_sq_biased")


def _est_from_buf(buf, N):
    d = {k: buf[i] for i, k in enumerate(_FIELDS)}
    d["_buf"] = buf
    d["N"] = N
    return d


def _f32(x):
    """_convert_nonfloat (moving_avg.py:188-192)."""
    return x if torch.is_floating_point(x) else x.to(torch.float32)


@dataclass(frozen=True)
class EMAEstimate:  # moving_avg.py:7-45
    decay: float
    eps: float = 1e-5

    def init_estimates(self, x):
        dim = x.shape[-1]
        dev = x.device
        return {"mu": torch.zeros(dim, dtype=torch.float32, device=dev),
                "mu_biased": torch.zeros(dim, dtype=torch.float32, device=dev),
                "N": torch.zeros((), dtype=torch.int32, device=dev)}

    def update_estimates(self, est, x):
        """moving_avg.py:20-44: bias-corrected EMA of the mean of x (over all
        of its elements), in f32."""
        x_mean = _f32(x).to(torch.float32).mean()
        one_minus_alpha = torch.tensor(self.decay, dtype=torch.float32, device=x.device)
        alpha = 1 - one_minus_alpha
        new_N = est["N"] + 1
        new_mu_biased = one_minus_alpha * est["mu_biased"] + alpha * x_mean
        bias_correction = -1 / torch.expm1(new_N.to(torch.float32) * torch.log(one_minus_alpha))
        return {"mu": new_mu_biased * bias_correction, "mu_biased": new_mu_biased, "N": new_N}


@dataclass(frozen=True)
class EMANormalizer:  # moving_avg.py:47-196
    decay: float
    norm_dtype: object = None
    inv_dtype: object = None
    eps: float = 1e-5
    disable: bool = False

    def __post_init__(self):
        if self.norm_dtype is not None:
            object.__setattr__(self, "norm_dtype", canonical_dtype(self.norm_dtype))
        if self.inv_dtype is not None:
            object.__setattr__(self, "inv_dtype", canonical_dtype(self.inv_dtype))

    # -- estimates ----------------------------------------------------------
    def init_estimates(self, x):
        """moving_avg.py:56-76: mu 0, sigma 1 (a no-op normaliser)."""
        if self.disable:
            return {}
        dim = x.shape[-1]
        buf = torch.zeros((5, dim), dtype=torch.float32, device=x.device)
        buf[1].fill_(1.0)
        buf[2].fill_(1.0)
        return _est_from_buf(buf, torch.zeros(1, dtype=torch.int32, device=x.device))

    def normalize(self, est, x):
        """moving_avg.py:78-85: (x - mu) * inv_sigma in x's dtype, cast to norm_dtype."""
        if self.disable:
            return x
        x = _f32(x)
        y = (x - est["mu"].to(x.dtype)) * est["inv_sigma"].to(x.dtype)
        return y.to(self.norm_dtype) if self.norm_dtype is not None else y

    def invert(self, est, x):
        """moving_avg.py:87-95: x * sigma + mu in inv_dtype."""
        if self.disable:
            return x
        x = _f32(x)
        dt = self.inv_dtype if self.inv_dtype is not None else x.dtype
        return x.to(dt) * est["sigma"].to(dt) + est["mu"].to(dt)

    # -- statistics ---------------------------------------------------------
    def init_input_stats(self, est):
        """moving_avg.py:97-105: (mean, var) zeros."""
        if self.disable:
            return {}
        return torch.zeros_like(est["mu"]), torch.zeros_like(est["mu"])

    def update_input_stats(self, cur_stats, num_prev_updates, x):
        """moving_avg.py:107-130 on the native kernel: batch mean / population
        variance over every axis but the last, merged into cur_stats with
        n_a = num_prev_updates.  Returns new (mean, var) tensors."""
        if self.disable:
            return {}
        from . import _native as nat
        a_mean, a_var = cur_stats
        x = _f32(x).to(torch.float32)
        dim = x.shape[-1]
        xs = x.reshape(-1, dim).contiguous()
        cur = torch.stack([a_mean.to(torch.float32), a_var.to(torch.float32)]).contiguous()
        out = torch.empty_like(cur)
        nat.check(nat.lib().mlearn_ema_input_stats(nat.ptr(xs), xs.shape[0], dim, nat.ptr(cur),
                                                   int(num_prev_updates), nat.ptr(out),
                                                   nat.stream_handle()), "ema_input_stats")
        return out[0], out[1]

    def update_estimates(self, est, input_stats):
        """moving_avg.py:132-180 (Schubert & Gertz weighted merge + EMA, bias
        correction, rsqrt(max(sigma^2, eps))) on the native kernel; returns
        new estimates (the inputs are not modified)."""
        if self.disable:
            return {}
        from . import _native as nat
        x_mean, x_var = input_stats
        stats = torch.stack([x_mean.to(torch.float32), x_var.to(torch.float32)]).contiguous()
        buf = est["_buf"].clone()
        N = est["N"].clone()
        nat.check(nat.lib().mlearn_ema_update_estimates(
            nat.ptr(stats), buf.shape[1], float(self.decay), float(self.eps), nat.ptr(buf),
            nat.ptr(N), nat.stream_handle()), "ema_update_estimates")
        return _est_from_buf(buf, N)

    def normalize_and_update_estimates(self, est, inputs):
        """moving_avg.py:182-186."""
        if self.disable:
            return inputs
        stats = self.update_input_stats(self.init_input_stats(est), 0, inputs)
        est = self.update_estimates(est, stats)
        return est, self.normalize(est, inputs)
