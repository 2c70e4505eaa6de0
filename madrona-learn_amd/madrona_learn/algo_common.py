"""Shared algorithm pieces (mirrors src/madrona_learn/algo_common.py).

``compute_advantages`` / ``compute_returns`` / ``zscore_data`` take torch
device tensors in the reference's [C, T/C, P, B, 1] store layout (any shape
whose leading dims flatten to [T, N]) and run the HIP kernels.
"""

from dataclasses import dataclass

import torch

from . import _native as nat


@dataclass(frozen=True)
class HyperParams:  # algo_common.py:15-21
    lr: float
    gamma: float
    gae_lambda: float
    normalize_values: bool
    value_normalizer_decay: float
    max_advantage_est_decay: float


class AlgoBase:  # algo_common.py:24-42
    def init_hyperparams(self, cfg):
        raise NotImplementedError

    def make_optimizer(self, hyper_params):
        raise NotImplementedError

    def update(self, *args, **kwargs):
        raise NotImplementedError

    def add_metrics(self, cfg, metrics):
        raise NotImplementedError


def _tn(x, T, N, dtype):
    x = x.reshape(T, N)
    if x.dtype != dtype:
        x = x.to(dtype)
    return x.contiguous()


def _gamma_lambda(cfg):
    """``cfg.gamma * cfg.gae_lambda`` as algo_common.py:120 forms it: a product
    of two Python floats (double precision), rounded to f32 once where it
    meets the f32 advantages (JAX weak typing) -- here by the ctypes float
    argument of mlearn_gae_f32."""
    return float(cfg.gamma) * float(cfg.gae_lambda)


def compute_advantages(cfg, rewards, values, dones, bootstrap_values, out_adv=None,
                       out_ret=None, value_norm=None, norm_cols=0):
    """algo_common.py:84-130 (+ returns = adv + values, rollouts.py:761-769).
    ``value_norm`` ([P, 8] f32 estimates, normalize_values): values and
    bootstrap are normalised critic outputs, inverted first (rollouts.py:726-738);
    column n uses estimate n // norm_cols.

    Returns (advantages, returns), both [T, N] f32; ``out_ret=False``: the
    returns are not materialised (the GAE writes 4 B per element instead of
    8; consumers form advantages + values) and None is returned for them."""
    T = cfg.steps_per_update
    N = rewards.numel() // T
    r = _tn(rewards, T, N, torch.float32)
    v = _tn(values, T, N, torch.float32)
    d = _tn(dones, T, N, torch.uint8) if dones.dtype != torch.bool else \
        dones.reshape(T, N).contiguous().view(torch.uint8)
    b = bootstrap_values.reshape(N).to(torch.float32).contiguous()
    adv = out_adv if out_adv is not None else torch.empty((T, N), dtype=torch.float32,
                                                          device=r.device)
    if out_ret is False:
        if value_norm is not None:
            raise ValueError("the value normaliser's statistics need materialised returns")
        nat.check(nat.lib().mlearn_gae_f32(nat.ptr(r), nat.ptr(v), nat.ptr(d), nat.ptr(b),
                                           nat.ptr(adv), None, T, N, float(cfg.gamma),
                                           _gamma_lambda(cfg), nat.stream_handle()), "gae")
        return adv, None
    ret = out_ret if out_ret is not None else torch.empty_like(adv)
    if value_norm is not None:
        nat.check(nat.lib().mlearn_gae_vnorm_f32(
            nat.ptr(r), nat.ptr(v), nat.ptr(d), nat.ptr(b), nat.ptr(value_norm),
            int(norm_cols or N), nat.ptr(adv), nat.ptr(ret), T, N, float(cfg.gamma),
            _gamma_lambda(cfg), nat.stream_handle()), "gae_vnorm")
        return adv, ret
    nat.check(nat.lib().mlearn_gae_f32(nat.ptr(r), nat.ptr(v), nat.ptr(d), nat.ptr(b),
                                       nat.ptr(adv), nat.ptr(ret), T, N, float(cfg.gamma),
                                       _gamma_lambda(cfg), nat.stream_handle()), "gae")
    return adv, ret


def compute_returns(cfg, rewards, dones, bootstrap_values, out=None):
    """algo_common.py:45-81."""
    T = cfg.steps_per_update
    N = rewards.numel() // T
    r = _tn(rewards, T, N, torch.float32)
    d = _tn(dones, T, N, torch.uint8) if dones.dtype != torch.bool else \
        dones.reshape(T, N).contiguous().view(torch.uint8)
    b = bootstrap_values.reshape(N).to(torch.float32).contiguous()
    ret = out if out is not None else torch.empty((T, N), dtype=torch.float32, device=r.device)
    nat.check(nat.lib().mlearn_returns_f32(nat.ptr(r), nat.ptr(d), nat.ptr(b), nat.ptr(ret), T,
                                           N, float(cfg.gamma), nat.stream_handle()), "returns")
    return ret


def zscore_data(data):
    """algo_common.py:133-140 over the whole tensor."""
    x = data.to(torch.float32).contiguous()
    out = torch.empty_like(x)
    ws = torch.empty(int(nat.lib().mlearn_zscore_workspace_bytes(x.numel())), dtype=torch.uint8,
                     device=x.device)
    nat.check(nat.lib().mlearn_zscore_f32(nat.ptr(x), x.numel(), nat.ptr(out), nat.ptr(ws),
                                          nat.stream_handle()), "zscore")
    return out
