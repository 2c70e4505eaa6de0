"""Model building blocks (mirrors src/madrona_learn/models.py).

Each class is both an architecture description and a torch module:

* fast path: the MI355X engine compiles a recognised ActorCritic tree
  (BackboneShared/BackboneEncoder + MLP (+ LSTM) + discrete actor + scalar
  or two-hot critic) into the fused HIP kernels of ``libmlearn.so`` (see
  train_state.compile_arch); its parameters then live in the engine's flat
  arena, created with the reference's initialisers (orthogonal with the
  same scales, zero biases, LayerNorm scale 1 / bias 0);
* slow path: inside a tree the engine does not recognise, the modules run
  as plain torch (``forward``), parameters created lazily on the first call
  with the same initialisers.
"""

import math

import numpy as np
import torch
from torch import nn

from .cfg import DiscreteActionsConfig, canonical_dtype

def orthogonal(scale=1.0):
    """jax.nn.initializers.orthogonal restated (column/row orthonormal * scale)
    for a Dense kernel of shape (fan_in, fan_out)."""

    def init(rng: np.random.Generator, shape):
        n_rows, n_cols = int(np.prod(shape[:-1])), shape[-1]
        mshape = (n_cols, n_rows) if n_rows < n_cols else (n_rows, n_cols)
        a = rng.standard_normal(mshape)
        q, r = np.linalg.qr(a)
        q = q * np.sign(np.diag(r))
        if n_rows < n_cols:
            q = q.T
        return (scale * q).reshape(shape).astype(np.float32)

    init.scale = scale
    return init


def constant(value):
    def init(rng, shape):
        return np.full(shape, value, dtype=np.float32)

    return init


def _init_rng():
    """numpy generator for lazily created slow-path parameters (follows torch's seed)."""
    return np.random.default_rng(int(torch.randint(0, 2 ** 31 - 1, ()).item()))


class _Dense(nn.Module):
    """flax nn.Dense with the given kernel init (bias init 0), created lazily."""

    def __init__(self, features, use_bias, dtype, kernel_init):
        super().__init__()
        self.features = int(features)
        self.use_bias = use_bias
        self.dtype = dtype
        self.kernel_init = kernel_init
        self.kernel = None
        self.bias = None

    def forward(self, x):
        if self.kernel is None:
            w = self.kernel_init(_init_rng(), (x.shape[-1], self.features))
            self.kernel = nn.Parameter(torch.from_numpy(np.asarray(w, np.float32)).to(x.device))
            if self.use_bias:
                self.bias = nn.Parameter(torch.zeros(self.features, device=x.device))
        y = x.to(self.dtype) @ self.kernel.to(self.dtype)
        if self.use_bias:
            y = y + self.bias.to(self.dtype)
        return y


class LayerNorm(nn.Module):  # models.py:46-56 (flax nn.LayerNorm: eps 1e-6, f32 statistics)
    def __init__(self, dtype):
        super().__init__()
        self.dtype = canonical_dtype(dtype)
        self.scale = None
        self.bias = None

    def forward(self, x):
        F = x.shape[-1]
        if self.scale is None:
            self.scale = nn.Parameter(torch.ones(F, device=x.device))
            self.bias = nn.Parameter(torch.zeros(F, device=x.device))
        xf = x.float()
        mean = xf.mean(-1, keepdim=True)
        var = torch.clamp((xf * xf).mean(-1, keepdim=True) - mean * mean, min=0.0)  # fast variance
        y = (xf - mean) * (torch.rsqrt(var + 1e-6) * self.scale) + self.bias
        return y.to(self.dtype)


class MLP(nn.Module):  # models.py:99-119: Dense(no bias) -> LayerNorm -> ReLU per layer
    def __init__(self, num_channels, num_layers, dtype, weight_init=orthogonal(math.sqrt(2))):
        super().__init__()
        self.num_channels = int(num_channels)
        self.num_layers = int(num_layers)
        self.dtype = canonical_dtype(dtype)
        self.weight_init = weight_init
        self.dense = nn.ModuleList([_Dense(num_channels, False, self.dtype, weight_init)
                                    for _ in range(self.num_layers)])
        self.norms = nn.ModuleList([LayerNorm(self.dtype) for _ in range(self.num_layers)])

    def forward(self, inputs, train=False):
        x = inputs
        for d, n in zip(self.dense, self.norms):
            x = torch.relu(n(d(x)))
        return x


def action_groups(cfg):
    """[(name, buckets)] of a DiscreteActionsConfig or of a dict name ->
    DiscreteActionsConfig (TrainConfig.actions, cfg.py:73)."""
    if isinstance(cfg, DiscreteActionsConfig):
        return [("actions", list(cfg.actions_num_buckets))]
    out = []
    for k, v in cfg.items():
        if not isinstance(v, DiscreteActionsConfig):
            raise NotImplementedError(f"action group {k!r}: only discrete actions are supported")
        out.append((k, list(v.actions_num_buckets)))
    return out


class DenseLayerDiscreteActor(nn.Module):  # models.py:122-139
    """cfg: one DiscreteActionsConfig (the reference's head), or a dict of
    them (several action groups from one Dense head, logits concatenated in
    dict order; the distributions are keyed like TrainConfig.actions)."""

    def __init__(self, cfg, dtype, weight_init=orthogonal(0.01)):
        super().__init__()
        self.cfg = cfg
        self.dtype = canonical_dtype(dtype)
        self.weight_init = weight_init
        self.groups = action_groups(cfg)
        self.buckets = [b for _, g in self.groups for b in g]
        self.impl = _Dense(sum(self.buckets), True, self.dtype, weight_init)

    def forward(self, features, train=False):
        from .dists import DiscreteActionDistributions
        return DiscreteActionDistributions(self.buckets, self.impl(features))


class DenseLayerCritic(nn.Module):  # models.py:142-154 (output cast to f32)
    def __init__(self, dtype, weight_init=orthogonal(1.0)):
        super().__init__()
        self.dtype = canonical_dtype(dtype)
        self.weight_init = weight_init
        self.impl = _Dense(1, True, self.dtype, weight_init)

    def forward(self, features, train=False):
        return self.impl(features).float()


class DreamerV3Critic(nn.Module):  # models.py:157-174 (SymExpTwoHotDistribution head)
    def __init__(self, dtype, weight_init=constant(0.0), num_bins=63):
        super().__init__()
        self.dtype = canonical_dtype(dtype)
        self.weight_init = weight_init
        self.num_bins = num_bins
        self.impl = _Dense(num_bins, True, self.dtype, weight_init)

    def forward(self, features, train=False):
        from .dists import SymExpTwoHotDistribution
        return SymExpTwoHotDistribution(self.impl(features))
