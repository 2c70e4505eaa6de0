"""Model building blocks (mirrors src/madrona_learn/models.py).

These are architecture *descriptions*: the MI355X engine compiles a
recognised ActorCritic tree (BackboneShared/BackboneEncoder + MLP + discrete
actor + scalar critic) into the fused HIP kernels of ``libmlearn.so``
(see train_state.compile_policy).  Parameters are created by the engine with
the reference's initialisers (orthogonal with the same scales, zero biases,
LayerNorm scale 1 / bias 0).
"""

import math

import numpy as np

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


class LayerNorm:  # models.py:46-56 (flax nn.LayerNorm, eps 1e-6, f32 statistics)
    def __init__(self, dtype):
        self.dtype = canonical_dtype(dtype)


class MLP:  # models.py:99-119: Dense(no bias) -> LayerNorm -> ReLU per layer
    def __init__(self, num_channels, num_layers, dtype, weight_init=orthogonal(math.sqrt(2))):
        self.num_channels = int(num_channels)
        self.num_layers = int(num_layers)
        self.dtype = canonical_dtype(dtype)
        self.weight_init = weight_init


class DenseLayerDiscreteActor:  # models.py:122-139
    def __init__(self, cfg: DiscreteActionsConfig, dtype, weight_init=orthogonal(0.01)):
        self.cfg = cfg
        self.dtype = canonical_dtype(dtype)
        self.weight_init = weight_init


class DenseLayerCritic:  # models.py:142-154 (output cast to f32)
    def __init__(self, dtype, weight_init=orthogonal(1.0)):
        self.dtype = canonical_dtype(dtype)
        self.weight_init = weight_init


class DreamerV3Critic:  # models.py:157-174 -- next row of SURVEY §8(f), not compiled yet
    def __init__(self, dtype, weight_init=constant(0.0), num_bins=63):
        self.dtype = canonical_dtype(dtype)
        self.weight_init = weight_init
        self.num_bins = num_bins
