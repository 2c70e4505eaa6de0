"""Observation preprocessing (mirrors src/madrona_learn/observations.py).

On the accelerated path the preprocess is fused into the rollout kernel:
``ObservationsPreprocessNoop`` (observations.py:151-158) and
``ObservationsCaster`` (135-148) both reduce to "cast to the compute dtype
before the first Dense", which is what flax's Dense does anyway.  The rollout
store holds the observations in the compute dtype.  ``ObservationsEMANormalizer``
(70-132) adds the per-feature affine and its running statistics.
"""

from dataclasses import dataclass, field
from typing import Callable, Dict, Set

import torch

from .cfg import canonical_dtype
from .moving_avg import EMANormalizer


@dataclass(frozen=True)
class ObservationsPreprocess:  # observations.py:13-68
    def fused_cast_dtype(self, compute_dtype):
        raise NotImplementedError


@dataclass(frozen=True)
class ObservationsPreprocessNoop(ObservationsPreprocess):
    @staticmethod
    def create():
        return ObservationsPreprocessNoop()

    def fused_cast_dtype(self, compute_dtype):
        return compute_dtype


@dataclass(frozen=True)
class ObservationsCaster(ObservationsPreprocess):
    dtype: object = None

    @staticmethod
    def create(dtype):
        return ObservationsCaster(dtype=canonical_dtype(dtype))

    def fused_cast_dtype(self, compute_dtype):
        if canonical_dtype(self.dtype) != compute_dtype:
            raise NotImplementedError(
                "ObservationsCaster to a dtype other than TrainConfig.compute_dtype is not "
                "supported on the fused path")
        return compute_dtype


@dataclass(frozen=True)
class ObservationsEMANormalizer(ObservationsPreprocess):  # observations.py:70-132
    """EMA mean / variance normalisation of the observations.  On the fused
    path the normalisation ((x - mu) * inv_sigma, then the cast) runs inside
    the rollout kernel, the per-step statistics are tile partials written by
    the same launch, and mlearn_obs_norm_update folds them into the estimates
    after the rollout (rollouts.py:670-678, train.py:193-204).  prep_fns run
    in torch before the kernel; an observation named in skip_normalization is
    only cast."""
    normalizer: EMANormalizer
    prep_fns: Dict[str, Callable] = field(default_factory=dict)
    skip_normalization: Set[str] = field(default_factory=set)

    @staticmethod
    def create(decay, dtype, eps=1e-5, prep_fns=None, skip_normalization=None):
        dtype = canonical_dtype(dtype)
        return ObservationsEMANormalizer(
            normalizer=EMANormalizer(decay=decay, norm_dtype=dtype, inv_dtype=dtype, eps=eps),
            prep_fns=dict(prep_fns or {}), skip_normalization=set(skip_normalization or ()))

    def fused_cast_dtype(self, compute_dtype):
        nd = canonical_dtype(self.normalizer.norm_dtype)
        if nd not in (compute_dtype, torch.float32):
            raise NotImplementedError(
                "ObservationsEMANormalizer with a norm dtype other than float32 or "
                "TrainConfig.compute_dtype is not supported on the fused path")
        return compute_dtype

    def normalizes(self, ob_name):
        return not self.normalizer.disable and ob_name not in self.skip_normalization

    def prep(self, ob_name, ob):
        fn = self.prep_fns.get(ob_name)
        return ob if fn is None else fn(ob)
