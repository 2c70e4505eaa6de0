"""Observation preprocessing (mirrors src/madrona_learn/observations.py).

On the accelerated path the preprocess is fused into the rollout kernel:
``ObservationsPreprocessNoop`` (observations.py:151-158) and
``ObservationsCaster`` (135-148) both reduce to "cast to the compute dtype
before the first Dense", which is what flax's Dense does anyway.  The rollout
store holds the observations in the compute dtype.
"""

from dataclasses import dataclass

from .cfg import canonical_dtype


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
class ObservationsEMANormalizer(ObservationsPreprocess):  # observations.py:70-132 (next row)
    decay: float = 0.99999
    dtype: object = None
    eps: float = 1e-5

    @staticmethod
    def create(decay, dtype, eps=1e-5, prep_fns=None, skip_normalization=None):
        return ObservationsEMANormalizer(decay=decay, dtype=dtype, eps=eps)

    def fused_cast_dtype(self, compute_dtype):
        raise NotImplementedError(
            "ObservationsEMANormalizer is the next SURVEY §8(f) row; not on the fused path yet")
