"""EMA estimators (mirrors src/madrona_learn/moving_avg.py).

Descriptions of the reference's estimators; the arithmetic runs natively
(mlearn_obs_norm_update in csrc/misc.hip) and is restated in
oracle/ppo_ref.py (ema_*).
"""

from dataclasses import dataclass

from .cfg import canonical_dtype


@dataclass(frozen=True)
class EMAEstimate:  # moving_avg.py:7-45
    decay: float
    eps: float = 1e-5


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
