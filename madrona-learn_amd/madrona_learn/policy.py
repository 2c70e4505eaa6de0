"""Policy bundle (mirrors src/madrona_learn/policy.py:13-17)."""

from dataclasses import dataclass
from typing import Callable, Optional

from .actor_critic import ActorCritic
from .observations import ObservationsPreprocess


@dataclass(frozen=True)
class Policy:
    actor_critic: ActorCritic
    obs_preprocess: Optional[ObservationsPreprocess] = None
    get_episode_scores: Optional[Callable] = None
