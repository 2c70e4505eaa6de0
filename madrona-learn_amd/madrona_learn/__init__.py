"""madrona_learn — MI355X-native batched PPO hot path.

Drop-in for the PPO training iteration of shacklettbp/madrona-learn
(rollout collection -> GAE -> minibatch PPO update) with the reference's
public names (src/madrona_learn/__init__.py:1-52).  Compute runs in the
hand-written gfx950 HIP kernels of ``_lib/libmlearn.so`` (C ABI in
include/mlearn.h); PyTorch-ROCm provides device memory, streams, HIP graphs
and torch.distributed (RCCL).
"""

from .actor_critic import (ActorCritic, Backbone, BackboneEncoder, BackboneSeparate,
                           BackboneShared, RecurrentBackboneEncoder)
from .cfg import (ContinuousActionsConfig, DiscreteActionsConfig, EvalConfig, ParamExplore,
                  PBTConfig, TrainConfig)
from .dists import DiscreteActionDistributions, PhiloxKey
from .observations import (ObservationsCaster, ObservationsEMANormalizer,
                           ObservationsPreprocessNoop)
from .policy import Policy
from .ppo import PPOConfig
from .profile import profile
from .train import TrainHooks, TrainingManager, init_training, stop_training, train
from .train_state import TrainStateManager
from .tensorboard import TensorboardWriter
from . import pbt
from . import models
from . import rnn

__all__ = [
    "init_training", "stop_training", "train", "TrainHooks", "TrainingManager",
    "DiscreteActionsConfig", "ContinuousActionsConfig", "TrainConfig", "PBTConfig",
    "ParamExplore", "EvalConfig", "TrainStateManager", "models", "rnn", "Policy",
    "DiscreteActionDistributions", "PhiloxKey", "ObservationsEMANormalizer",
    "ObservationsCaster", "ObservationsPreprocessNoop", "ActorCritic", "BackboneEncoder",
    "RecurrentBackboneEncoder", "Backbone", "BackboneShared", "BackboneSeparate", "PPOConfig",
    "profile", "TensorboardWriter", "pbt",
]
