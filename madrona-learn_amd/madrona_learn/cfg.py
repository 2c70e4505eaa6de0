"""Training configuration dataclasses (mirrors src/madrona_learn/cfg.py:1-142).

Field names, order and defaults are the reference's.  The one type change:
``compute_dtype`` is a torch dtype (``torch.float32`` / ``torch.bfloat16`` on the fused
kernels; ``torch.float16`` trains on the torch path with DynamicScale)
instead of a jnp dtype; strings such as ``"bf16"`` are accepted too.
"""

import dataclasses
from dataclasses import dataclass
from typing import Dict, List, Optional, Union

import torch


@dataclass(frozen=True)
class DiscreteActionsConfig:  # cfg.py:9-11
    actions_num_buckets: List[int]


@dataclass(frozen=True)
class ContinuousActionsConfig:  # cfg.py:13-17 (not on the accelerated path)
    stddev_min: float
    stddev_max: float
    num_dims: int


class AlgoConfig:  # cfg.py:19-24
    def name(self):
        raise NotImplementedError

    def setup(self):
        raise NotImplementedError


@dataclass(frozen=True)
class ParamExplore:  # cfg.py:27-46
    base: float
    min_scale: float
    max_scale: float
    log10_scale: bool = False
    ln_scale: bool = False
    clip_perturb: bool = False
    perturb_rnd_min: float = 0.8
    perturb_rnd_max: float = 1.2

    def __repr__(self):
        if self.log10_scale:
            type_str = "log10, "
        elif self.ln_scale:
            type_str = "ln, "
        else:
            type_str = ""
        return (f"{self.base * self.min_scale}, {self.base * self.max_scale} "
                f"[{type_str}{self.perturb_rnd_min, self.perturb_rnd_max}]")


@dataclass(frozen=True)
class PBTConfig:  # cfg.py:49-65
    num_teams: int
    team_size: int
    num_train_policies: int
    num_past_policies: int
    self_play_portion: float
    cross_play_portion: float
    past_play_portion: float
    policy_overwrite_threshold: float = 0.7
    reward_hyper_params_explore: Dict[str, ParamExplore] = dataclasses.field(
        default_factory=dict)
    rollout_policy_chunk_size_override: int = 0


_DTYPE_ALIASES = {
    "f32": torch.float32, "fp32": torch.float32, "float32": torch.float32,
    "bf16": torch.bfloat16, "bfloat16": torch.bfloat16,
    # (after the bf16 names: "bfloat16" must not match "float16" first)
    "fp16": torch.float16, "float16": torch.float16, "half": torch.float16,
}


def canonical_dtype(d):
    if isinstance(d, torch.dtype):
        return d
    if isinstance(d, str) and d.lower() in _DTYPE_ALIASES:
        return _DTYPE_ALIASES[d.lower()]
    name = getattr(d, "__name__", None) or getattr(d, "name", None) or str(d)
    name = str(name).lower()
    for k, v in _DTYPE_ALIASES.items():
        if name.endswith(k):
            return v
    raise ValueError(f"unsupported compute dtype {d!r}")


@dataclass(frozen=True)
class TrainConfig:  # cfg.py:68-127
    num_worlds: int
    num_agents_per_world: int
    num_updates: int
    actions: Dict[str, Union[DiscreteActionsConfig, ContinuousActionsConfig]]
    steps_per_update: int
    lr: Union[float, ParamExplore]
    algo: AlgoConfig
    num_bptt_chunks: int
    gamma: float
    seed: int
    metrics_buffer_size: int
    baseline_policy_id: int = 0
    custom_policy_ids: List[int] = dataclasses.field(default_factory=lambda: [])
    gae_lambda: float = 1.0
    pbt: Optional[PBTConfig] = None
    dreamer_v3_critic: bool = True
    hlgauss_critic: bool = False
    compute_advantages: bool = True
    normalize_advantages: bool = True
    normalize_returns: bool = True
    normalize_values: bool = False
    filter_advantages: bool = False
    importance_sample_trajectories: bool = False
    importance_sample_num_minibatches: int = 0
    value_normalizer_decay: float = 0.99999
    max_advantage_est_decay: float = 0.99999
    compute_dtype: torch.dtype = torch.float32

    def __post_init__(self):
        object.__setattr__(self, "compute_dtype", canonical_dtype(self.compute_dtype))

    def __repr__(self):
        rep = "TrainConfig:"
        for k, v in self.__dict__.items():
            if k == "algo":
                rep += f"\n  {v.name()}:"
                for ak, av in self.algo.__dict__.items():
                    rep += f"\n    {ak}: {av}"
            elif k == "pbt":
                if v is None:
                    rep += "\n  pbt: Disabled"
                else:
                    rep += "\n  pbt:"
                    for pk, pv in self.pbt.__dict__.items():
                        rep += f"\n    {pk}: {pv}"
            elif k == "compute_dtype":
                rep += "\n  compute_dtype: " + {torch.bfloat16: "bf16",
                                                 torch.float16: "fp16"}.get(v, "fp32")
            else:
                rep += f"\n  {k}: {v}"
        return rep


@dataclass(frozen=True)
class EvalConfig:  # cfg.py:130-142 (eval is outside the accelerated path)
    num_worlds: int
    num_teams: int
    team_size: int
    num_eval_steps: int
    actions: Dict[str, Union[DiscreteActionsConfig, ContinuousActionsConfig]]
    reward_gamma: float
    policy_dtype: torch.dtype
    eval_competitive: bool
    use_deterministic_policy: bool = True
    clear_fitness: bool = True
    custom_policy_ids: List[int] = dataclasses.field(default_factory=lambda: [])
