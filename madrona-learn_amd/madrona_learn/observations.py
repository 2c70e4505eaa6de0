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


class _Bare(dict):
    """The state (or statistics) of a bare, unnamed observation tensor: a dict
    marked apart from the dict of per-name states a dict of observations
    keeps, so the state-only hooks know which of the two they were given."""


def _wrap(x):
    return _Bare(x) if isinstance(x, dict) else x


def _unwrap(x):
    return dict(x) if isinstance(x, _Bare) else x


def _pick(x, k):
    return x[k] if isinstance(x, dict) and not isinstance(x, _Bare) else None


def _map_obs(cb, obs, *states):
    """observations.py:36-57: cb(ob_name, ob, *per-observation states) over
    the names of the observation dict obs; a bare tensor is one observation
    named None whose states are kept _Bare-marked.  The reference's vmap over
    the policy axis has no counterpart: one policy's state per call."""
    if not isinstance(obs, dict):
        return cb(None, obs, *[_unwrap(s) for s in states])
    return {k: cb(k, obs[k], *[_pick(s, k) for s in states]) for k in obs}


def _map_states(cb, states, *more):
    """cb(ob_name, state, *more states) over a state structure (a _Bare or
    None state is the bare observation's); results keep the structure."""
    if states is None or isinstance(states, _Bare):
        return _wrap(cb(None, _unwrap(states), *[_unwrap(m) for m in more]))
    return {k: cb(k, states[k], *[_pick(m, k) for m in more]) for k in states}


@dataclass(frozen=True)
class ObservationsPreprocess:  # observations.py:13-68
    """The reference's plugin interface: subclasses override ``_preprocess``
    (and, for stateful preprocessing, ``_init_state`` / ``_update_state`` /
    ``_init_obs_stats`` / ``_update_obs_stats``).  The built-in Noop / Caster
    / EMANormalizer run fused into the rollout kernel on the fused path; any
    other subclass selects the torch path of init_training (generic.py),
    which calls these hooks as rollouts.py:838-840, 670-678 and
    train.py:193-204 do.  ``vmap`` is accepted for signature parity (one
    policy's state per call here)."""

    def preprocess(self, states, obs, vmap=False):
        return _map_obs(lambda k, ob, st: self._preprocess(k, st, ob), obs, states)

    def init_state(self, obs, vmap=False):
        r = _map_obs(lambda k, ob: self._init_state(k, ob), obs)
        return r if isinstance(obs, dict) else _wrap(r)

    def update_state(self, states, o_stats, vmap=False):
        return _map_states(self._update_state, states, o_stats)

    def init_obs_stats(self, states, vmap=False):
        return _map_states(self._init_obs_stats, states)

    def update_obs_stats(self, states, cur_obs_stats, num_prev_updates, obs, vmap=False):
        r = _map_obs(lambda k, ob, st, cs: self._update_obs_stats(k, st, cs, num_prev_updates, ob),
                     obs, states, cur_obs_stats)
        return r if isinstance(obs, dict) else _wrap(r)

    def _preprocess(self, ob_name, state, ob):
        return ob

    def _init_state(self, ob_name, ob):
        return None

    def _update_state(self, ob_name, est, ob_stats):
        return None

    def _init_obs_stats(self, ob_name, est):
        return None

    def _update_obs_stats(self, ob_name, est, ob_stats, num_prev_updates, ob):
        return None

    def has_state(self):
        """True when a subclass keeps state (overrides a state hook)."""
        base = ObservationsPreprocess
        return any(getattr(type(self), f) is not getattr(base, f)
                   for f in ("_init_state", "_update_state", "_init_obs_stats",
                             "_update_obs_stats"))

    def fused_cast_dtype(self, compute_dtype):
        """The dtype the fused rollout kernel casts the observations to when
        it implements this preprocess; NotImplementedError selects the torch
        path (generic.py) for a user's subclass."""
        raise NotImplementedError(
            f"{type(self).__name__} is not one of the fused preprocessors (Noop, Caster, "
            "EMANormalizer)")


@dataclass(frozen=True)
class ObservationsPreprocessNoop(ObservationsPreprocess):
    @staticmethod
    def create():
        return ObservationsPreprocessNoop()

    def fused_cast_dtype(self, compute_dtype):
        return compute_dtype

    def _preprocess(self, ob_name, state, ob):  # observations.py:157-158
        return ob


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

    def _preprocess(self, ob_name, state, ob):  # observations.py:147-148
        return ob.to(canonical_dtype(self.dtype))


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

    # observations.py:93-132 (the torch path's hooks; the fused path runs the
    # same arithmetic in the rollout kernel + mlearn_obs_norm_update)
    def _preprocess(self, ob_name, est, ob):
        ob = self.prep(ob_name, ob)
        if not self.normalizes(ob_name):
            return ob
        return self.normalizer.normalize(est, ob)

    def _init_state(self, ob_name, ob):
        if not self.normalizes(ob_name):
            return None
        return self.normalizer.init_estimates(self.prep(ob_name, ob))

    def _update_state(self, ob_name, est, ob_stats):
        if not self.normalizes(ob_name):
            return None
        return self.normalizer.update_estimates(est, ob_stats)

    def _init_obs_stats(self, ob_name, est):
        if not self.normalizes(ob_name):
            return None
        return self.normalizer.init_input_stats(est)

    def _update_obs_stats(self, ob_name, est, ob_stats, num_prev_updates, ob):
        if not self.normalizes(ob_name):
            return None
        return self.normalizer.update_input_stats(ob_stats, num_prev_updates,
                                                  self.prep(ob_name, ob))
