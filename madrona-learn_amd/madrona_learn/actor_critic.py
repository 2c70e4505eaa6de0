"""Actor-critic plugin surface (mirrors src/madrona_learn/actor_critic.py).

Same class names, constructor fields and methods as the reference's flax
modules, as torch ``nn.Module`` s:

* ``ActorCritic.rollout / actor_only / critic_only / update``
  (actor_critic.py:55-128) and ``Backbone.__call__ / actor_only /
  critic_only / sequence`` (actor_critic.py:13-35, 131-303).
* Fast path: when the tree is one the fused kernels implement
  (``BackboneShared(encoder=BackboneEncoder(net=MLP))`` or
  ``RecurrentBackboneEncoder(net=MLP, rnn=LSTM)``, ``DenseLayerDiscreteActor``,
  ``DenseLayerCritic`` / ``DreamerV3Critic``) the methods run the HIP
  kernels of ``libmlearn.so`` on the parameters of the ``PolicyState`` the
  tree is bound to (``init_training`` binds the training policy; an unbound
  tree compiles one on first use with the reference initialisers).
* Slow path: any other tree (a user's own ``Backbone`` / net / actor /
  critic ``nn.Module`` s) runs as plain torch modules, with the discrete
  distribution's sampling and statistics still on the HIP kernels
  (``DiscreteActionDistributions``).  ``init_training`` trains recognised
  trees only.
"""

from typing import Any, Callable, Union

import torch
from torch import nn

from . import _native as nat


def _identity_prefix(x, train=False):
    return x


def _flatten_obs_sequence(obs):  # actor_critic.py:14-15
    if isinstance(obs, dict):
        return {k: v.reshape(-1, *v.shape[2:]) for k, v in obs.items()}
    return obs.reshape(-1, *obs.shape[2:])


def _call(m, *args, train=False):
    try:
        return m(*args, train=train)
    except TypeError:
        return m(*args)


class Backbone(nn.Module):  # actor_critic.py:13-35
    def init_recurrent_state(self, N):
        raise NotImplementedError

    def clear_recurrent_state(self, recurrent_states, should_clear):
        raise NotImplementedError

    def forward(self, rnn_states, inputs, train=False):
        raise NotImplementedError

    def sequence(self, rnn_start_states, sequence_ends, flattened_inputs, train=False):
        raise NotImplementedError


class BackboneEncoder(nn.Module):  # actor_critic.py:131-153 (no recurrent state)
    def __init__(self, net):
        super().__init__()
        self.net = net

    def init_recurrent_state(self, N):
        return ()

    def clear_recurrent_state(self, recurrent_states, should_clear):
        return ()

    def forward(self, rnn_states, inputs, train=False):
        return _call(self.net, inputs, train=train), ()

    def sequence(self, rnn_start_states, sequence_ends, flattened_inputs, train=False):
        return _call(self.net, flattened_inputs, train=train)


class RecurrentBackboneEncoder(nn.Module):  # actor_critic.py:156-199
    def __init__(self, net, rnn):
        super().__init__()
        self.net = net
        self.rnn = rnn

    def init_recurrent_state(self, N):
        return self.rnn.init_recurrent_state(N)

    def clear_recurrent_state(self, recurrent_states, should_clear):
        return self.rnn.clear_recurrent_state(recurrent_states, should_clear)

    def forward(self, rnn_states_in, inputs, train=False):
        features = _call(self.net, inputs, train=train)
        return self.rnn(rnn_states_in, features, train)

    def sequence(self, rnn_start_states, sequence_ends, flattened_inputs, train=False):
        features = _call(self.net, flattened_inputs, train=train)
        T, N = sequence_ends.shape[0:2]
        seq = features.reshape(T, N, *features.shape[1:])
        out = self.rnn.sequence(rnn_start_states, sequence_ends, seq, train=train)
        return out.reshape(-1, *out.shape[2:])


class BackboneShared(Backbone):  # actor_critic.py:202-244
    def __init__(self, prefix: Union[Callable, Any] = None, encoder=None):
        super().__init__()
        self.prefix = prefix if prefix is not None else _identity_prefix
        self.encoder = encoder

    def init_recurrent_state(self, N):
        return self.encoder.init_recurrent_state(N)

    def clear_recurrent_state(self, recurrent_states, should_clear):
        return self.encoder.clear_recurrent_state(recurrent_states, should_clear)

    def _rollout_common(self, rnn_states_in, obs_in, train):
        processed = _call(self.prefix, obs_in, train=train)
        return self.encoder(rnn_states_in, processed, train=train)

    def forward(self, rnn_states_in, obs_in, train=False):
        features, rnn_states_out = self._rollout_common(rnn_states_in, obs_in, train)
        return features, features, rnn_states_out

    def actor_only(self, rnn_states_in, obs_in, train=False):
        return self._rollout_common(rnn_states_in, obs_in, train)

    def critic_only(self, rnn_states_in, obs_in, train=False):
        return self._rollout_common(rnn_states_in, obs_in, train)

    def sequence(self, rnn_start_states, sequence_ends, obs_in, train=False):
        processed = _call(self.prefix, _flatten_obs_sequence(obs_in), train=train)
        features = self.encoder.sequence(rnn_start_states, sequence_ends, processed, train=train)
        return features, features


class BackboneSeparate(Backbone):  # actor_critic.py:247-303
    def __init__(self, prefix=None, actor_encoder=None, critic_encoder=None):
        super().__init__()
        self.prefix = prefix if prefix is not None else _identity_prefix
        self.actor_encoder = actor_encoder
        self.critic_encoder = critic_encoder

    def init_recurrent_state(self, N):
        return (self.actor_encoder.init_recurrent_state(N),
                self.critic_encoder.init_recurrent_state(N))

    def clear_recurrent_state(self, recurrent_states, should_clear):
        return (self.actor_encoder.clear_recurrent_state(recurrent_states[0], should_clear),
                self.critic_encoder.clear_recurrent_state(recurrent_states[1], should_clear))

    def forward(self, rnn_states_in, obs_in, train=False):
        processed = _call(self.prefix, obs_in, train=train)
        af, ar = self.actor_encoder(rnn_states_in[0], processed, train=train)
        cf, cr = self.critic_encoder(rnn_states_in[1], processed, train=train)
        return af, cf, (ar, cr)

    def actor_only(self, rnn_states_in, obs_in, train=False):
        processed = _call(self.prefix, obs_in, train=train)
        f, r = self.actor_encoder(rnn_states_in[0], processed, train=train)
        return f, (r, rnn_states_in[1])

    def critic_only(self, rnn_states_in, obs_in, train=False):
        processed = _call(self.prefix, obs_in, train=train)
        f, r = self.critic_encoder(rnn_states_in[1], processed, train=train)
        return f, (rnn_states_in[0], r)

    def sequence(self, rnn_start_states, sequence_ends, obs_in, train=False):
        processed = _call(self.prefix, _flatten_obs_sequence(obs_in), train=train)
        af = self.actor_encoder.sequence(rnn_start_states[0], sequence_ends, processed,
                                         train=train)
        cf = self.critic_encoder.sequence(rnn_start_states[1], sequence_ends, processed,
                                          train=train)
        return af, cf


def _key_parts(prng_key):
    """(k0, k1, step, env_offset) of a PhiloxKey or a (k0, k1[, step]) tuple."""
    from .dists import PhiloxKey
    if isinstance(prng_key, PhiloxKey):
        return prng_key.k0, prng_key.k1, prng_key.step, prng_key.env_offset
    t = tuple(int(x) for x in prng_key)
    return t[0] & 0xFFFFFFFF, t[1] & 0xFFFFFFFF, (t[2] if len(t) > 2 else 0), 0


class ActorCritic(nn.Module):  # actor_critic.py:38-128
    def __init__(self, backbone, actor, critic):
        super().__init__()
        self.backbone = backbone
        self.actor = actor
        self.critic = critic
        self._bound = None       # PolicyState of the fused path (bind / lazy compile)
        self._fast = None        # None: not decided yet

    def init_recurrent_state(self, N):
        return self.backbone.init_recurrent_state(N)

    def clear_recurrent_state(self, recurrent_states, should_clear):
        return self.backbone.clear_recurrent_state(recurrent_states, should_clear)

    # -- fast path ----------------------------------------------------------
    def bind(self, policy_state):
        """Run the methods on this PolicyState's parameters (the fused path)."""
        object.__setattr__(self, "_bound", policy_state)
        object.__setattr__(self, "_fast", True)
        return self

    @property
    def policy_state(self):
        return self._bound

    def _fused(self, obs):
        """The bound / lazily compiled PolicyState, or None (slow path)."""
        if self._fast is False:
            return None
        if self._bound is not None:
            return self._bound
        from .train_state import PolicyState, compile_arch
        import numpy as np
        x = self._obs_matrix(obs)
        try:
            enc = self.backbone.encoder if isinstance(self.backbone, BackboneShared) else None
            dtype = getattr(getattr(enc, "net", None), "dtype", None)
            if dtype is None:
                raise NotImplementedError("no MLP trunk")
            arch = compile_arch(self, x.shape[1], dtype)
        except NotImplementedError:
            object.__setattr__(self, "_fast", False)
            return None
        ps = PolicyState(self, arch, None, x.device, np.random.default_rng(0))
        return self.bind(ps)._bound

    def _obs_matrix(self, obs, train=False):
        from .rollouts import obs_to_matrix
        x = self.backbone.prefix(obs, train=train) if hasattr(self.backbone, "prefix") else obs
        if isinstance(x, dict):
            x = next(iter(x.values())) if len(x) == 1 else x
        n = x.shape[0]
        return obs_to_matrix(x, n)

    def _carry(self, ps, rnn_states, N):
        """LstmCarry over fresh copies of the (c_states, h_states) input."""
        c_states, h_states = rnn_states
        dt = ps.arch.dtype
        h = h_states[0].to(dt).contiguous().clone()
        c = c_states[0].to(dt).contiguous().clone()
        d = nat.LstmCarry()
        d.h, d.c = h.data_ptr(), c.data_ptr()
        d.commit = 1
        return d, h, c

    def _fused_step(self, ps, rnn_states, obs, key=None, sample=True, actions=True,
                    eval_actions=None, clear=None):
        x = self._obs_matrix(obs)
        N = x.shape[0]
        dev = x.device
        K = ps.arch.num_groups
        out = {}
        acts = torch.empty((N, K), dtype=torch.int32, device=dev) if actions else None
        logp = torch.empty((N, K), dtype=torch.float32, device=dev) \
            if (actions and sample) or eval_actions is not None else None
        ent = torch.empty((N, K), dtype=torch.float32, device=dev) \
            if eval_actions is not None else None
        vals = torch.empty((N,), dtype=torch.float32, device=dev)
        k0, k1, step, eoff = _key_parts(key) if key is not None else (0, 0, 0, 0)
        L = nat.lib()
        strm = nat.stream_handle()
        new_states = ()
        carry = None
        if ps.recurrent:
            carry, h, c = self._carry(ps, rnn_states, N)
            if clear is not None:
                clear = clear.reshape(-1).to(torch.uint8).contiguous()
                carry.clear = clear.data_ptr()
            new_states = ([c], [h])
        if eval_actions is not None:
            ea = eval_actions.reshape(N, K).to(torch.int32).contiguous()
            if ps.recurrent:
                nat.check(L.mlearn_lstm_policy_evaluate(ps.desc, ps.lstm_desc, carry, nat.ptr(x), N,
                                                        nat.ptr(ea), nat.ptr(logp), nat.ptr(ent),
                                                        nat.ptr(vals), strm), "lstm_evaluate")
            else:
                nat.check(L.mlearn_policy_evaluate(ps.desc, nat.ptr(x), N, nat.ptr(ea),
                                                   nat.ptr(logp), nat.ptr(ent), nat.ptr(vals),
                                                   strm), "policy_evaluate")
            return {"log_probs": logp, "entropies": ent, "critic": vals[:, None]}, new_states
        if ps.recurrent:
            nat.check(L.mlearn_lstm_policy_rollout_step(
                ps.desc, ps.lstm_desc, carry, nat.ptr(x), N, None, nat.ptr(acts), nat.ptr(logp),
                nat.ptr(vals), k0, k1, None, step, eoff, 1 if sample else 0, None, strm),
                "lstm_rollout")
        else:
            nat.check(L.mlearn_policy_rollout_step(
                ps.desc, nat.ptr(x), N, None, nat.ptr(acts), nat.ptr(logp), nat.ptr(vals), k0, k1,
                None, step, eoff, 1 if sample else 0, None, strm), "policy_rollout")
        if actions:
            out["actions"] = acts
            if sample:
                out["log_probs"] = logp
        out["critic"] = vals[:, None]
        return out, new_states

    # -- the reference's methods ---------------------------------------------
    def actor_only(self, rnn_states_in, obs_in, train=False):  # actor_critic.py:55-63
        ps = self._fused(obs_in)
        if ps is not None:
            out, st = self._fused_step(ps, rnn_states_in, obs_in, sample=False)
            return {"actions": out["actions"]}, st
        features, rnn_states_out = self.backbone.actor_only(rnn_states_in, obs_in, train=train)
        dists = _call(self.actor, features, train=train)
        return {"actions": dists.best()}, rnn_states_out

    def critic_only(self, rnn_states_in, obs_in, train=False):  # actor_critic.py:65-72
        ps = self._fused(obs_in)
        if ps is not None:
            out, st = self._fused_step(ps, rnn_states_in, obs_in, actions=False)
            return {"critic": out["critic"]}, st
        features, rnn_states_out = self.backbone.critic_only(rnn_states_in, obs_in, train=train)
        return {"critic": _call(self.critic, features, train=train)}, rnn_states_out

    def rollout(self, prng_key, rnn_states_in, obs_in, train=False, sample_actions=True,
                return_debug=False):  # actor_critic.py:74-96
        ps = self._fused(obs_in)
        if ps is not None:
            return self._fused_step(ps, rnn_states_in, obs_in, key=prng_key,
                                    sample=sample_actions)
        actor_features, critic_features, rnn_states_out = self.backbone(
            rnn_states_in, obs_in, train=train)
        dists = _call(self.actor, actor_features, train=train)
        results = {}
        if sample_actions:
            actions, log_probs = dists.sample(prng_key)
            results["log_probs"] = log_probs
        else:
            actions = dists.best()
        results["actions"] = actions
        results["critic"] = _call(self.critic, critic_features, train=train)
        return results, rnn_states_out

    def update(self, rnn_states, sequence_breaks, rollout_actions, obs,
               train=True):  # actor_critic.py:98-128
        if isinstance(rollout_actions, dict):
            rollout_actions = torch.cat([rollout_actions[k] for k in rollout_actions], dim=-1)
        T, N = sequence_breaks.shape[0:2]
        flat_obs = _flatten_obs_sequence(obs)
        ps = self._fused(flat_obs)
        if ps is not None:
            acts = rollout_actions.reshape(T * N, -1)
            if not ps.recurrent:
                out, _ = self._fused_step(ps, rnn_states, flat_obs, eval_actions=acts)
            else:
                # LSTM.sequence (rnn.py:81-111): the carry enters step t cleared
                # where step t - 1 ended a sequence
                seq_obs = obs if not isinstance(obs, dict) else next(iter(obs.values()))
                outs = []
                st = rnn_states
                for t in range(T):
                    o, st = self._fused_step(
                        ps, st, seq_obs[t], eval_actions=rollout_actions[t],
                        clear=sequence_breaks[t - 1] if t > 0 else None)
                    outs.append(o)
                out = {k: torch.cat([o[k] for o in outs], 0) for k in outs[0]}
            return {k: v.reshape(T, N, *v.shape[1:]) for k, v in out.items()}
        actor_features, critic_features = self.backbone.sequence(
            rnn_states, sequence_breaks, obs, train=train)
        dists = _call(self.actor, actor_features, train=train)
        critic_out = _call(self.critic, critic_features, train=train)
        flat_actions = rollout_actions.reshape(T * N, *rollout_actions.shape[2:])
        log_probs, entropies = dists.action_stats(flat_actions)
        return {"log_probs": log_probs.reshape(T, N, *log_probs.shape[1:]),
                "entropies": entropies.reshape(T, N, *entropies.shape[1:]),
                "critic": critic_out.reshape(T, N, *critic_out.shape[1:])}
