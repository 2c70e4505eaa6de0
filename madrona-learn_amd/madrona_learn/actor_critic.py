"""Actor-critic plugin surface (mirrors src/madrona_learn/actor_critic.py).

Same class names and constructor fields as the reference's flax modules.
The computation itself runs in the fused HIP kernels; these classes carry
the architecture and the recurrent-state helpers of the reference API.
"""

from typing import Any, Callable, Union


def _identity_prefix(x, train=False):
    return x


class Backbone:  # actor_critic.py:13-35
    def init_recurrent_state(self, N):
        raise NotImplementedError

    def clear_recurrent_state(self, recurrent_states, should_clear):
        raise NotImplementedError


class BackboneEncoder:  # actor_critic.py:131-153 (no recurrent state)
    def __init__(self, net):
        self.net = net

    def init_recurrent_state(self, N):
        return ()

    def clear_recurrent_state(self, recurrent_states, should_clear):
        return ()


class RecurrentBackboneEncoder:  # actor_critic.py:156-199 (LSTM path: SURVEY §8(f) next)
    def __init__(self, net, rnn):
        self.net = net
        self.rnn = rnn

    def init_recurrent_state(self, N):
        return self.rnn.init_recurrent_state(N)

    def clear_recurrent_state(self, recurrent_states, should_clear):
        return self.rnn.clear_recurrent_state(recurrent_states, should_clear)


class BackboneShared(Backbone):  # actor_critic.py:202-244
    def __init__(self, prefix: Union[Callable, Any] = None, encoder=None):
        self.prefix = prefix if prefix is not None else _identity_prefix
        self.encoder = encoder

    def init_recurrent_state(self, N):
        return self.encoder.init_recurrent_state(N)

    def clear_recurrent_state(self, recurrent_states, should_clear):
        return self.encoder.clear_recurrent_state(recurrent_states, should_clear)


class BackboneSeparate(Backbone):  # actor_critic.py:247-303
    def __init__(self, prefix=None, actor_encoder=None, critic_encoder=None):
        self.prefix = prefix if prefix is not None else _identity_prefix
        self.actor_encoder = actor_encoder
        self.critic_encoder = critic_encoder

    def init_recurrent_state(self, N):
        return (self.actor_encoder.init_recurrent_state(N),
                self.critic_encoder.init_recurrent_state(N))

    def clear_recurrent_state(self, recurrent_states, should_clear):
        return (self.actor_encoder.clear_recurrent_state(recurrent_states[0], should_clear),
                self.critic_encoder.clear_recurrent_state(recurrent_states[1], should_clear))


class ActorCritic:  # actor_critic.py:38-128
    def __init__(self, backbone, actor, critic):
        self.backbone = backbone
        self.actor = actor
        self.critic = critic

    def init_recurrent_state(self, N):
        return self.backbone.init_recurrent_state(N)

    def clear_recurrent_state(self, recurrent_states, should_clear):
        return self.backbone.clear_recurrent_state(recurrent_states, should_clear)
