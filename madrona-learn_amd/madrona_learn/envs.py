"""Synthetic dummy vec-env (test/bench sim plugin).

Stands in for a Madrona simulator behind the reference's ``sim_fns``
protocol (rollouts.py:206-215, 905-936): ``init() -> {'state', 'obs'}`` and
``step({'state', 'actions', 'resets', 'sim_ctrl', 'pbt'}) -> {'state', 'obs',
'rewards', 'dones'}``.  One HIP launch per step (misc.hip env_step_kernel).
Deterministic: staggered fixed episode lengths, Philox observations and
rewards, reward depends on action[0].  With ``sim_fns()['native_step']`` the
rollout fuses the step into the policy launch (policy.hip), which removes the
sim launch and its round trip from every env step.
"""

import torch

from . import _native as nat


class DummyVecEnv:
    def __init__(self, num_envs, obs_dim=64, num_actions=6, seed=0, env_offset=0,
                 device="cuda"):
        self.N = int(num_envs)
        self.D = int(obs_dim)
        self.K = int(num_actions)
        self.k0 = (seed * 0x9E3779B9 + 0x1234) & 0xFFFFFFFF
        self.k1 = (seed * 0x85EBCA6B + 0x5678) & 0xFFFFFFFF
        self.env_offset = int(env_offset)
        dev = torch.device(device)
        self.state = torch.zeros((self.N, 4), dtype=torch.int32, device=dev)
        self.obs = torch.zeros((self.N, self.D), dtype=torch.float32, device=dev)
        self.rewards = torch.zeros((self.N, 1), dtype=torch.float32, device=dev)
        self.dones = torch.zeros((self.N, 1), dtype=torch.bool, device=dev)

    def init(self):
        nat.check(nat.lib().mlearn_dummy_env_reset(
            nat.ptr(self.state), self.N, self.D, self.k0, self.k1, self.env_offset,
            nat.ptr(self.obs), nat.stream_handle()), "env_reset")
        return {"state": self.state, "obs": self.obs}

    def step(self, inp):
        acts = inp["actions"]
        if isinstance(acts, dict):  # several action groups: the first drives the reward
            acts = next(iter(acts.values()))
        if acts.dtype != torch.int32 or not acts.is_contiguous():
            acts = acts.to(torch.int32).contiguous()
        nat.check(nat.lib().mlearn_dummy_env_step(
            nat.ptr(self.state), nat.ptr(acts), acts.shape[-1], self.N, self.D, self.k0, self.k1,
            self.env_offset, nat.ptr(self.obs), nat.ptr(self.rewards), nat.ptr(self.dones),
            nat.stream_handle()), "env_step")
        return {"state": self.state, "obs": self.obs, "rewards": self.rewards,
                "dones": self.dones}

    def get_ckpts(self):
        """Per-env checkpoints (sim_fns['get_ckpts'], rollouts.py:300-301)."""
        return self.state.clone()

    def load_ckpts(self, ckpts, load_trigger=None):
        """Restore per-env state (sim_fns['load_ckpts'], rollouts.py:303-309)."""
        if load_trigger is None:
            self.state.copy_(ckpts)
        else:
            m = load_trigger.reshape(-1).bool()
            self.state[m] = ckpts.to(self.state.device)[m]
        return self.obs

    def native_step(self, col0=0, ncols=None):
        """Descriptor of this sim's step for the env columns [col0, col0 +
        ncols), run inside the rollout policy launch that samples their
        actions (mlearn_policy_rollout_step_env; bit-identical to step()).
        Outputs land in the same state / obs / rewards / dones tensors."""
        ncols = self.N - col0 if ncols is None else ncols
        assert 0 <= col0 and col0 + ncols <= self.N
        d = nat.DummyEnv()
        d.state = self.state.data_ptr() + col0 * 16
        d.obs = self.obs.data_ptr() + col0 * self.D * 4
        d.rewards = self.rewards.data_ptr() + col0 * 4
        d.dones = self.dones.data_ptr() + col0
        d.k0, d.k1 = self.k0, self.k1
        d.env_offset = (self.env_offset + col0) & 0xFFFFFFFF
        return d

    def native_outputs(self):
        """The step() output dict the fused step fills."""
        return {"state": self.state, "obs": self.obs, "rewards": self.rewards,
                "dones": self.dones}

    def sim_fns(self, fused=True):
        """The reference's sim_fns dict (rollouts.py:206-215, 905-936); with
        fused=True also 'native_step' (this build's extension): the rollout
        then runs the env step inside the policy launch instead of calling
        'step' between launches."""
        fns = {"init": self.init, "step": self.step, "get_ckpts": self.get_ckpts,
               "load_ckpts": self.load_ckpts}
        if fused:
            fns["native_step"] = self
        return fns
