"""Rollout engine (mirrors src/madrona_learn/rollouts.py).

``RolloutManager.collect`` runs the reference's rollout_loop (rollouts.py:
829-978) as, per step: one fused HIP launch for preprocess + policy +
sample + store (policy.hip) with the previous step's post-step (rewards /
dones store, env returns), then the user's sim step (the built-in synthetic
sim's step runs inside the same launch instead, envs.DummyVecEnv.native_step).  Then the bootstrap critic, GAE/returns
and the rollout metrics.  No finalize transpose (rollouts.py:786-804): the
store stays [T][N] = [C][T/C][P][B] and the PPO kernels index sequences
directly.
"""

import math
from dataclasses import dataclass
from typing import Any, Callable, Dict, Optional

import torch

from . import _native as nat
from .algo_common import compute_advantages, compute_returns
from .cfg import DiscreteActionsConfig


@dataclass(frozen=True)
class RolloutConfig:  # rollouts.py:28-134 (self-play / single-policy path)
    sim_batch_size: int
    num_worlds: int
    actions_cfg: Dict
    policy_chunk_size: int
    num_policy_chunks: int
    total_policy_batch_size: int
    reward_gamma: float
    policy_dtype: torch.dtype
    reward_dtype: torch.dtype = torch.float32
    prob_dtype: torch.dtype = torch.float32
    pbt: Any = None

    @staticmethod
    def setup(num_current_policies, num_past_policies, num_teams, team_size, sim_batch_size,
              actions_cfg, self_play_portion, cross_play_portion, past_play_portion,
              static_play_portion, reward_gamma, custom_policy_ids, policy_dtype,
              reward_dtype=torch.float32, prob_dtype=torch.float32,
              policy_chunk_size_override=0):
        complex_mm = (num_current_policies > 1 and self_play_portion != 1.0) or \
            num_past_policies > 0 or cross_play_portion > 0 or past_play_portion > 0 or \
            static_play_portion > 0
        if complex_mm:
            raise NotImplementedError(
                "cross-play / past-play matchmaking (pbt.py:135-247) is outside the fused "
                "path; populations use the self-play split (pbt.py:130-133): policy p owns "
                "env columns [p*B, (p+1)*B)")
        assert sim_batch_size % num_current_policies == 0
        policy_chunk_size = sim_batch_size // num_current_policies  # rollouts.py:104-108
        if policy_chunk_size_override != 0:
            policy_chunk_size = policy_chunk_size_override
        num_policy_chunks = -(sim_batch_size // -policy_chunk_size)
        return RolloutConfig(
            sim_batch_size=sim_batch_size,
            num_worlds=sim_batch_size // (team_size * num_teams),
            actions_cfg=actions_cfg,
            policy_chunk_size=policy_chunk_size,
            num_policy_chunks=num_policy_chunks,
            total_policy_batch_size=num_policy_chunks * policy_chunk_size,
            reward_gamma=reward_gamma,
            policy_dtype=policy_dtype,
            reward_dtype=reward_dtype,
            prob_dtype=prob_dtype,
        )


class RolloutState:  # rollouts.py:171-309
    def __init__(self, cfg, step_fn, sim_state, cur_obs, prng_key, rnn_states, sim_ctrl,
                 env_returns, counters, policy_assignments, native_step=None):
        self.cfg = cfg
        self.step_fn = step_fn
        # the built-in synthetic sim's fused step (envs.DummyVecEnv.native_step),
        # or None: the sim's 'step' runs between the policy launches
        self.native_step = native_step
        self.sim_state = sim_state
        self.cur_obs = cur_obs
        self.prng_key = prng_key
        self.rnn_states = rnn_states
        self.sim_ctrl = sim_ctrl
        self.env_returns = env_returns
        self.counters = counters  # device int64[8]: [0] rollout step, [1] epoch
        self.policy_assignments = policy_assignments

    @staticmethod
    def create(rollout_cfg, sim_fns, prng_key, rnn_states, init_sim_ctrl,
               static_play_assignments=None, device="cuda"):
        init_out = sim_fns["init"]()
        dev = torch.device(device)
        return RolloutState(
            cfg=rollout_cfg,
            step_fn=sim_fns["step"],
            sim_state=init_out["state"],
            cur_obs=init_out["obs"],
            prng_key=prng_key,
            rnn_states=rnn_states,
            sim_ctrl=init_sim_ctrl,
            env_returns=torch.zeros(rollout_cfg.sim_batch_size, dtype=torch.float32, device=dev),
            counters=torch.zeros(8, dtype=torch.int64, device=dev),
            # self-play: every agent runs policy 0 (pbt.py:130-133)
            policy_assignments=torch.zeros((rollout_cfg.sim_batch_size, 1), dtype=torch.int32,
                                           device=dev),
            native_step=sim_fns.get("native_step"),
        )


class RolloutData:  # rollouts.py:311-334
    """Views of the [T][N] store.  ``minibatch`` gathers whole sequences
    ([T/C, mb, ...], time-major) like the reference for user hooks; the PPO
    kernels never materialise it."""

    def __init__(self, store, num_bptt_chunks):
        self.store = store
        self.C = num_bptt_chunks

    def all(self):
        return self.store.as_dict()

    def minibatch(self, indices):
        s = self.store
        T, N, C = s.T, s.N, self.C
        Tc = T // C
        idx = indices.to(torch.int64)
        c, b = idx // N, idx % N
        t = (c[None, :] * Tc + torch.arange(Tc, device=idx.device)[:, None])  # [Tc, mb]
        rows = t * N + b[None, :]
        out = {}
        for k, v in s.as_dict().items():
            flat = v.reshape(T * N, *v.shape[2:])
            out[k] = flat[rows.reshape(-1)].reshape(Tc, idx.numel(), *v.shape[2:])
        return out


class RolloutStore:
    def __init__(self, T, N, obs_dim, K, compute_dtype, device, num_chunks=1, rnn_hidden=0):
        self.T, self.N = T, N
        f32 = torch.float32
        self.obs = torch.zeros((T, N, obs_dim), dtype=compute_dtype, device=device)
        self.actions = torch.zeros((T, N, K), dtype=torch.int32, device=device)
        self.log_probs = torch.zeros((T, N, K), dtype=f32, device=device)
        self.values = torch.zeros((T, N), dtype=f32, device=device)
        self.rewards = torch.zeros((T, N), dtype=f32, device=device)
        self.dones = torch.zeros((T, N), dtype=torch.uint8, device=device)
        self.advantages = torch.zeros((T, N), dtype=f32, device=device)
        # returns = advantages + values (rollouts.py:761-769).  With
        # derive_returns (GAE path without a value normaliser) the GAE writes
        # only the advantages and every consumer forms the sum (the same f32
        # addition): the [T][N] column below is then not written and
        # `returns` reads as advantages + values
        self._returns = torch.zeros((T, N), dtype=f32, device=device)
        self.derive_returns = False
        self.env_returns_trace = torch.zeros((T, N), dtype=f32, device=device)
        self.bootstrap = torch.zeros((N,), dtype=f32, device=device)
        # rnn_start_states (rollouts.py:528-537): the carry entering every BPTT
        # chunk, [C][N][H] in the compute dtype (recurrent policies only)
        self.start_h = self.start_c = None
        if rnn_hidden:
            self.start_h = torch.zeros((num_chunks, N, rnn_hidden), dtype=compute_dtype,
                                       device=device)
            self.start_c = torch.zeros_like(self.start_h)

    @property
    def returns(self):
        return self.advantages + self.values if self.derive_returns else self._returns

    def as_dict(self, targets=True):
        """The store leaves; ``targets=False`` leaves out 'advantages' and
        'returns' (the rollout before compute_advantages, as the reference
        hands it to TrainHooks.finish_rollouts, rollouts.py:743-745)."""
        d = {"obs": self.obs, "actions": self.actions, "log_probs": self.log_probs,
             "values": self.values, "rewards": self.rewards, "dones": self.dones}
        if targets:
            d["advantages"] = self.advantages
            d["returns"] = self.returns
        return d

    def view(self, bptt_len, col0=0, ncols=None):
        """Rollout view of env columns [col0, col0 + ncols) (one policy of a
        population; the whole store by default)."""
        ncols = self.N - col0 if ncols is None else ncols
        assert 0 <= col0 and col0 + ncols <= self.N
        D = self.obs.shape[2]
        K = self.actions.shape[2]
        v = nat.RolloutView()
        v.obs = self.obs.data_ptr() + col0 * D * self.obs.element_size()
        v.actions = self.actions.data_ptr() + col0 * K * 4
        v.log_probs = self.log_probs.data_ptr() + col0 * K * 4
        v.advantages = self.advantages.data_ptr() + col0 * 4
        v.returns = None if self.derive_returns else self._returns.data_ptr() + col0 * 4
        v.values = self.values.data_ptr() + col0 * 4
        v.dones = self.dones.data_ptr() + col0
        v.T = self.T
        v.bptt_len = bptt_len
        v.N = ncols
        v.ld = self.N
        return v


# (order of the metric jobs below; 'Advantages' only with compute_advantages,
# rollouts.py:482-499)
ROLLOUT_METRICS = ["Rewards", "Values", "Est Returns", "Env Returns", "Bootstrap Values",
                   "Advantages"]


def obs_to_matrix(obs, N):
    """Identity prefix: a tensor, or a dict holding exactly one tensor."""
    if isinstance(obs, dict):
        if len(obs) != 1:
            raise ValueError("obs dict with several entries needs a BackboneShared prefix "
                             "that returns one [N, obs_dim] tensor")
        obs = next(iter(obs.values()))
    x = obs.reshape(N, -1)
    if x.dtype != torch.float32:
        x = x.float()
    return x.contiguous()


class RolloutManager:  # rollouts.py:373-826
    """Runs the rollout of every train policy on this rank.  ``policy_states``
    is one PolicyState, or a list of them for a population: policy p owns the
    contiguous env columns [p*B, (p+1)*B) of the rank's N envs (the self-play
    split of pbt_init_matchmaking, pbt.py:130-133) and writes those columns
    of the shared [T][N] store, so the sim steps all N envs at once and GAE
    runs over the whole store in one launch.

    Launch shape of the built-in sim's rollout (same bits in every form):
    ``whole_rollout`` (default True) runs every step and the bootstrap in one
    launch per policy (mlearn_policy_rollout_env); False issues one
    rollout_step_env call per step from the host.  ``rollout_workgroups`` is
    that launch's mlearn_rollout_out.max_workgroups: 0 one workgroup per
    resident slot, > 0 at most that many (env tiles in series), < 0 the
    entry's own per-step launches.  ``population_launch`` (default True): a
    population's whole rollouts go out as ONE launch over every policy's env
    tiles (mlearn_policy_rollout_env_pop), so P launches of B / 32 workgroups
    each become one that fills the chip; False issues one launch per policy.
    A ``rollout_workgroups`` cap > 0 caps that launch too (tiles of several
    policies in series per workgroup).  Same bits either way while both
    launches run the same kernel: with ``rollout_kernel`` 0 an uncapped
    population launch may take the row-split kernel where the per-policy
    launches or a capped population launch take the feature split (the row
    split needs >= 65 536 envs per launch, the population form >= 2 048 16-env
    tiles in all), and the two kernels' logits may differ by a bf16 ulp, so
    a sampled action may differ where two perturbed logits nearly tie; set
    ``rollout_kernel`` = 1 for bit-identical trajectories across these
    switches.
    ``rollout_kernel`` is mlearn_rollout_out.policy_kernel of the whole-rollout
    launch: 0 the library's choice (the row-split rollout at the headline
    shape, include/mlearn.h), 1 the feature-split kernel (the per-step
    launches' body: bit-identical to them), 2 the row-split kernel.  The
    population launch follows it too (mlearn_policy_rollout_pop_kernel: the
    row split uncapped where it applies; 1 runs the feature split on its own
    grid, 2 raises where the row split does not apply)."""

    whole_rollout = True
    # GAE inside the single-policy whole-rollout launch where it applies
    # (mlearn_rollout_out.advantages); False: always its own launch (A/B runs)
    fused_gae = True
    rollout_workgroups = 0
    rollout_kernel = 0
    population_launch = True

    def __init__(self, train_cfg, init_rollout_state: RolloutState, policy_states, env_offset=0):
        self.train_cfg = train_cfg
        self._cfg = init_rollout_state.cfg
        assert train_cfg.steps_per_update % train_cfg.num_bptt_chunks == 0  # rollouts.py:387
        self.T = train_cfg.steps_per_update
        self.C = train_cfg.num_bptt_chunks
        self.bptt = self.T // self.C
        self.N = self._cfg.sim_batch_size
        self.policies = list(policy_states) if isinstance(policy_states, (list, tuple)) \
            else [policy_states]
        self.P = len(self.policies)
        if self.N % self.P != 0:
            raise ValueError(f"{self.N} envs do not split over {self.P} policies")
        self.B = self.N // self.P
        self.policy_state = self.policies[0]
        self.prefix = getattr(self.policy_state.actor_critic.backbone, "prefix", None)
        for ps in self.policies:
            ps.attach_obs_stats(self.T, self.N // len(self.policies))
        arch = self.policy_state.arch
        for ps in self.policies[1:]:
            assert ps.arch == arch, "population policies must share one architecture"
        self.store = RolloutStore(self.T, self.N, arch.obs_dim, arch.num_groups, arch.dtype,
                                  self.policy_state.device, self.C, arch.lstm_hidden)
        # GAE without a value normaliser: returns not materialised (RolloutStore)
        self.store.derive_returns = bool(train_cfg.compute_advantages and
                                         not train_cfg.normalize_values)
        self.R = arch.lstm_hidden
        if self.R:
            # the live recurrent carry (c_states, h_states) of rollouts.py:898-901,
            # one layer, [N][H] compute dtype, kept in the rollout state
            rs = init_rollout_state.rnn_states
            ok = (isinstance(rs, (tuple, list)) and len(rs) == 2 and len(rs[0]) == 1 and
                  all(isinstance(x[0], torch.Tensor) and x[0].shape == (self.N, self.R) and
                      x[0].dtype == arch.dtype and x[0].device == self.policy_state.device and
                      x[0].is_contiguous() for x in rs))
            if not ok:
                z = lambda: torch.zeros((self.N, self.R), dtype=arch.dtype,  # noqa: E731
                                        device=self.policy_state.device)
                init_rollout_state.rnn_states = ([z()], [z()])
            self._carries = {}
        self.env_offset = int(env_offset)
        self.use_advantages = train_cfg.compute_advantages
        dev = self.policy_state.device
        self._resets = torch.zeros((self._cfg.num_worlds, 1), dtype=torch.int32, device=dev)
        self._metrics_ws = torch.zeros(int(nat.lib().mlearn_metrics_workspace_bytes(6)),
                                       dtype=torch.uint8, device=dev)
        s = self.store
        TN = self.T * self.B
        self._jobs = []
        self._nmet = len(ROLLOUT_METRICS) - (0 if self.use_advantages else 1)
        for p in range(self.P):
            c0 = p * self.B
            jobs = (nat.MetricJob * 6)()
            srcs = [(s.rewards, TN, self.B), (s.values, TN, self.B), (s._returns, TN, self.B),
                    (s.env_returns_trace, TN, self.B), (s.bootstrap, self.B, 0),
                    (s.advantages, TN, self.B)]
            for i, (x, n, cols) in enumerate(srcs[:self._nmet]):
                jobs[i].x = x.data_ptr() + c0 * 4
                if i == 2 and s.derive_returns:  # 'Est Returns' = values + advantages
                    jobs[i].x = s.values.data_ptr() + c0 * 4
                    jobs[i].x2 = s.advantages.data_ptr() + c0 * 4
                jobs[i].n = n
                jobs[i].cols = cols if self.P > 1 else 0
                jobs[i].ld = self.N
                jobs[i].abs_value = 0
            self._jobs.append(jobs)

    def view(self, p=0):
        """Rollout view of policy p's env columns.  With compute_advantages=False
        the surrogate objective reads the returns (ppo.py:139-143): the view's
        advantage column is the returns column."""
        v = self.store.view(self.bptt, p * self.B, self.B)
        if not self.use_advantages:
            v.advantages = v.returns
        return v

    def start_states(self, p=0):
        """Device pointers of policy p's rnn_start_states columns ([C][ld][H],
        ld = the store's N), as the recurrent minibatch kernel reads them."""
        s = self.store
        off = p * self.B * self.R * s.start_h.element_size()
        return s.start_h.data_ptr() + off, s.start_c.data_ptr() + off

    def _carry(self, rollout_state, p, t):
        """LstmCarry of policy p at env step t (t = T: the bootstrap critic,
        which clears the carry where the last step ended an episode but does
        not advance it)."""
        key = (p, t)
        d = self._carries.get(key)
        c_states, h_states = rollout_state.rnn_states
        h, c = h_states[0], c_states[0]
        if d is None or d.h != h.data_ptr() + p * self.B * self.R * h.element_size():
            d = nat.LstmCarry()
            es = h.element_size()
            d.h = h.data_ptr() + p * self.B * self.R * es
            d.c = c.data_ptr() + p * self.B * self.R * es
            if t < self.T and t % self.bptt == 0:
                sh = self.store.start_h[t // self.bptt, p * self.B:(p + 1) * self.B]
                sc = self.store.start_c[t // self.bptt, p * self.B:(p + 1) * self.B]
                d.start_h, d.start_c = sh.data_ptr(), sc.data_ptr()
            d.commit = 1 if t < self.T else 0
            self._carries[key] = d
        return d

    def _sim_actions(self, t):
        """The sim's 'actions' input of step t: the [N, K] store slice, or with
        several action groups a dict keyed like TrainConfig.actions of [N, K_g]
        views (rollouts.py:985-1002)."""
        from .models import action_groups
        if not hasattr(self, "_act_groups"):
            self._act_groups = action_groups(self.train_cfg.actions)
        a = self.store.actions[t]
        if len(self._act_groups) == 1:
            return a
        out, off = {}, 0
        for name, b in self._act_groups:
            out[name] = a[:, off:off + len(b)]
            off += len(b)
        return out

    def _env_desc(self, sim, p):
        """nat.DummyEnv of policy p's env columns (cached per sim)."""
        key = (id(sim), p)
        if not hasattr(self, "_env_descs"):
            self._env_descs = {}
        d = self._env_descs.get(key)
        if d is None:
            d = sim.native_step(p * self.B, self.B)
            self._env_descs[key] = d
        return d

    def add_metrics(self, train_cfg, names):  # rollouts.py:482-499
        return list(names) + ROLLOUT_METRICS[:self._nmet]

    def prep_obs(self, obs):
        x = self.prefix(obs, train=False)
        pre = self.policy_state.obs_preprocess
        if hasattr(pre, "prep_fns") and pre.prep_fns and isinstance(x, dict) and len(x) == 1:
            k = next(iter(x))
            x = {k: pre.prep(k, x[k])}  # ObservationsEMANormalizer prep_fns (observations.py:99-101)
        return obs_to_matrix(x, self.N)

    def _post_desc(self, t, p, rew, dn, rollout_state, gamma):
        """Post-step descriptor of env step t for policy p's columns
        (rollouts.py:933-973); the tensors it points at are kept alive until
        the next collect."""
        s = self.store
        if not hasattr(self, "_posts"):
            self._posts = [[nat.PostStep() for _ in range(self.P)] for _ in range(self.T)]
            self._post_keep = [None] * self.T
        c = slice(p * self.B, (p + 1) * self.B)
        d = self._posts[t][p]
        d.rewards, d.dones = nat.ptr(rew[c]), nat.ptr(dn[c])
        d.store_rewards, d.store_dones = nat.ptr(s.rewards[t, c]), nat.ptr(s.dones[t, c])
        d.env_returns = nat.ptr(rollout_state.env_returns[c])
        d.env_returns_trace = nat.ptr(s.env_returns_trace[t, c])
        d.gamma = gamma
        self._post_keep[t] = (rew, dn)
        return d

    def collect(self, train_state_mgr, rollout_state: RolloutState, metrics, user_hooks):
        """rollouts.py:501-577 restated on the fused kernels."""
        s = self.store
        L = nat.lib()
        strm = nat.stream_handle()
        gamma = float(self._cfg.reward_gamma)
        rollout_state, train_state_mgr.user_state = user_hooks.start_rollouts(
            rollout_state, train_state_mgr.user_state)
        if getattr(self.policy_state, "generic", False):
            # a tree outside the fused kernels: torch modules per step (generic.py)
            from .generic import TorchRollout
            TorchRollout(self).collect(rollout_state, gamma)
            return self._finish(train_state_mgr, rollout_state, metrics, user_hooks)
        key = rollout_state.prng_key
        step_ctr = rollout_state.counters[0:1]
        B = self.B
        posts = [None] * self.P  # post-step of env step t-1, fused into the policy launches of t
        sim = rollout_state.native_step
        obs0 = self.prep_obs(rollout_state.cur_obs)
        if sim is not None and obs0.data_ptr() == sim.obs.data_ptr() and self.whole_rollout:
            # the built-in sim: every step + the bootstrap in one launch per
            # policy, or one launch for the whole population
            if not self._population_rollout(rollout_state, obs0, sim, key, step_ctr, gamma):
                # one policy: GAE rides the rollout launch (mlearn_rollout_out.advantages:
                # fused into the row-split kernel's epilogue) where nothing may
                # change the rollout between the two (no finish_rollouts hook, no
                # value normaliser, advantages only)
                fuse = self.P == 1 and self._gae_in_rollout(train_state_mgr, user_hooks)
                for p, ps in enumerate(self.policies):
                    c = slice(p * B, (p + 1) * B)
                    o = self._rollout_out(rollout_state, p, gamma)
                    if fuse:
                        from .algo_common import _gamma_lambda
                        o.advantages = s.advantages.data_ptr()
                        o.gae_gamma = float(self.train_cfg.gamma)
                        o.gae_gamma_lambda = _gamma_lambda(self.train_cfg)
                    else:
                        o.advantages = None
                    ps.rollout_all(obs0[c], o, key,
                                   step_ctr, self.env_offset + p * B, self._env_desc(sim, p),
                                   carry=self._carry(rollout_state, p, 0) if self.R else None)
                self._gae_done = fuse
            out = sim.native_outputs()
            rollout_state.sim_state = out["state"]
            rollout_state.cur_obs = out["obs"]
            return self._finish(train_state_mgr, rollout_state, metrics, user_hooks)
        for t in range(self.T):
            obs = self.prep_obs(rollout_state.cur_obs)
            # the built-in sim steps inside the policy launches when they read
            # its observation buffer directly (no preprocessing copy)
            fused = sim is not None and obs.data_ptr() == sim.obs.data_ptr()
            for p, ps in enumerate(self.policies):
                c = slice(p * B, (p + 1) * B)
                ps.rollout_step(obs[c], s.obs[t, c], s.actions[t, c], s.log_probs[t, c],
                                s.values[t, c], key, step_ctr, t, self.env_offset + p * B,
                                sample=True, post=posts[p],
                                carry=self._carry(rollout_state, p, t) if self.R else None,
                                env=self._env_desc(sim, p) if fused else None)
            if fused:
                out = sim.native_outputs()
            else:
                step_input = {
                    "state": rollout_state.sim_state,
                    "actions": self._sim_actions(t),
                    "resets": self._resets,
                    "sim_ctrl": rollout_state.sim_ctrl,
                    "pbt": {"policy_assignments": rollout_state.policy_assignments},
                }
                out = rollout_state.step_fn(step_input)
            rew = out["rewards"].reshape(-1)
            if rew.dtype != torch.float32:
                rew = rew.float()
            dn = out["dones"].reshape(-1)
            dn = dn.view(torch.uint8) if dn.dtype == torch.bool else (dn != 0).view(torch.uint8)
            rew, dn = rew.contiguous(), dn.contiguous()
            posts = [self._post_desc(t, p, rew, dn, rollout_state, gamma)
                     for p in range(self.P)]
            rollout_state.sim_state = out["state"]
            rollout_state.cur_obs = out["obs"]
            # population fitness from the episodes that ended (pbt_update_fitness,
            # pbt.py:382-470; episode_results from the sim's 'pbt' output)
            res = (out.get("pbt") or {}).get("episode_results")
            if res is not None and getattr(self, "get_episode_scores", None) is not None:
                from .pbt import pbt_update_fitness
                pbt_update_fitness([(ps.episode_score, p * B, B)
                                    for p, ps in enumerate(self.policies)],
                                   self.get_episode_scores(res), dn,
                                   team_size=self.train_cfg.num_agents_per_world)
        # bootstrap values (rollouts.py:607-635), with the last post-step
        obs = self.prep_obs(rollout_state.cur_obs)
        for p, ps in enumerate(self.policies):
            c = slice(p * B, (p + 1) * B)
            ps.critic_only(obs[c], s.bootstrap[c], post=posts[p],
                           carry=self._carry(rollout_state, p, self.T) if self.R else None)
        return self._finish(train_state_mgr, rollout_state, metrics, user_hooks)

    def _population_rollout(self, rollout_state, obs0, sim, key, step_ctr, gamma):
        """mlearn_policy_rollout_env_pop over every policy's env columns; False
        when the per-policy launches must run instead (one policy, the
        population launch switched off, per-step launches asked for
        (rollout_workgroups < 0), or the launch arguments changed while a
        graph is being captured)."""
        cap = int(self.rollout_workgroups)
        if self.P < 2 or not self.population_launch or cap < 0:
            return False
        B, P = self.B, self.P
        outs = [self._rollout_out(rollout_state, p, gamma) for p in range(P)]
        for o in outs:  # the population launch takes its cap as an argument
            o.max_workgroups = 0
        envs = [self._env_desc(sim, p) for p in range(P)]
        descs = [ps.desc for ps in self.policies]
        lstms = [ps.lstm_desc for ps in self.policies] if self.R else None
        carries = [self._carry(rollout_state, p, 0) for p in range(P)] if self.R else None
        obs = [obs0[p * B:(p + 1) * B].data_ptr() for p in range(P)]
        offs = [self.env_offset + p * B for p in range(P)]
        parts = descs + outs + envs + (lstms or []) + (carries or [])
        sig = b"".join(bytes(x) for x in parts) + repr((obs, offs)).encode()
        L = nat.lib()
        if getattr(self, "_pop_sig", None) != sig:
            if torch.cuda.is_current_stream_capturing():
                return False  # (the prepare copy cannot run inside a capture)
            if getattr(self, "_pop_buf", None) is None:
                self._pop_buf = torch.empty(int(L.mlearn_policy_pop_bytes(P)), dtype=torch.uint8,
                                            device=self.policy_state.device)
            arr = lambda T, xs: (T * P)(*xs)  # noqa: E731
            nat.check(L.mlearn_policy_pop_prepare(
                arr(nat.MlpPolicy, descs), arr(nat.Lstm, lstms) if lstms else None,
                arr(nat.LstmCarry, carries) if carries else None, (nat.c_void_p * P)(*obs), B,
                arr(nat.RolloutOut, outs), (nat.c_uint32 * P)(*offs), arr(nat.DummyEnv, envs), P,
                nat.ptr(self._pop_buf), nat.stream_handle()), "policy_pop_prepare")
            self._pop_sig = sig
        lstm0 = self.policy_state.lstm_desc if self.R else None
        kern = int(L.mlearn_policy_rollout_pop_kernel(self.policy_state.desc, lstm0, B, P, cap))
        if self.rollout_kernel == 1 and kern == 2:
            # the feature split on the grid it takes uncapped
            cap = int(L.mlearn_policy_rollout_pop_workgroups(self.policy_state.desc, lstm0, B, P, 0))
        elif self.rollout_kernel == 2 and kern != 2:
            raise RuntimeError("rollout_kernel 2: the row-split population rollout does not apply "
                               f"({P} policies x {B} envs, cap {cap})")
        nat.check(L.mlearn_policy_rollout_env_pop(
            self.policy_state.desc, lstm0, nat.ptr(self._pop_buf), P, B, key[0], key[1],
            nat.ptr(step_ctr), cap, nat.stream_handle()), "policy_rollout_env_pop")
        return True

    def _gae_in_rollout(self, train_state_mgr, user_hooks):
        """Whether the advantages can be computed by the rollout launch itself:
        the GAE objective with returns derived (no value normaliser) and the
        default finish_rollouts hook (which would otherwise see, and may
        rewrite, the rollout before the advantages exist)."""
        from .train import TrainHooks
        return bool(self.use_advantages and self.store.derive_returns and
                    train_state_mgr.value_norm is None and self.fused_gae and
                    type(user_hooks).finish_rollouts is TrainHooks.finish_rollouts)

    def _rollout_out(self, rollout_state, p, gamma):
        """nat.RolloutOut of policy p's store columns (cached)."""
        if not hasattr(self, "_routs"):
            self._routs = {}
        s = self.store
        key = (p, rollout_state.env_returns.data_ptr())
        o = self._routs.get(key)
        if o is None:
            c0 = p * self.B
            o = nat.RolloutOut()
            o.obs = s.obs.data_ptr() + c0 * s.obs.shape[2] * s.obs.element_size()
            o.actions = s.actions.data_ptr() + c0 * s.actions.shape[2] * 4
            o.log_probs = s.log_probs.data_ptr() + c0 * s.log_probs.shape[2] * 4
            o.values = s.values.data_ptr() + c0 * 4
            o.rewards = s.rewards.data_ptr() + c0 * 4
            o.dones = s.dones.data_ptr() + c0
            o.env_returns_trace = s.env_returns_trace.data_ptr() + c0 * 4
            o.bootstrap = s.bootstrap.data_ptr() + c0 * 4
            o.env_returns = rollout_state.env_returns.data_ptr() + c0 * 4
            if self.R:
                es = s.start_h.element_size()
                o.start_h = s.start_h.data_ptr() + c0 * self.R * es
                o.start_c = s.start_c.data_ptr() + c0 * self.R * es
            o.T, o.bptt_len, o.ld, o.gamma = self.T, self.bptt, self.N, gamma
            self._routs[key] = o
        o.max_workgroups = int(self.rollout_workgroups)
        o.policy_kernel = int(self.rollout_kernel)
        return o

    def _finish(self, train_state_mgr, rollout_state, metrics, user_hooks):
        s = self.store
        L = nat.lib()
        strm = nat.stream_handle()
        # obs statistics -> normaliser estimates for the next rollout
        # (update_state, train.py:193-204; the update trains on the stored,
        # already normalised observations)
        for ps in self.policies:
            ps.update_obs_norm()
        from .train import TrainHooks
        if type(user_hooks).finish_rollouts is not TrainHooks.finish_rollouts:
            # rollouts.py:726-745: the hook sees the rollout before the
            # advantages exist, plus the critic outputs inverted by the value
            # normaliser; leaves it returns in place of the store's are copied
            # back (e.g. reshaped rewards), so the GAE below uses them
            vals, boot = s.values, s.bootstrap
            vn = train_state_mgr.value_norm
            if vn is not None:  # EMANormalizer.invert: v * sigma + mu per policy
                sig = vn[:, 2].repeat_interleave(self.B)
                mu = vn[:, 0].repeat_interleave(self.B)
                vals, boot = s.values * sig + mu, s.bootstrap * sig + mu
            before = s.as_dict(targets=False)
            rollouts, train_state_mgr.user_state = user_hooks.finish_rollouts(
                dict(before), s.bootstrap, vals, boot, train_state_mgr.user_state)
            for k, v in (rollouts or {}).items():
                if k in before and v is not before[k]:
                    before[k].copy_(v.reshape(before[k].shape))
        if getattr(self, "_gae_done", False):
            self._gae_done = False  # (the rollout launch wrote the advantages)
        elif self.use_advantages:
            compute_advantages(self.train_cfg, s.rewards, s.values, s.dones, s.bootstrap,
                               out_adv=s.advantages,
                               out_ret=False if s.derive_returns else s._returns,
                               value_norm=train_state_mgr.value_norm, norm_cols=self.B)
        else:
            compute_returns(self.train_cfg, s.rewards, s.dones, s.bootstrap, out=s._returns)
        for p in range(self.P):
            nat.check(L.mlearn_metrics_f32(self._jobs[p], self._nmet,
                                           nat.ptr(metrics.slots("Rewards", self._nmet, policy=p)),
                                           nat.ptr(self._metrics_ws), strm), "rollout metrics")
        nat.check(L.mlearn_counters_add(nat.ptr(rollout_state.counters), 1,
                                        (nat.c_uint64 * 1)(self.T), strm), "counters")
        data = RolloutData(s, self.C)
        metrics = user_hooks.rollout_metrics(metrics, data, train_state_mgr.user_state)
        return train_state_mgr, rollout_state, data, None, metrics
