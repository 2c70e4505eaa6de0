"""Policy / train state (mirrors src/madrona_learn/train_state.py:34-488).

``compile_policy`` recognises the ActorCritic tree the fused kernels
implement and builds a ``PolicyState``: one flat f32 parameter arena in HBM
(layout of ``mlearn_param_count``) plus the compute-dtype weight images the
kernels read, all bound into one ``mlearn_mlp_policy`` descriptor.
``PolicyTrainState`` holds Adam moments, the Adam step counter, the initial
weight norms (train_state.py:413-423) and the minibatch RNG key.
"""

import math
from dataclasses import dataclass, field
from typing import Any, Optional

import numpy as np

import torch

from . import _native as nat
from .actor_critic import (ActorCritic, BackboneEncoder, BackboneShared,
                           RecurrentBackboneEncoder)
from .cfg import DiscreteActionsConfig, TrainConfig
from .models import MLP, DenseLayerCritic, DenseLayerDiscreteActor, DreamerV3Critic
from .observations import ObservationsEMANormalizer, ObservationsPreprocessNoop
from .rnn import LSTM


@dataclass(frozen=True)
class MlpArch:
    obs_dim: int
    hidden: int
    num_layers: int
    buckets: tuple
    dtype: torch.dtype
    lstm_hidden: int = 0  # width of the LSTM after the trunk (0: feed-forward policy)
    critic_bins: int = 1  # 1: DenseLayerCritic; odd > 1: DreamerV3Critic two-hot bins

    @property
    def num_logits(self):
        return int(sum(self.buckets))

    @property
    def head_cols(self):
        return nat.head_cols(self.num_logits, self.critic_bins)

    @property
    def num_groups(self):
        return len(self.buckets)


def param_layout(arch: MlpArch):
    """Python mirror of LayoutK / mlearn_param_count (csrc/ppo.hip)."""
    H, A1 = arch.hidden, arch.num_logits + arch.critic_bins
    off = 0
    lay = {"w": [], "s": [], "b": []}
    for l in range(arch.num_layers):
        fin = arch.obs_dim if l == 0 else H
        lay["w"].append((off, (fin, H)))
        off += fin * H
        lay["s"].append((off, (H,)))
        off += H
        lay["b"].append((off, (H,)))
        off += H
    lay["hw"] = (off, (H, A1))
    off += H * A1
    lay["hb"] = (off, (A1,))
    off += A1
    if arch.lstm_hidden:
        # mlearn_lstm_param_offset: the LSTM segment starts 64-float aligned
        R = arch.lstm_hidden
        off = (off + 63) // 64 * 64
        lay["lstm_off"] = off
        lay["wi"] = (off, (H, 4 * R))   # input kernels ii | if | ig | io
        off += 4 * R * H
        lay["wr"] = (off, (R, 4 * R))   # hidden kernels hi | hf | hg | ho
        off += 4 * R * R
        lay["bl"] = (off, (4 * R,))     # hidden-kernel biases
        off += 4 * R
    lay["total"] = off
    return lay


def _actions_buckets(actor, cfg_actions):
    if not isinstance(actor, DenseLayerDiscreteActor):
        raise NotImplementedError(
            "fused path supports DenseLayerDiscreteActor (models.py:122-139); got "
            f"{type(actor).__name__}")
    return tuple(int(b) for b in actor.buckets)


def compile_arch(actor_critic: ActorCritic, obs_dim: int, compute_dtype) -> MlpArch:
    bb = actor_critic.backbone
    enc = bb.encoder if isinstance(bb, BackboneShared) else bb
    lstm_hidden = 0
    if isinstance(enc, RecurrentBackboneEncoder):
        rnn = enc.rnn
        if not isinstance(rnn, LSTM):
            raise NotImplementedError(f"recurrent fused path needs rnn.LSTM, got "
                                      f"{type(rnn).__name__}")
        if rnn.num_layers != 1:
            raise NotImplementedError("recurrent fused path: one LSTM layer (rnn.py:10-45)")
        if rnn.num_hidden_channels != getattr(enc.net, "num_channels", None):
            raise NotImplementedError("recurrent fused path: LSTM width must equal the MLP "
                                      "width")
        lstm_hidden = rnn.num_hidden_channels
    elif not isinstance(enc, BackboneEncoder):
        raise NotImplementedError(
            "fused path supports BackboneShared(encoder=BackboneEncoder(net=MLP)) and "
            "RecurrentBackboneEncoder(net=MLP, rnn=LSTM) (actor_critic.py:131-244); "
            "separate backbones are outside the fused path")
    net = enc.net
    if not isinstance(net, MLP):
        raise NotImplementedError(f"fused path needs an MLP trunk, got {type(net).__name__}")
    # the shapes the kernels are instantiated for (csrc/policy.hip
    # validate_policy); any other MLP (models.py:99-119 takes any width and
    # depth) trains on the torch path
    if net.num_channels not in (64, 128, 256) or not 1 <= net.num_layers <= nat.MAX_LAYERS:
        raise NotImplementedError(f"fused path: MLP width 64 / 128 / 256 and 1..{nat.MAX_LAYERS} "
                                  f"layers, got {net.num_channels} x {net.num_layers}")
    if not (16 <= int(obs_dim) <= 256 and int(obs_dim) % 16 == 0):
        raise NotImplementedError(f"fused path: observation width a multiple of 16 in "
                                  f"[16, 256], got {obs_dim}")
    critic = actor_critic.critic
    if isinstance(critic, DenseLayerCritic):
        critic_bins = 1
    elif isinstance(critic, DreamerV3Critic):
        critic_bins = int(critic.num_bins)
        if critic_bins < 3 or critic_bins % 2 != 1:
            raise ValueError(f"DreamerV3Critic num_bins must be odd and > 1 (dists.py:131), "
                             f"got {critic_bins}")
    else:
        raise NotImplementedError(
            "fused path supports DenseLayerCritic (models.py:142-154) and DreamerV3Critic "
            f"(157-174); got {type(critic).__name__}")
    buckets = _actions_buckets(actor_critic.actor, None)
    arch = MlpArch(obs_dim=int(obs_dim), hidden=net.num_channels, num_layers=net.num_layers,
                   buckets=buckets, dtype=compute_dtype, lstm_hidden=lstm_hidden,
                   critic_bins=critic_bins)
    arch.head_cols  # raises when the head does not fit
    return arch


class PolicyState:
    """Parameters + compute images of one policy (train_state.py:34-82)."""

    def __init__(self, actor_critic, arch: MlpArch, obs_preprocess, device, rng, obs_key=None):
        self.actor_critic = actor_critic
        self.arch = arch
        self.obs_preprocess = obs_preprocess or ObservationsPreprocessNoop.create()
        self.device = torch.device(device)
        self.layout = param_layout(arch)
        H, D, L, A1 = arch.hidden, arch.obs_dim, arch.num_layers, arch.num_logits + arch.critic_bins
        dt = arch.dtype

        host = np.zeros(self.layout["total"], dtype=np.float32)
        enc = actor_critic.backbone.encoder if isinstance(
            actor_critic.backbone, BackboneShared) else actor_critic.backbone
        net = enc.net
        init_norms = []
        for l in range(L):
            o, shp = self.layout["w"][l]
            w = net.weight_init(rng, shp)
            host[o:o + w.size] = w.reshape(-1)
            init_norms.append(float(np.linalg.norm(w.astype(np.float64))))
            o, shp = self.layout["s"][l]
            host[o:o + H] = 1.0
        o, _ = self.layout["hw"]
        wa = actor_critic.actor.weight_init(rng, (H, arch.num_logits))
        wv = actor_critic.critic.weight_init(rng, (H, arch.critic_bins))
        host[o:o + H * A1] = np.concatenate([wa, wv], axis=1).reshape(-1)
        if arch.lstm_hidden:
            # OptimizedLSTMCell (rnn.py:30-36): orthogonal per gate kernel, zero bias;
            # every gate kernel is projected to its own initial norm (ppo.py:303-310)
            R = arch.lstm_hidden
            for key, init in (("wi", enc.rnn.cell.kernel_init),
                              ("wr", enc.rnn.cell.recurrent_kernel_init)):
                o, (fin, _) = self.layout[key]
                blocks = [init(rng, (fin, R)) for _ in range(4)]
                host[o:o + fin * 4 * R] = np.concatenate(blocks, axis=1).reshape(-1)
                init_norms += [float(np.linalg.norm(b.astype(np.float64))) for b in blocks]

        self.params = torch.from_numpy(host).to(self.device)
        self.init_norms = torch.tensor(init_norms, dtype=torch.float32, device=self.device)
        # compute-dtype fragment-order images read by the kernels (frag.py)
        self.w_t, self.w = [], []
        for l in range(L):
            fin = D if l == 0 else H
            self.w_t.append(torch.zeros(H * fin, dtype=dt, device=self.device))
            self.w.append(torch.zeros(fin * H if l > 0 else 0, dtype=dt, device=self.device))
        HC = arch.head_cols
        self.head_t = torch.zeros(HC * H, dtype=dt, device=self.device)
        self.head = torch.zeros(H * HC, dtype=dt, device=self.device)
        self.head_b = torch.zeros((HC,), dtype=torch.float32, device=self.device)

        d = nat.MlpPolicy()
        d.dtype = nat.dtype_code(dt)
        d.obs_dim = D
        d.hidden = H
        d.num_layers = L
        d.critic_bins = arch.critic_bins
        d.actions = nat.action_layout(arch.buckets)
        for l in range(L):
            d.w_t[l] = self.w_t[l].data_ptr()
            d.w[l] = self.w[l].data_ptr() if l > 0 else None
            d.ln_scale[l] = self.params.data_ptr() + 4 * self.layout["s"][l][0]
            d.ln_bias[l] = self.params.data_ptr() + 4 * self.layout["b"][l][0]
        d.head_t = self.head_t.data_ptr()
        d.head = self.head.data_ptr()
        d.head_bias = self.head_b.data_ptr()
        # ObservationsEMANormalizer estimates (init_estimates, moving_avg.py:56-76):
        # [5][D] = mu, inv_sigma, sigma, mu_biased, sigma_sq_biased, + update count
        self.obs_est = self.obs_count = None
        pre = self.obs_preprocess
        if isinstance(pre, ObservationsEMANormalizer) and pre.normalizes(obs_key):
            self.obs_est = torch.zeros((5, D), dtype=torch.float32, device=self.device)
            self.obs_est[1:3] = 1.0
            self.obs_count = torch.zeros(1, dtype=torch.int32, device=self.device)
            d.obs_mu = self.obs_est.data_ptr()
            d.obs_inv_sigma = self.obs_est.data_ptr() + 4 * D
        self.desc = d
        # population fitness (MovingEpisodeScore, train_state.py:359-366)
        from .pbt import MovingEpisodeScore
        self.episode_score = MovingEpisodeScore(self.device)
        self.lstm_desc = None
        if arch.lstm_hidden:
            R = arch.lstm_hidden
            self.lstm_wi_perm = torch.zeros(4 * R * H, dtype=dt, device=self.device)
            self.lstm_wi_nat = torch.zeros(4 * R * H, dtype=dt, device=self.device)
            self.lstm_wh_nat = torch.zeros(4 * R * R, dtype=dt, device=self.device)
            self.lstm_w_bwd = torch.zeros((H + R) * 4 * R, dtype=dt, device=self.device)
            self.head_t_nat = torch.zeros(HC * R, dtype=dt, device=self.device)
            ld = nat.Lstm()
            ld.hidden = R
            ld.num_layers = 1
            ld.wi_perm = self.lstm_wi_perm.data_ptr()
            ld.wi_nat = self.lstm_wi_nat.data_ptr()
            ld.wh_nat = self.lstm_wh_nat.data_ptr()
            ld.w_bwd = self.lstm_w_bwd.data_ptr()
            ld.head_t_nat = self.head_t_nat.data_ptr()
            ld.bias = self.params.data_ptr() + 4 * self.layout["bl"][0]
            self.lstm_desc = ld
            n = nat.lib().mlearn_lstm_param_count(d, ld)
            if nat.lib().mlearn_lstm_param_offset(d) != self.layout["lstm_off"]:
                raise RuntimeError("LSTM parameter offset mismatch")
        else:
            n = nat.lib().mlearn_param_count(d)
        if n != self.layout["total"]:
            raise RuntimeError(f"param layout mismatch: native {n} vs {self.layout['total']}")
        self.sync_weights()

    # -- views --------------------------------------------------------------
    def view(self, key, l=None):
        o, shp = self.layout[key][l] if l is not None else self.layout[key]
        return self.params[o:o + int(np.prod(shp))].view(*shp)

    @property
    def param_tree(self):
        """flax-style nested dict of views into the arena (train_state.py:65)."""
        L, A = self.arch.num_layers, self.arch.num_logits
        net = {}
        for l in range(L):
            net[f"Dense_{l}"] = {"kernel": self.view("w", l)}
            net[f"LayerNorm_{l}"] = {"impl": {"scale": self.view("s", l),
                                              "bias": self.view("b", l)}}
        hw, hb = self.view("hw"), self.view("hb")
        enc = {"net": net}
        if self.arch.lstm_hidden:
            # flax OptimizedLSTMCell leaves ii..io (kernel), hi..ho (kernel, bias)
            R = self.arch.lstm_hidden
            wi, wr, bl = self.view("wi"), self.view("wr"), self.view("bl")
            cell = {}
            for g, name in enumerate("ifgo"):
                cell[f"i{name}"] = {"kernel": wi[:, g * R:(g + 1) * R]}
                cell[f"h{name}"] = {"kernel": wr[:, g * R:(g + 1) * R],
                                    "bias": bl[g * R:(g + 1) * R]}
            enc["rnn"] = {"cell": {"OptimizedLSTMCell_0": cell}}
        return {
            "backbone": {"encoder": enc},
            "actor": {"impl": {"kernel": hw[:, :A], "bias": hb[:A]}},
            "critic": {"Dense_0": {"kernel": hw[:, A:], "bias": hb[A:]}},
        }

    def sync_weights(self):
        if self.lstm_desc is not None:
            nat.check(nat.lib().mlearn_lstm_sync_weights(self.desc, self.lstm_desc,
                                                         nat.ptr(self.params),
                                                         nat.stream_handle()), "sync_weights")
            return
        nat.check(nat.lib().mlearn_policy_sync_weights(self.desc, nat.ptr(self.params),
                                                       nat.stream_handle()), "sync_weights")

    @property
    def recurrent(self):
        return self.lstm_desc is not None

    # -- kernels ------------------------------------------------------------
    def rollout_step(self, obs, obs_store, actions, log_probs, values, key, step_ctr, step,
                     env_offset=0, sample=True, post=None, carry=None, env=None):
        """ActorCritic.rollout + store (actor_critic.py:74-96, rollouts.py:637-668);
        post: optional nat.PostStep of the previous env step; carry: the
        nat.LstmCarry of a recurrent policy; env: optional nat.DummyEnv of the
        built-in synthetic sim, whose step on the sampled actions then runs
        in the same launch (mlearn_policy_rollout_step_env)."""
        N = obs.shape[0]
        L = nat.lib()
        if self.lstm_desc is not None:
            self._check_carry(carry)
            args = (self.desc, self.lstm_desc, carry, nat.ptr(obs, torch.float32, name="obs"), N,
                    nat.ptr(obs_store), nat.ptr(actions), nat.ptr(log_probs), nat.ptr(values),
                    key[0], key[1], nat.ptr(step_ctr), step, env_offset, 1 if sample else 0, post)
            if env is None:
                nat.check(L.mlearn_lstm_policy_rollout_step(*args, nat.stream_handle()),
                          "lstm_policy_rollout_step")
            else:
                nat.check(L.mlearn_lstm_policy_rollout_step_env(*args, env, nat.stream_handle()),
                          "lstm_policy_rollout_step_env")
            return
        args = (self.desc, nat.ptr(obs, torch.float32, name="obs"), N, nat.ptr(obs_store),
                nat.ptr(actions), nat.ptr(log_probs), nat.ptr(values), key[0], key[1],
                nat.ptr(step_ctr), step, env_offset, 1 if sample else 0, post)
        if env is None:
            nat.check(L.mlearn_policy_rollout_step(*args, nat.stream_handle()),
                      "policy_rollout_step")
        else:
            nat.check(L.mlearn_policy_rollout_step_env(*args, env, nat.stream_handle()),
                      "policy_rollout_step_env")

    def rollout_all(self, obs, out, key, step_ctr, env_offset, env, carry=None):
        """The whole rollout of the built-in synthetic sim in one launch
        (mlearn_policy_rollout_env): T rollout steps with the fused env step
        and post-steps, then the bootstrap critic; `out` is the
        nat.RolloutOut of this policy's store columns, `carry` the
        nat.LstmCarry (h, c) of a recurrent policy."""
        if self.lstm_desc is not None:
            self._check_carry(carry)
        N = obs.shape[0]
        nat.check(nat.lib().mlearn_policy_rollout_env(
            self.desc, self.lstm_desc, carry if self.lstm_desc is not None else None,
            nat.ptr(obs, torch.float32, name="obs"), N, out, key[0], key[1], nat.ptr(step_ctr),
            env_offset, env, nat.stream_handle()), "policy_rollout_env")

    def _check_carry(self, carry):
        if not isinstance(carry, nat.LstmCarry) or not carry.h or not carry.c:
            raise ValueError("a recurrent policy needs its LstmCarry (rollout carry h, c)")

    def critic_only(self, obs, values, post=None, carry=None):
        """ActorCritic.critic_only (actor_critic.py:65-72).  A recurrent policy
        runs the cell from the carry without advancing it (carry.commit = 0:
        the carry is only cleared where post's dones are set)."""
        N = obs.shape[0]
        if self.lstm_desc is not None:
            self._check_carry(carry)
            nat.check(nat.lib().mlearn_lstm_policy_rollout_step(
                self.desc, self.lstm_desc, carry, nat.ptr(obs, torch.float32, name="obs"), N,
                None, None, None, nat.ptr(values), 0, 0, None, 0, 0, 0, post,
                nat.stream_handle()), "lstm_critic_only")
            return
        nat.check(nat.lib().mlearn_policy_rollout_step(
            self.desc, nat.ptr(obs, torch.float32, name="obs"), N, None, None, None,
            nat.ptr(values), 0, 0, None, 0, 0, 0, post, nat.stream_handle()), "critic_only")

    def state_dict(self):
        sd = {"params": self.params.detach().cpu(),
              "episode_score": [t.cpu() for t in self.episode_score.tensors()]}
        if self.obs_est is not None:
            sd["obs_est"] = self.obs_est.cpu()
            sd["obs_count"] = self.obs_count.cpu()
        return sd

    def load_state_dict(self, sd):
        self.params.copy_(sd["params"].to(self.device))
        if "episode_score" in sd:
            for a, b in zip(self.episode_score.tensors(), sd["episode_score"]):
                a.copy_(b)
        if self.obs_est is not None and "obs_est" in sd:
            self.obs_est.copy_(sd["obs_est"].to(self.device))
            self.obs_count.copy_(sd["obs_count"].to(self.device))
        self.sync_weights()

    def attach_obs_stats(self, T, B):
        """Per-step tile statistics buffer of the rollout (policy B envs)."""
        if self.obs_est is None:
            return
        tiles = (B + 31) // 32
        D = self.arch.obs_dim
        self.obs_stats = torch.zeros((T, tiles, D, 2), dtype=torch.float32, device=self.device)
        self.desc.obs_stats = self.obs_stats.data_ptr()
        self.desc.obs_stats_tiles = tiles
        self.desc.obs_stats_steps = T
        self._obs_B = B

    def update_obs_norm(self):
        """Fold the rollout's statistics into the estimates (train.py:193-204)."""
        if self.obs_est is None:
            return
        n = self.obs_preprocess.normalizer
        nat.check(nat.lib().mlearn_obs_norm_update(
            nat.ptr(self.obs_stats), self.obs_stats.shape[0], self.obs_stats.shape[1],
            self._obs_B, self.arch.obs_dim, float(n.decay), float(n.eps), nat.ptr(self.obs_est),
            nat.ptr(self.obs_count), nat.stream_handle()), "obs_norm_update")


class PolicyTrainState:
    """Optimizer + per-policy training state (train_state.py:85-136)."""

    # mlearn_optim_state.launch_form of the optimizer step: 0 the library's
    # choice (the fused one-launch chain where it applies), 1 the split
    # launches, 2 the fused launch (A/B runs; bit-identical results)
    optim_launch_form = 0

    def __init__(self, cfg: TrainConfig, hyper_params, policy_state: PolicyState, key):
        self.hyper_params = hyper_params
        dev = policy_state.device
        P = policy_state.layout["total"]
        self.adam_m = torch.zeros(P, dtype=torch.float32, device=dev)
        self.adam_v = torch.zeros(P, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(P, dtype=torch.float32, device=dev)
        self.step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.initial_weight_norms = policy_state.init_norms
        self.update_prng_key = (int(key[0]) & 0xFFFFFFFF, int(key[1]) & 0xFFFFFFFF)
        if policy_state.lstm_desc is not None:
            nbytes = nat.lib().mlearn_lstm_optim_workspace_bytes(policy_state.desc,
                                                                 policy_state.lstm_desc)
        else:
            nbytes = nat.lib().mlearn_optim_workspace_bytes(policy_state.desc)
        self.optim_ws = torch.zeros(max(nbytes, 16), dtype=torch.uint8, device=dev)
        # value normaliser state (normalize_values; views into the manager's
        # [P][8] estimates, set by init_training): train_state.py:86-116, 307-316
        self.value_norm_est = None
        self.value_norm_count = None
        o = nat.OptimState()
        o.params = policy_state.params.data_ptr()
        o.grads = self.grads.data_ptr()
        o.adam_m = self.adam_m.data_ptr()
        o.adam_v = self.adam_v.data_ptr()
        o.init_norms = self.initial_weight_norms.data_ptr()
        o.step = self.step.data_ptr()
        o.lr = float(hyper_params.lr)
        o.b1, o.b2, o.eps = 0.9, 0.999, 1e-8  # optax.adam defaults (optax 0.1.9)
        o.max_grad_norm = float(hyper_params.max_grad_norm)
        o.normalize_params = 1
        o.normalize_layernorms = 1
        o.launch_form = int(self.optim_launch_form)
        self.optim_desc = o

    def optimizer_step(self, policy_state: PolicyState):
        if policy_state.lstm_desc is not None:
            nat.check(nat.lib().mlearn_lstm_optim_step(policy_state.desc, policy_state.lstm_desc,
                                                       self.optim_desc, nat.ptr(self.optim_ws),
                                                       nat.stream_handle()), "lstm_optim_step")
            return
        nat.check(nat.lib().mlearn_optim_step(policy_state.desc, self.optim_desc,
                                              nat.ptr(self.optim_ws), nat.stream_handle()),
                  "optim_step")

    def state_dict(self):
        sd = {"adam_m": self.adam_m.cpu(), "adam_v": self.adam_v.cpu(), "step": self.step.cpu(),
              "update_prng_key": torch.tensor(self.update_prng_key, dtype=torch.int64)}
        hp = self.hyper_params
        if not isinstance(getattr(hp, "entropy_coef", None), dict):
            ec = hp.entropy_coef
            sd["hyper_params"] = torch.tensor(
                [hp.lr, ec.base if hasattr(ec, "base") else float(ec)], dtype=torch.float64)
        if self.value_norm_est is not None:
            sd["value_norm_est"] = self.value_norm_est.cpu()
            sd["value_norm_count"] = self.value_norm_count.cpu()
        return sd

    def load_state_dict(self, sd):
        self.adam_m.copy_(sd["adam_m"])
        self.adam_v.copy_(sd["adam_v"])
        self.step.copy_(sd["step"])
        if "update_prng_key" in sd:
            self.update_prng_key = tuple(int(x) for x in sd["update_prng_key"].tolist())
        if "hyper_params" in sd:
            import dataclasses
            lr, ec = (float(x) for x in sd["hyper_params"].tolist())
            self.hyper_params = dataclasses.replace(self.hyper_params, lr=lr, entropy_coef=ec)
        if self.value_norm_est is not None and "value_norm_est" in sd:
            self.value_norm_est.copy_(sd["value_norm_est"])
            self.value_norm_count.copy_(sd["value_norm_count"])


@dataclass
class TrainStateManager:  # train_state.py:139-304
    """``policy_states`` / ``train_states`` are one PolicyState /
    PolicyTrainState, or lists of them when the rank holds several train
    policies of a population (the reference stacks them on a leading policy
    axis)."""
    policy_states: Any
    train_states: Any
    pbt_rng: Any = None
    user_state: Any = None
    value_norm: Any = None  # [P][8] f32 value-normaliser estimates (normalize_values)
    past_list: Any = None   # past-policy snapshots (pbt.PastPolicy), every rank

    @property
    def policy_list(self):
        ps = self.policy_states
        return list(ps) if isinstance(ps, (list, tuple)) else [ps]

    @property
    def train_list(self):
        ts = self.train_states
        return list(ts) if isinstance(ts, (list, tuple)) else [ts]

    def state_dict(self):
        """The reference's TrainStateManager checkpoint tree (train_state.py:
        145-163): policy states, train states (Adam moments and count, value
        normaliser; the minibatch RNG's position is the rollout's epoch
        counter, saved by TrainingManager), pbt_rng, user_state."""
        return {"policies": [p.state_dict() for p in self.policy_list],
                "train": [t.state_dict() for t in self.train_list],
                "pbt_rng": self.pbt_rng if isinstance(self.pbt_rng, (torch.Tensor, type(None)))
                else None,
                "user_state": _ckpt_safe(self.user_state),
                "past": [p.state_dict() for p in (self.past_list or [])]}

    def load_state_dict(self, sd):
        pol, tr = sd["policies"], sd["train"]
        if len(pol) != len(self.policy_list):
            raise ValueError(f"checkpoint holds {len(pol)} policies, this rank trains "
                             f"{len(self.policy_list)}")
        for p, d in zip(self.policy_list, pol):
            p.load_state_dict(d)
        for t, d in zip(self.train_list, tr):
            t.load_state_dict(d)
        if sd.get("user_state") is not None:
            self.user_state = sd["user_state"]
        if sd.get("pbt_rng") is not None:
            self.pbt_rng = sd["pbt_rng"]
        past = sd.get("past") or []
        if len(past) != len(self.past_list or []):
            raise ValueError(f"checkpoint holds {len(past)} past policies, expected "
                             f"{len(self.past_list or [])}")
        for p, d in zip(self.past_list or [], past):
            p.load_state_dict(d)
        return self

    def save(self, update_idx, path, extra=None):  # train_state.py:145-163
        torch.save({"update_idx": int(update_idx), "state": self.state_dict(),
                    **(extra or {})}, path)

    def load(self, path):  # train_state.py:165-196
        sd = torch.load(path, map_location="cpu", weights_only=True)
        self.load_state_dict(sd["state"])
        return self, sd["update_idx"]


def _ckpt_safe(x):
    """user_state as saved: tensors / numbers / strings and dicts, lists or
    tuples of them (what a weights_only load restores); anything else is not
    checkpointed."""
    if x is None or isinstance(x, (torch.Tensor, int, float, bool, str)):
        return x.detach().cpu() if isinstance(x, torch.Tensor) else x
    if isinstance(x, dict):
        return {k: _ckpt_safe(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_ckpt_safe(v) for v in x)
    return None
