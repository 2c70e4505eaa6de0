"""Training of ActorCritic trees the fused kernels do not implement.

The reference trains whatever flax module the ``Policy`` holds:
``jax.value_and_grad`` over ``apply_fn(..., method='update')``
(ppo.py:119-127, 276-281).  A tree that ``train_state.compile_arch``
recognises (BackboneShared over BackboneEncoder(MLP) or
RecurrentBackboneEncoder(MLP, LSTM), DenseLayerDiscreteActor,
DenseLayerCritic / DreamerV3Critic) trains on the fused HIP kernels; any
other feed-forward tree -- ``BackboneSeparate`` (actor_critic.py:247-303), a
user's own nets, actors, critics or ``ObservationsPreprocess`` -- trains
here: the user's torch modules run forward and backward under torch
autograd, while everything around them stays on the HIP kernels of
``libmlearn.so``:

* the rollout's Gumbel-max sampling (``DiscreteActionDistributions.sample``,
  mlearn_discrete_sample_f32) and the post-step bookkeeping
  (mlearn_rollout_post_step);
* GAE / returns (mlearn_gae_f32), the epoch permutation
  (mlearn_minibatch_perm) and the per-minibatch advantage statistics of
  ``zscore_data`` (mlearn_adv_stats / _finish, all-reduced under DP);
* ``action_stats`` (mlearn_action_stats_f32 forward; its backward through
  the softmax in torch);
* clip_by_global_norm + Adam + normalize_params / normalize_layernorms over
  the flat parameter vector (mlearn_flat_optim_step).

Parameters live in one flat f32 arena (the module's parameters are views of
it, their ``.grad`` views of the gradient arena), so the optimizer and the
data-parallel all-reduce see one buffer.  Projection groups follow the
reference's rules: every Dense kernel (``_Dense.kernel``, or a torch
``nn.Linear.weight``) outside the top-level ``actor`` / ``critic`` modules
goes back to its initial Frobenius norm (ppo.py:303-310,
train_state.py:413-423), every LayerNorm's (scale, bias) to |s|^2 + |b|^2 =
features (ppo.py:312-338; ``models.LayerNorm`` or torch ``nn.LayerNorm``).
An LSTM layer's weights (rnn.MultiLayerLSTMCell ``wi`` / ``wh``, gates
concatenated along the output axis) project per gate, each of the 8 gate
kernels to its own initial norm, as flax's separate per-gate Dense leaves do
(rnn.py:30-36; the fused optimizer's per-gate slots).
Recurrent trees (a user's recurrent backbone, multi-layer LSTMs) train here
with the rollout carry and per-chunk start states.  After one eager update
the whole update (rollout included: the sampling kernel reads the device
step counter itself) is captured in HIP graphs; where the user's sim or
modules cannot be captured, the PPO update alone, else nothing
(TrainingManager._update_torch; fp16 stays eager).
"""

import ctypes
from dataclasses import dataclass

import numpy as np
import torch
from torch import nn

from . import _native as nat
from .dists import DiscreteActionDistributions, PhiloxKey, SymExpTwoHotDistribution


@dataclass(frozen=True)
class GenericArch:
    """What the rollout store and the update need to know of a torch tree."""
    obs_dim: int            # width of the flattened preprocessed observation row
    buckets: tuple
    dtype: torch.dtype      # compute dtype (the store's observation dtype)
    critic_bins: int = 1    # 1: scalar critic; > 1: SymExpTwoHotDistribution logits
    lstm_hidden: int = 0

    @property
    def num_logits(self):
        return int(sum(self.buckets))

    @property
    def num_groups(self):
        return len(self.buckets)


class ObsCodec:
    """Preprocessed observations (a tensor [N, ...] or a dict of them) <->
    one [N, obs_dim] row per env (the [T][N][obs_dim] rollout store)."""

    def __init__(self, obs):
        if isinstance(obs, dict):
            self.keys = list(obs.keys())
            self.shapes = [tuple(obs[k].shape[1:]) for k in self.keys]
        else:
            self.keys = None
            self.shapes = [tuple(obs.shape[1:])]
        self.sizes = [int(np.prod(s)) if s else 1 for s in self.shapes]
        self.width = int(sum(self.sizes))

    def encode(self, obs, out):
        """obs -> out[N, width] (cast to out's dtype)."""
        parts = [obs[k] for k in self.keys] if self.keys is not None else [obs]
        o = 0
        for x, n in zip(parts, self.sizes):
            out[:, o:o + n].copy_(x.reshape(x.shape[0], n))
            o += n

    def decode(self, rows):
        """rows [..., width] -> obs with the same leading dims."""
        lead = rows.shape[:-1]
        out, o = [], 0
        for s, n in zip(self.shapes, self.sizes):
            out.append(rows[..., o:o + n].reshape(*lead, *s))
            o += n
        return dict(zip(self.keys, out)) if self.keys is not None else out[0]


def _projection_groups(ac):
    """[(kind, params...)] in module order: kind 1 = a Dense kernel outside
    the top-level actor / critic (train_state.py:413-423 gives only those an
    initial norm), kind 2 = a LayerNorm (anywhere, ppo.py:312-338), kind 3 =
    one gate's kernel of an LSTM layer (weight, gate): flax OptimizedLSTMCell
    keeps the 8 gate kernels (ii, if, ig, io without bias, hi, hf, hg, ho
    with bias; rnn.py:30-36) as separate Dense leaves, each projected to its
    own initial norm -- the same per-gate slots as the fused optimizer
    (optim.hip proj_slot)."""
    from .models import LayerNorm, _Dense
    from .rnn import MultiLayerLSTMCell
    groups = []
    for name, m in ac.named_modules():
        top = name.split(".", 1)[0]
        if isinstance(m, MultiLayerLSTMCell) and top not in ("actor", "critic"):
            for l in range(len(m.wi)):
                for w in (m.wi[l], m.wh[l]):
                    for gate in range(4):
                        groups.append((3, w, gate))
        elif isinstance(m, _Dense) and m.kernel is not None and top not in ("actor", "critic"):
            groups.append((1, m.kernel))
        elif isinstance(m, nn.Linear) and top not in ("actor", "critic"):
            groups.append((1, m.weight))
        elif isinstance(m, LayerNorm) and m.scale is not None:
            groups.append((2, m.scale, m.bias))
        elif isinstance(m, nn.LayerNorm) and m.elementwise_affine:
            groups.append((2, m.weight, m.bias))
    return groups


class _ActionStats(torch.autograd.Function):
    """DiscreteActionDistributions.action_stats (dists.py:54-77) with the
    forward on mlearn_action_stats_f32 and the backward through the
    per-group softmax: d logp[a] / d l_j = [j == a] - p_j, d H / d l_j =
    -p_j (log p_j + H)."""

    @staticmethod
    def forward(ctx, logits, actions, buckets):
        layout = nat.action_layout(list(buckets))
        lg = logits.float().contiguous()
        N, K = lg.shape[0], len(buckets)
        acts = actions.to(torch.int32).reshape(N, K).contiguous()
        logp = torch.empty((N, K), dtype=torch.float32, device=lg.device)
        ent = torch.empty((N, K), dtype=torch.float32, device=lg.device)
        nat.check(nat.lib().mlearn_action_stats_f32(
            nat.ptr(lg), lg.shape[1], layout, N, nat.ptr(acts), nat.ptr(logp), nat.ptr(ent),
            nat.stream_handle()), "action_stats")
        ctx.save_for_backward(lg, acts, ent)
        ctx.buckets = tuple(buckets)
        ctx.in_dtype = logits.dtype
        return logp, ent

    @staticmethod
    def backward(ctx, g_logp, g_ent):
        lg, acts, ent = ctx.saved_tensors
        d = torch.zeros_like(lg)
        off = 0
        for k, b in enumerate(ctx.buckets):
            x = lg[:, off:off + b]
            lsm = torch.log_softmax(x, -1)
            p = lsm.exp()
            onehot = torch.nn.functional.one_hot(acts[:, k].long(), b).to(p.dtype)
            dk = torch.zeros_like(x)
            if g_logp is not None:
                dk = dk + g_logp[:, k:k + 1] * (onehot - p)
            if g_ent is not None:
                dk = dk + g_ent[:, k:k + 1] * (-p * (lsm + ent[:, k:k + 1]))
            d[:, off:off + b] = dk
            off += b
        return d.to(ctx.in_dtype), None, None


def action_stats_autograd(dists: DiscreteActionDistributions, actions):
    lg = dists.all_logits
    flat = lg.reshape(-1, lg.shape[-1])
    logp, ent = _ActionStats.apply(flat, actions, tuple(dists.actions_num_buckets))
    shape = lg.shape[:-1] + (len(dists.actions_num_buckets),)
    return logp.reshape(shape), ent.reshape(shape)


class TorchPolicyState:
    """A policy whose tree runs as torch modules (the slow path): the
    reference's PolicyState fields (params, obs_preprocess + its state) plus
    the flat parameter / gradient arenas."""

    generic = True
    recurrent = False
    lstm_desc = None
    obs_est = None
    obs_count = None

    def __init__(self, actor_critic, preprocess, device, sample_obs, compute_dtype, buckets,
                 seed):
        # the tree's methods run its torch modules (never a lazily compiled
        # fused PolicyState, actor_critic.ActorCritic._fused)
        object.__setattr__(actor_critic, "_fast", False)
        object.__setattr__(actor_critic, "_bound", None)
        self.actor_critic = actor_critic.to(device)
        self.obs_preprocess = preprocess
        self.device = device
        self.compute_dtype = compute_dtype
        self.obs_pre_state = preprocess.init_state(sample_obs, False) \
            if _has_state(preprocess) else None
        # a bare (unnamed) observation tensor keeps its preprocess state
        # _Bare-marked; a checkpoint stores plain dicts, so load re-marks it
        self._bare_obs = not isinstance(sample_obs, dict)
        pre = self.preprocess(sample_obs)
        # materialise the lazily created parameters (the reference's
        # apply_fn init with the 'rollout' method, train_state.py:318-379)
        torch.manual_seed(int(seed))
        with torch.no_grad():
            one = _slice_obs(pre, 0, 1)
            rnn = _to_device(self.actor_critic.init_recurrent_state(1), device)
            # recurrent trees (e.g. a multi-layer rnn.LSTM) carry their state
            # through the rollout (rollout_state.rnn_states) and train from the
            # per-chunk start states (TorchRollout / TorchPPO); otherwise the
            # tree's (empty) state structure, e.g. ((), ()) for
            # BackboneSeparate, is passed wherever the tree takes rnn states
            self.recurrent = rnn not in ((), None) and _nonempty(rnn)
            self.rnn0 = rnn
            out, _ = self.actor_critic.rollout(PhiloxKey(0, 0), rnn, one)
        crit = out["critic"]
        self.critic_bins = 1 if not isinstance(crit, SymExpTwoHotDistribution) \
            else int(crit.logits.shape[-1])
        self.codec = ObsCodec(pre)
        self.arch = GenericArch(obs_dim=self.codec.width, buckets=tuple(int(b) for b in buckets),
                                dtype=compute_dtype, critic_bins=self.critic_bins)
        named = [(n, p) for n, p in self.actor_critic.named_parameters()]
        total = int(sum(p.numel() for _, p in named))
        self.params = torch.zeros(total, dtype=torch.float32, device=device)
        self.grads = torch.zeros(total, dtype=torch.float32, device=device)
        self.layout = {"total": total, "params": []}
        off = 0
        for n, p in named:
            if p.dtype != torch.float32:
                raise TypeError(f"parameter {n}: the master parameters are f32 (got {p.dtype}); "
                                "cast to the compute dtype inside the module")
            k = p.numel()
            self.params[off:off + k].copy_(p.data.reshape(-1))
            p.data = self.params[off:off + k].view_as(p)
            p.grad = self.grads[off:off + k].view_as(p)
            self.layout["params"].append((n, off, tuple(p.shape)))
            off += k
        # episode-score fitness (PBT); the population path is fused-only
        from .pbt import MovingEpisodeScore
        self.episode_score = MovingEpisodeScore(device)

    # -- the reference's obs_preprocess hooks (observations.py:13-68) ----------
    def preprocess(self, obs):
        pre = self.obs_preprocess
        if pre is None:
            return obs
        if hasattr(pre, "preprocess"):
            return pre.preprocess(self.obs_pre_state, obs, False)
        return obs

    def attach_obs_stats(self, T, N):
        self.T = T

    def begin_rollout(self):
        pre = self.obs_preprocess
        self.obs_stats = pre.init_obs_stats(self.obs_pre_state, False) if _has_state(pre) else None

    def observe(self, t, obs):
        pre = self.obs_preprocess
        if _has_state(pre):
            self.obs_stats = pre.update_obs_stats(self.obs_pre_state, self.obs_stats, t, obs,
                                                  False)

    def update_obs_norm(self):
        pre = self.obs_preprocess
        if _has_state(pre) and getattr(self, "obs_stats", None) is not None:
            self.obs_pre_state = _carry_back(
                self.obs_pre_state, pre.update_state(self.obs_pre_state, self.obs_stats, False))

    def sync_weights(self):
        pass  # the modules read the arena directly

    def state_dict(self):
        from .train_state import _ckpt_safe
        return {"params": self.params.detach().cpu(),
                "obs_pre_state": _ckpt_safe(self.obs_pre_state)}

    def load_state_dict(self, sd):
        self.params.copy_(sd["params"])
        if sd.get("obs_pre_state") is not None:
            st = _to_device(sd["obs_pre_state"], self.device)
            if self._bare_obs:
                from .observations import _wrap
                st = _wrap(st)
            self.obs_pre_state = st

    def policy_tensors(self):
        return [self.params]


def _to_device(x, dev):
    if isinstance(x, torch.Tensor):
        return x.to(dev)
    if isinstance(x, dict):
        r = {k: _to_device(v, dev) for k, v in x.items()}
        return type(x)(r) if type(x) is not dict else r  # (keeps a _Bare marker)
    if isinstance(x, (list, tuple)):
        return type(x)(_to_device(v, dev) for v in x)
    return x


def _map_leaves(fn, x):
    """fn over every tensor of a recurrent-state pytree (lists / tuples / dicts)."""
    if isinstance(x, torch.Tensor):
        return fn(x)
    if isinstance(x, dict):
        return {k: _map_leaves(fn, v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_map_leaves(fn, v) for v in x)
    return x


def _zip_leaves(fn, a, b):
    """fn(a_leaf, b_leaf) over two pytrees of the same structure."""
    if isinstance(a, torch.Tensor):
        fn(a, b)
    elif isinstance(a, dict):
        for k in a:
            _zip_leaves(fn, a[k], b[k])
    elif isinstance(a, (list, tuple)):
        for x, y in zip(a, b):
            _zip_leaves(fn, x, y)


def _leaf_pairs(a, b, out):
    if isinstance(a, torch.Tensor):
        out.append((a, b))
        return isinstance(b, torch.Tensor)
    if isinstance(a, dict):
        return isinstance(b, dict) and a.keys() == b.keys() and \
            all(_leaf_pairs(a[k], b[k], out) for k in a)
    if isinstance(a, (list, tuple)):
        return isinstance(b, (list, tuple)) and len(a) == len(b) and \
            all(_leaf_pairs(x, y, out) for x, y in zip(a, b))
    return a is b or (isinstance(a, (int, float, bool, str, type(None))) and type(a) is type(b)
                      and a == b)


def _carry_back(start, cur):
    """State carried from one update to the next (the sim state, the current
    observations, the recurrent carry, a preprocess's estimates) kept at the
    addresses it had when the update began: cur's tensors are copied into
    start's, which is returned.  A captured update (HIP graph) reads these
    tensors at its start and must find the previous replay's values there.
    cur is returned as is where the structures, shapes or dtypes differ."""
    pairs = []
    if start is cur or not _leaf_pairs(start, cur, pairs):
        return cur
    if any(a.shape != b.shape or a.dtype != b.dtype or a.device != b.device for a, b in pairs):
        return cur
    for a, b in pairs:
        if a is not b:
            a.copy_(b)
    return start


def _nonempty(x):
    if isinstance(x, torch.Tensor):
        return True
    if isinstance(x, (tuple, list)):
        return any(_nonempty(y) for y in x)
    if isinstance(x, dict):
        return any(_nonempty(y) for y in x.values())
    return x is not None


def _has_state(pre):
    """A preprocess with the reference's stateful hooks (observations.py:13-68)."""
    from .observations import ObservationsPreprocess
    return isinstance(pre, ObservationsPreprocess) and pre.has_state()


def _slice_obs(obs, a, b):
    if isinstance(obs, dict):
        return {k: v[a:b] for k, v in obs.items()}
    return obs[a:b]


class TorchTrainState:
    """PolicyTrainState of a torch-path policy: Adam moments and counter over
    the flat arena, the projection groups (initial kernel norms), the
    minibatch RNG key."""

    def __init__(self, cfg, hyper_params, ps: TorchPolicyState, update_prng_key):
        dev = ps.device
        n = ps.layout["total"]
        self.hyper_params = hyper_params
        self.update_prng_key = update_prng_key
        self.grads = ps.grads
        self.adam_m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.adam_v = torch.zeros(n, dtype=torch.float32, device=dev)
        self.step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.value_norm_est = self.value_norm_count = None
        off = {p.data_ptr(): (p.data_ptr() - ps.params.data_ptr()) // 4
               for _, p in ps.actor_critic.named_parameters()}
        rows = []
        for g in _projection_groups(ps.actor_critic):
            if g[0] == 1:
                w = g[1]
                rows.append((off[w.data_ptr()], w.numel(), 0, 0, 1, 0,
                             float(torch.linalg.vector_norm(w.detach().float()).item())))
            elif g[0] == 3:  # gate column block of a row-major [in][4R] LSTM weight
                w, gate = g[1], g[2]
                R = w.shape[1] // 4
                blk = w.detach()[:, gate * R:(gate + 1) * R]
                rows.append((off[w.data_ptr()] + gate * R, R, w.shape[1], w.shape[0], 3, 0,
                             float(torch.linalg.vector_norm(blk.float()).item())))
            else:
                s, b = g[1], g[2]
                rows.append((off[s.data_ptr()], s.numel(), off[b.data_ptr()], b.numel(), 2,
                             s.numel(), 0.0))
        self.num_groups = len(rows)
        gt = (nat.FlatGroup * max(self.num_groups, 1))()
        for i, r in enumerate(rows):
            gt[i].offset, gt[i].count, gt[i].offset2, gt[i].count2 = r[0], r[1], r[2], r[3]
            gt[i].kind, gt[i].features, gt[i].init_norm = r[4], r[5], r[6]
        raw = bytes(gt)
        self.groups = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
        self.init_norms = torch.tensor([r[6] for r in rows if r[4] != 2], dtype=torch.float32)
        self.ws = torch.zeros(int(nat.lib().mlearn_flat_optim_workspace_bytes(n, self.num_groups)),
                              dtype=torch.uint8, device=dev)
        d = nat.FlatOptim()
        d.params, d.grads = ps.params.data_ptr(), ps.grads.data_ptr()
        d.adam_m, d.adam_v, d.step = (self.adam_m.data_ptr(), self.adam_v.data_ptr(),
                                      self.step.data_ptr())
        d.n = n
        d.groups = self.groups.data_ptr()
        d.num_groups = self.num_groups
        d.lr = float(hyper_params.lr)
        d.b1, d.b2, d.eps = 0.9, 0.999, 1e-8  # optax.adam defaults (optax 0.1.9)
        d.max_grad_norm = float(hyper_params.max_grad_norm)
        d.normalize_params = 1
        d.normalize_layernorms = 1
        # fp16: DynamicScale (train_state.py:402-403); a non-finite step keeps
        # params and optimizer state (ppo.py:288-291)
        self.scaler = None
        if ps.compute_dtype == torch.float16:
            from .dynamic_scale import DynamicScale
            self.scaler = DynamicScale(dev)
            d.skip_nonfinite = 1
        self.optim_desc = d

    def optimizer_step(self, policy_state):
        nat.check(nat.lib().mlearn_flat_optim_step(self.optim_desc, nat.ptr(self.ws),
                                                   nat.stream_handle()), "flat_optim_step")

    def state_dict(self):
        sd = {"adam_m": self.adam_m.cpu(), "adam_v": self.adam_v.cpu(), "step": self.step.cpu(),
              "update_prng_key": list(self.update_prng_key)}
        if self.scaler is not None:
            sd["scaler"] = self.scaler.state_dict()
        if self.value_norm_est is not None:
            sd["value_norm_est"] = self.value_norm_est.cpu()
            sd["value_norm_count"] = self.value_norm_count.cpu()
        return sd

    def load_state_dict(self, sd):
        self.adam_m.copy_(sd["adam_m"])
        self.adam_v.copy_(sd["adam_v"])
        self.step.copy_(sd["step"])
        self.update_prng_key = tuple(sd["update_prng_key"])
        if self.scaler is not None and "scaler" in sd:
            self.scaler.load_state_dict(sd["scaler"])
        if self.value_norm_est is not None and "value_norm_est" in sd:
            self.value_norm_est.copy_(sd["value_norm_est"])
            self.value_norm_count.copy_(sd["value_norm_count"])


def _critic_value(crit):
    """_compute_value_estimate (rollouts.py:601-605): the scalar critic, or
    SymExpTwoHotDistribution.mean()."""
    if isinstance(crit, SymExpTwoHotDistribution):
        return crit.mean().reshape(-1)
    return crit.float().reshape(-1)


class TorchRollout:
    """rollout_loop (rollouts.py:829-978) for a torch-path policy, on the
    RolloutManager's store: per step the preprocess, ActorCritic.rollout
    (torch modules, HIP sampling), the store writes, the sim's own step and
    the post-step bookkeeping (mlearn_rollout_post_step); then the bootstrap
    critic (rollouts.py:607-635)."""

    def __init__(self, mgr):
        self.mgr = mgr

    def collect(self, rollout_state, gamma):
        m = self.mgr
        ps = m.policy_state
        s = m.store
        L = nat.lib()
        strm = nat.stream_handle()
        key = rollout_state.prng_key
        # the sampling counter lives on the device (RolloutState.counters[0]);
        # the sampling kernel adds it to the step itself (no host read, so the
        # rollout can be captured in a HIP graph)
        ctr = rollout_state.counters[0:1]
        N = m.N
        rec = ps.recurrent
        if m.P > 1:
            # a population (self-play split, pbt.py:130-133): policy p acts for
            # env columns [p B, (p + 1) B) (init_training excluded recurrent
            # and stateful-preprocess populations on this path)
            return self._collect_population(rollout_state, gamma, key, ctr)
        start_state, start_obs = rollout_state.sim_state, rollout_state.cur_obs
        ps.begin_rollout()
        if rec:
            # the live carry in sim order (rollouts.py:898-901, 941-942) and
            # the carry entering every BPTT chunk (rnn_start_states,
            # rollouts.py:528-537), one [C][N][...] tensor per state leaf
            rollout_state.rnn_states = _to_device(rollout_state.rnn_states, ps.device)
            bptt, C = m.bptt, m.C
            if getattr(s, "torch_start", None) is None:
                s.torch_start = _map_leaves(
                    lambda x: torch.zeros((C, *x.shape), dtype=x.dtype, device=x.device),
                    rollout_state.rnn_states)
            start_rnn = rollout_state.rnn_states
        for t in range(m.T):
            obs = rollout_state.cur_obs
            pre = ps.preprocess(obs)
            ps.observe(t, obs)
            rnn_in = ps.rnn0
            if rec:
                if t % bptt == 0:
                    _zip_leaves(lambda dst, src: dst[t // bptt].copy_(src), s.torch_start,
                                rollout_state.rnn_states)
                rnn_in = rollout_state.rnn_states
            with torch.no_grad():
                out, rnn_out = ps.actor_critic.rollout(
                    PhiloxKey(key[0], key[1], t, m.env_offset, ctr=ctr), rnn_in, pre)
            ps.codec.encode(pre, s.obs[t])
            s.actions[t].copy_(out["actions"].reshape(N, -1))
            s.log_probs[t].copy_(out["log_probs"].reshape(N, -1))
            s.values[t].copy_(_critic_value(out["critic"]))
            step_input = {
                "state": rollout_state.sim_state,
                "actions": m._sim_actions(t),
                "resets": m._resets,
                "sim_ctrl": rollout_state.sim_ctrl,
                "pbt": {"policy_assignments": rollout_state.policy_assignments},
            }
            so = rollout_state.step_fn(step_input)
            rew = so["rewards"].reshape(-1)
            rew = (rew if rew.dtype == torch.float32 else rew.float()).contiguous()
            dn = so["dones"].reshape(-1)
            dn = (dn.view(torch.uint8) if dn.dtype == torch.bool else (dn != 0).view(torch.uint8)) \
                .contiguous()
            nat.check(L.mlearn_rollout_post_step(
                nat.ptr(rew), nat.ptr(dn), N, nat.ptr(s.rewards[t]), nat.ptr(s.dones[t]),
                nat.ptr(rollout_state.env_returns), nat.ptr(s.env_returns_trace[t]), gamma, strm),
                "rollout_post_step")
            rollout_state.sim_state = so["state"]
            rollout_state.cur_obs = so["obs"]
            if rec:  # rnn_reset_fn(rnn_states, dones) (rollouts.py:941-942)
                rollout_state.rnn_states = ps.actor_critic.clear_recurrent_state(
                    rnn_out, so["dones"].reshape(-1) != 0)
        with torch.no_grad():
            rnn_in = rollout_state.rnn_states if rec else ps.rnn0
            out, _ = ps.actor_critic.critic_only(rnn_in, ps.preprocess(rollout_state.cur_obs))
        s.bootstrap.copy_(_critic_value(out["critic"]))
        rollout_state.sim_state = _carry_back(start_state, rollout_state.sim_state)
        rollout_state.cur_obs = _carry_back(start_obs, rollout_state.cur_obs)
        if rec:
            rollout_state.rnn_states = _carry_back(start_rnn, rollout_state.rnn_states)

    def _step_sim(self, rollout_state, t, gamma):
        m = self.mgr
        s = m.store
        N = m.N
        step_input = {
            "state": rollout_state.sim_state,
            "actions": m._sim_actions(t),
            "resets": m._resets,
            "sim_ctrl": rollout_state.sim_ctrl,
            "pbt": {"policy_assignments": rollout_state.policy_assignments},
        }
        so = rollout_state.step_fn(step_input)
        rew = so["rewards"].reshape(-1)
        rew = (rew if rew.dtype == torch.float32 else rew.float()).contiguous()
        dn = so["dones"].reshape(-1)
        dn = (dn.view(torch.uint8) if dn.dtype == torch.bool else (dn != 0).view(torch.uint8)) \
            .contiguous()
        nat.check(nat.lib().mlearn_rollout_post_step(
            nat.ptr(rew), nat.ptr(dn), N, nat.ptr(s.rewards[t]), nat.ptr(s.dones[t]),
            nat.ptr(rollout_state.env_returns), nat.ptr(s.env_returns_trace[t]), gamma,
            nat.stream_handle()), "rollout_post_step")
        rollout_state.sim_state = so["state"]
        rollout_state.cur_obs = so["obs"]

    def _collect_population(self, rollout_state, gamma, key, ctr):
        """rollout_loop for P torch-path policies: per step every policy's
        ActorCritic.rollout on its own env columns (its sampling counters are
        those of its env ids, as in the fused population launch), the store
        columns written, then one sim step and post-step for all envs."""
        m = self.mgr
        s = m.store
        B = m.B
        start_state, start_obs = rollout_state.sim_state, rollout_state.cur_obs
        for t in range(m.T):
            obs = rollout_state.cur_obs
            for p, ps in enumerate(m.policies):
                c = slice(p * B, (p + 1) * B)
                pre = ps.preprocess(_slice_obs(obs, p * B, (p + 1) * B))
                with torch.no_grad():
                    out, _ = ps.actor_critic.rollout(
                        PhiloxKey(key[0], key[1], t, m.env_offset + p * B, ctr=ctr), ps.rnn0,
                        pre)
                ps.codec.encode(pre, s.obs[t, c])
                s.actions[t, c].copy_(out["actions"].reshape(B, -1))
                s.log_probs[t, c].copy_(out["log_probs"].reshape(B, -1))
                s.values[t, c].copy_(_critic_value(out["critic"]))
            self._step_sim(rollout_state, t, gamma)
        obs = rollout_state.cur_obs
        for p, ps in enumerate(m.policies):
            with torch.no_grad():
                out, _ = ps.actor_critic.critic_only(
                    ps.rnn0, ps.preprocess(_slice_obs(obs, p * B, (p + 1) * B)))
            s.bootstrap[p * B:(p + 1) * B].copy_(_critic_value(out["critic"]))
        rollout_state.sim_state = _carry_back(start_state, rollout_state.sim_state)
        rollout_state.cur_obs = _carry_back(start_obs, rollout_state.cur_obs)


class TorchPPO:
    """_ppo (ppo.py:366-488) for a torch-path policy: the fused path's
    permutation and per-minibatch advantage statistics (HIP, all-reduced
    under DP), then per minibatch the loss of ppo.py:129-262 under torch
    autograd over ActorCritic.update, the gradient all-reduce, and the flat
    HIP optimizer step."""

    def __init__(self, base):
        self.base = base  # the fused PPO instance (its prepare() buffers are reused)

    def __getattr__(self, k):
        return getattr(self.base, k)

    def add_metrics(self, cfg, names):
        return self.base.add_metrics(cfg, names)

    def init_hyperparams(self, cfg):
        return self.base.init_hyperparams(cfg)

    def prepare(self, cfg, ps, ts, view, dp, policy_idx=0, start_states=None):
        from .models import action_groups
        b = self.base
        algo = cfg.algo
        if cfg.filter_advantages or cfg.importance_sample_trajectories:
            raise NotImplementedError("filter_advantages / importance_sample_trajectories")
        C = cfg.num_bptt_chunks
        b.bptt = cfg.steps_per_update // C
        b.num_seq = C * view.N
        G = dp.world_size
        if int(algo.minibatch_size) % G != 0:
            raise ValueError(f"minibatch_size {algo.minibatch_size} does not split over {G} ranks")
        b.mb = int(algo.minibatch_size) // G
        if b.num_seq % b.mb != 0:  # ppo.py:439
            raise ValueError(f"{b.num_seq * G} sequences not divisible by minibatch_size "
                             f"{algo.minibatch_size}")
        b.num_mb = b.num_seq // b.mb
        b.E = int(algo.num_epochs)
        dev = ps.device
        b.perm = torch.zeros((b.E, b.num_seq), dtype=torch.int32, device=dev)
        b.adv_part = torch.zeros((b.E, b.num_mb * 66), dtype=torch.float64, device=dev)
        b.adv_stats = torch.zeros((b.E, b.num_mb, 2), dtype=torch.float32, device=dev)
        b.adv_sums = torch.zeros((b.E, 2 * b.num_mb), dtype=torch.float64, device=dev)
        b.view = view
        b.policy_idx = policy_idx
        b.dp = dp
        b.count = float(b.mb * dp.world_size * b.bptt)
        # value normaliser (normalize_values, ppo.py:190-211): the same
        # per-minibatch return sums and estimate chain as the fused path
        # (mlearn_return_stats / mlearn_value_norm_chain); the loss reads
        # record m = {adv mean, adv rstd, mu', inv_sigma' after minibatch m's
        # update, mu, sigma before it}
        b.vnorm = bool(cfg.normalize_values)
        if b.vnorm and ps.critic_bins > 1:
            # ppo.py:57 asserts not normalize_values for distributional
            # critics: the two-hot loss ignores the normaliser, yet GAE would
            # invert the two-hot mean with drifting estimates
            raise ValueError("normalize_values with a SymExpTwoHotDistribution critic "
                             "(the reference asserts against it, ppo.py:57)")
        if b.vnorm:
            b.vn_est = ts.value_norm_est
            b.vn_count = ts.value_norm_count
            b.vn_decay = float(cfg.value_normalizer_decay)
            b.ret_part = torch.zeros_like(b.adv_part)
            b.vn_rec = torch.zeros((b.E, b.num_mb, 8), dtype=torch.float32, device=dev)
            b.adv_sums = torch.zeros((b.E, 4 * b.num_mb), dtype=torch.float64, device=dev)
        self.groups = action_groups(cfg.actions)
        if tuple(x for _, g in self.groups for x in g) != tuple(ps.arch.buckets):
            raise ValueError(f"TrainConfig.actions {self.groups} does not match the actor's "
                             f"head {ps.arch.buckets}")
        ec = algo.entropy_coef
        from .ppo import _base
        self.ecoef = [float(_base(ec[n] if isinstance(ec, dict) else ec)) for n, _ in self.groups]
        self.clip = float(algo.clip_coef)
        self.vcoef = float(algo.value_loss_coef)
        self.clip_vl = bool(algo.clip_value_loss)
        self.huber = bool(algo.huber_value_loss)
        self.norm_adv = bool(cfg.normalize_advantages if cfg.compute_advantages
                             else cfg.normalize_returns)
        self.loss_scale = 1.0 / dp.world_size
        self.store = None  # set by init_training (the RolloutManager's store)

    def _minibatch(self, seqs):
        """RolloutData.minibatch (rollouts.py:319-329): whole sequences of
        bptt steps, time-major [bptt, mb, ...]; store row of (t, seq) =
        (c * bptt + t) * N + b with c, b = divmod(seq, N)."""
        s = self.store
        # this policy's env columns [col0, col0 + view.N) of the [T][N] store
        # (a population's policy p: col0 = p B)
        N, bp = int(self.view.N), self.bptt
        col0 = int(getattr(self, "col0", 0))
        seq = seqs.long()
        c, b = seq // N, seq % N
        t = torch.arange(bp, device=seq.device)[:, None]
        rows = (c[None, :] * bp + t) * s.N + col0 + b[None, :]  # [bptt, mb]
        flat = lambda x: x.reshape(s.T * s.N, *x.shape[2:])   # noqa: E731
        # the view's advantage column (the returns column with
        # compute_advantages=False, RolloutManager.view), at this policy's col0
        adv_src = s.advantages if self.view.advantages == s.advantages.data_ptr() + 4 * col0 \
            else s.returns
        out = {"obs": flat(s.obs)[rows], "actions": flat(s.actions)[rows],
               "log_probs": flat(s.log_probs)[rows], "values": flat(s.values)[rows],
               "returns": flat(s.returns)[rows], "advantages": flat(adv_src)[rows],
               "dones": flat(s.dones)[rows]}
        if getattr(s, "torch_start", None) is not None:
            # rnn_start_states of the minibatch's sequences (chunk c, env b)
            out["rnn_start"] = _map_leaves(lambda x: x[c, b], s.torch_start)
        return out

    def _loss(self, ps, mbd, adv_stats):
        """ppo.py:129-262 on one minibatch (torch autograd through the user's
        modules; action_stats on the HIP kernel)."""
        ac = ps.actor_critic
        obs = ps.codec.decode(mbd["obs"])
        T, M = mbd["dones"].shape
        act_f = ac.actor
        # ActorCritic.update (actor_critic.py:98-128) with the autograd-capable
        # action_stats
        feats_a, feats_c = ac.backbone.sequence(mbd.get("rnn_start", ps.rnn0),
                                                mbd["dones"][..., None], obs, train=True)
        dists = act_f(feats_a, train=True) if _takes_train(act_f) else act_f(feats_a)
        crit = ac.critic(feats_c, train=True) if _takes_train(ac.critic) else ac.critic(feats_c)
        logp, ent = action_stats_autograd(dists, mbd["actions"].reshape(T * M, -1))
        K = logp.shape[-1]
        logp = logp.reshape(T, M, K)
        ent = ent.reshape(T, M, K)
        adv = mbd["advantages"].float()
        if self.norm_adv:
            adv = (adv - adv_stats[0]) * adv_stats[1]  # zscore_data with the minibatch's stats
        ratio = torch.exp(logp - mbd["log_probs"])
        a = adv[..., None]
        surr1 = a * ratio
        # jnp.clip = minimum(maximum(x, lo), hi): 0.5 derivatives at ties
        lo = torch.full_like(ratio, 1.0 - self.clip)
        hi = torch.full_like(ratio, 1.0 + self.clip)
        surr2 = a * torch.minimum(torch.maximum(ratio, lo), hi)
        obj = torch.minimum(surr1, surr2)
        action_obj = 0.0
        entropy_term = 0.0
        off = 0
        for (name, g), c in zip(self.groups, self.ecoef):
            k = len(g)
            action_obj = action_obj + obj[..., off:off + k].mean()
            entropy_term = entropy_term + c * ent[..., off:off + k].mean()
            off += k
        R = mbd["returns"].float()
        verr = None
        if isinstance(crit, SymExpTwoHotDistribution):
            vl = crit.two_hot_cross_entropy_loss(R.reshape(-1, 1)).reshape(T, M)
            V = crit.mean().reshape(T, M)
        else:
            V = crit.float().reshape(T, M)
            vpred = V
            tgt = R
            if self.base.vnorm:
                # ppo.py:190-211: errors of the critic inverted with the estimates
                # before this minibatch; the target = the returns normalised with
                # the estimates after normalize_and_update_estimates
                with torch.no_grad():
                    verr = (V.detach() * adv_stats[5] + adv_stats[4] - R).abs()
                tgt = (R - adv_stats[2]) * adv_stats[3]
            if self.clip_vl:  # ppo.py:197-203: jnp.clip(V, ov - clip, ov + clip)
                ov = mbd["values"].float()
                vpred = torch.minimum(torch.maximum(V, ov - self.clip), ov + self.clip)
            e = vpred - tgt
            if self.huber:  # optax.huber_loss (delta 1)
                ae = e.abs()
                q = torch.clamp(ae, max=1.0)
                vl = 0.5 * q * q + (ae - q)
            else:  # optax.l2_loss
                vl = 0.5 * e * e
        value_loss = vl.mean()
        loss = -action_obj + self.vcoef * value_loss - entropy_term
        with torch.no_grad():
            met = {"Loss": loss.detach(), "Action Obj": obj.detach(), "Value Loss": vl.detach(),
                   "Value Errors": (V.detach() - R).abs() if verr is None else verr,
                   "Entropy": ent.detach()}
        return loss, met

    def update_program(self, cfg, policy_state, train_state, rollout_data, user_metrics_cb,
                       metrics, epoch_ctr):
        b = self.base
        L = nat.lib()
        strm = nat.stream_handle()
        k0, k1 = train_state.update_prng_key
        for e in range(b.E):
            nat.check(L.mlearn_minibatch_perm(k0, k1, nat.ptr(epoch_ctr), e, b.dp.rank,
                                              b.num_seq, nat.ptr(b.perm[e]), strm), "perm")
            nat.check(L.mlearn_adv_stats(b.view, nat.ptr(b.perm[e]), b.num_mb, b.mb,
                                         nat.ptr(b.adv_part[e]), strm), "adv_stats")
            if b.vnorm:
                nat.check(L.mlearn_return_stats(b.view, nat.ptr(b.perm[e]), b.num_mb, b.mb,
                                                nat.ptr(b.ret_part[e]), strm), "return_stats")
        n2 = 2 * b.num_mb
        if b.dp.world_size > 1:
            for e in range(b.E):
                b.adv_sums[e, :n2].copy_(b.adv_part[e, :n2])
                if b.vnorm:
                    b.adv_sums[e, n2:2 * n2].copy_(b.ret_part[e, :n2])
            yield ("allreduce", b.adv_sums)
            for e in range(b.E):
                b.adv_part[e, :n2].copy_(b.adv_sums[e, :n2])
                if b.vnorm:
                    b.ret_part[e, :n2].copy_(b.adv_sums[e, n2:2 * n2])
        for e in range(b.E):
            nat.check(L.mlearn_adv_stats_finish(nat.ptr(b.adv_part[e]), b.num_mb, b.count,
                                                nat.ptr(b.adv_stats[e]), strm), "adv_stats_finish")
        if b.vnorm:  # the estimates move minibatch by minibatch, epochs in order (ppo.py:346)
            for e in range(b.E):
                nat.check(L.mlearn_value_norm_chain(
                    nat.ptr(b.ret_part[e]), nat.ptr(b.adv_stats[e]), b.num_mb, b.count,
                    b.vn_decay, 1e-5, nat.ptr(b.vn_est), nat.ptr(b.vn_count),
                    nat.ptr(b.vn_rec[e]), strm), "value_norm_chain")
        ps, ts = policy_state, train_state
        for e in range(b.E):
            for m in range(b.num_mb):
                seqs = b.perm[e, m * b.mb:(m + 1) * b.mb]
                mbd = self._minibatch(seqs)
                ps.grads.zero_()
                loss, met = self._loss(ps, mbd, b.vn_rec[e, m] if b.vnorm else b.adv_stats[e, m])
                sc = ts.scaler
                if sc is None:
                    (loss * self.loss_scale).backward()
                else:  # DynamicScale.value_and_grad: scaled loss, f32 gradient / scale
                    sc.scale_loss(loss * self.loss_scale).backward()
                    sc.unscale_(ps.grads)
                if b.dp.world_size > 1:
                    yield ("allreduce", ps.grads)
                ts.optimizer_step(ps)
                if sc is not None:
                    sc.update(ps.grads)
                if e == b.E - 1 and m == b.num_mb - 1:
                    _record_metrics(metrics, b.policy_idx, met)
                metrics = user_metrics_cb(metrics, e, {"sequence_ids": seqs}, ps, ts)
        return metrics


def _takes_train(m):
    import inspect
    try:
        return "train" in inspect.signature(m.forward).parameters
    except (TypeError, ValueError):
        return False


def _record_metrics(metrics, policy_idx, met):
    """TrainingMetrics.record of the PPO metrics (ppo.py:351-362): {mean, m2,
    min, max, count} per metric into the 'Loss' .. 'Entropy' slots."""
    out = metrics.slots("Loss", 5, policy=policy_idx)
    rows = []
    for k in ("Loss", "Action Obj", "Value Loss", "Value Errors", "Entropy"):
        x = met[k].double().reshape(-1)
        n = float(x.numel())
        mean = x.mean()
        # (the count by a fill, not a host copy: this runs inside HIP-graph capture)
        rows.append(torch.stack([mean, ((x - mean) ** 2).sum(), x.min(), x.max(),
                                 torch.full((), n, dtype=torch.float64, device=x.device)]))
    out.copy_(torch.stack(rows).reshape(out.shape).to(out.dtype))
