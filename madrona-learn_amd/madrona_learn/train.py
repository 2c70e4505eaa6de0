"""Training orchestration (mirrors src/madrona_learn/train.py:35-391).

``init_training`` builds the same pieces as the reference's _init_training
(train.py:268-391); ``TrainingManager.update_iter`` runs one PPO iteration
(``_update_impl``, train.py:155-225).  The reference compiles an update into
one XLA executable (utils.py:42-57); here the whole update (T fused rollout
steps, the sim, bootstrap, GAE, metrics, every minibatch step) is captured
into HIP graphs after one eager warm-up iteration and replayed, with the
data-parallel collectives (if any) issued between graph segments.
"""

import os
import re
from dataclasses import dataclass
from typing import Any, Callable, Dict, Optional

import numpy as np
import torch

from . import _native as nat
from .cfg import TrainConfig
from .dist import DataParallel, policy_placement, world
from .metrics import TrainingMetrics
from .policy import Policy
from .profile import profile
from .rollouts import RolloutConfig, RolloutManager, RolloutState
from .train_state import PolicyState, PolicyTrainState, TrainStateManager, compile_arch


@dataclass(frozen=True)
class TrainHooks:  # train.py:75-128
    def init_user_state(self):
        return None

    def start_rollouts(self, rollout_state, user_state):
        return rollout_state, user_state

    def finish_rollouts(self, rollouts, bootstrap_values, unnormalized_values,
                        unnormalized_bootstrap_values, user_state):
        return rollouts, user_state

    def add_metrics(self, metrics):
        return metrics

    def rollout_metrics(self, metrics, rollouts, user_state):
        return metrics

    def optimize_metrics(self, metrics, epoch_idx, minibatch, policy_state, train_state):
        return metrics


def _split_seed(seed, stream):
    """Deterministic 2x32-bit key for an RNG stream from the config seed."""
    ss = np.random.SeedSequence([int(seed) & 0xFFFFFFFF, stream])
    w = ss.generate_state(2, dtype=np.uint32)
    return int(w[0]), int(w[1])


class TrainingManager:  # train.py:35-64
    def __init__(self, state, rollout, metrics, cfg, rollout_mgr, algos, user_hooks, dp,
                 update_idx=0, use_graph=True, profile_port=None):
        self.state = state
        self.rollout = rollout
        self.metrics = metrics
        self.cfg = cfg
        self.rollout_mgr = rollout_mgr
        self.algos = list(algos)
        self.algo = self.algos[0]
        self.user_hooks = user_hooks
        self.dp = dp
        self.update_idx = int(update_idx)
        self.use_graph = use_graph
        self.profile_port = profile_port
        self._segments = None
        self._eager_iters = 0
        # "all": the whole update is captured (the fused kernels); "learn":
        # the torch path (generic.py) -- its rollout runs eagerly (it reads the
        # device sampling counter on the host once per rollout) and the PPO
        # update (autograd through the user's modules, HIP action_stats and
        # flat optimizer) is captured; a tree whose modules cannot be captured
        # falls back to eager updates
        self.graph_scope = "all"
        self._side = None  # the torch path's stream (its warm-up and capture)
        self._torch_path = False  # set by _init_training_torch (see _update_torch)

    # -- one update as a generator over collectives --------------------------
    def _collect(self):
        with profile("Collect Rollouts"):
            (self.state, self.rollout, self._rollout_data, _obs_stats,
             self.metrics) = self.rollout_mgr.collect(self.state, self.rollout, self.metrics,
                                                      self.user_hooks)

    def _learn(self):
        with profile("Learn"):
            # algo_wrapper = vmap over the train policies (train.py:165-174,
            # 206-210): each local policy updates on its own env columns
            epoch_ctr = self.rollout.counters[1:2]
            for ps, ts, algo in zip(self.state.policy_list, self.state.train_list, self.algos):
                self.metrics = yield from algo.update_program(
                    self.cfg, ps, ts, self._rollout_data, self.user_hooks.optimize_metrics,
                    self.metrics, epoch_ctr)
            self.algos[0].advance_epochs(epoch_ctr)

    def _program(self):
        with profile("Update Iter"):
            self._collect()
            yield from self._learn()

    def _run_eager(self, gen=None):
        gen = self._program() if gen is None else gen
        try:
            while True:
                op, t = next(gen)
                if op == "allreduce":
                    self.dp.all_reduce_sum_(t)
        except StopIteration:
            pass

    def _capture(self, gen=None, s=None):
        """Capture the update (or the generator gen) into HIP graphs split at
        the collectives."""
        gen = self._program() if gen is None else gen
        segments = []
        done = False
        s = torch.cuda.Stream() if s is None else s
        s.wait_stream(torch.cuda.current_stream())
        while not done:
            g = torch.cuda.CUDAGraph()
            coll = None
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    try:
                        op, coll = next(gen)
                    except StopIteration:
                        done = True
            segments.append((g, coll))
        torch.cuda.current_stream().wait_stream(s)
        return segments

    def _replay(self):
        for g, coll in self._segments:
            g.replay()
            if coll is not None:
                self.dp.all_reduce_sum_(coll)

    def _update_learn_graph(self):
        """graph_scope "learn": eager rollout, then the update from HIP graphs
        (one eager update first, on the stream the capture uses, so that the
        lazily created library handles and autograd's stream state exist
        before capture)."""
        import sys
        self._collect()
        if self._side is None:
            self._side = torch.cuda.Stream()
        cur = torch.cuda.current_stream()
        if self._segments is None and self._eager_iters >= 1:
            try:
                self._segments = self._capture(self._learn(), self._side)
            except RuntimeError as e:  # modules with host reads / syncs: stay eager
                cur.wait_stream(self._side)
                torch.cuda.synchronize()
                print(f"[madrona_learn] torch-path update not capturable ({type(e).__name__}: "
                      f"{e}); updating eagerly", file=sys.stderr)
                self._segments = None
                self.use_graph = False
                self._run_eager(self._learn())
                return
            self._replay()  # the capture recorded the update without running it
        elif self._segments is not None:
            self._replay()
        else:
            self._side.wait_stream(cur)
            with torch.cuda.stream(self._side):
                self._run_eager(self._learn())
            cur.wait_stream(self._side)
            self._eager_iters += 1

    def _host_refs(self):
        # the Python references a (failed) capture may have moved to tensors
        # of its never-executed graph (sim state, observations, carries, ...)
        objs = [self, self.state, self.rollout, self.rollout_mgr, self.rollout_mgr.store]
        objs += list(self.state.policy_list) + list(self.state.train_list)
        return [(o, dict(vars(o))) for o in objs]

    @staticmethod
    def _restore_host_refs(saved):
        for o, d in saved:
            vars(o).clear()
            vars(o).update(d)

    def _update_torch(self):
        """The torch path (generic.py) under use_graph: update 1 runs eagerly
        on the capture stream; update 2 captures the whole program (rollout +
        update, split at the collectives) and replays it from then on.  If the
        user's sim or modules cannot be captured, the host references the
        failed capture moved are restored and only the PPO update is captured
        (graph_scope "learn"; if that fails too, updates run eagerly)."""
        import sys
        if self.graph_scope == "learn":
            return self._update_learn_graph()
        if self._side is None:
            self._side = torch.cuda.Stream()
        cur = torch.cuda.current_stream()
        if self._segments is not None:
            self._replay()
        elif self._eager_iters < 1:
            self._side.wait_stream(cur)
            with torch.cuda.stream(self._side):
                self._run_eager()
            cur.wait_stream(self._side)
            self._eager_iters += 1
        else:
            saved = self._host_refs()
            try:
                self._segments = self._capture(self._program(), self._side)
            except RuntimeError as e:
                cur.wait_stream(self._side)
                torch.cuda.synchronize()
                self._restore_host_refs(saved)
                print(f"[madrona_learn] torch-path rollout not capturable ({type(e).__name__}: "
                      f"{e}); capturing the PPO update only", file=sys.stderr)
                self.graph_scope = "learn"
                return self._update_learn_graph()
            self._replay()  # the capture recorded the update without running it

    def update_iter(self):
        """One PPO iteration; returns self (the reference returns a new pytree)."""
        if self.use_graph and self._torch_path:
            self._update_torch()
        elif self.use_graph and self.graph_scope == "learn":
            self._update_learn_graph()
        elif self.use_graph and self._segments is None and self._eager_iters >= 1:
            # capture runs the program once: it performs this iteration's work
            self._segments = self._capture()
            self._replay_collectives_of_capture()
        elif self._segments is not None:
            self._replay()
        else:
            self._run_eager()
            self._eager_iters += 1
        self.metrics.advance()
        self.update_idx += 1
        return self

    def _replay_collectives_of_capture(self):
        # Capturing records kernels without executing them: run the captured
        # graphs once now so this call still performs exactly one update.
        self._replay()

    def save_ckpt(self, path):  # train.py:44-46
        """<path>/<update_idx>.pt: the train state (TrainStateManager.save) plus
        the rollout state a bit-identical resume needs: the device RNG counters
        (rollout step = action sampling, epoch = minibatch permutations), the
        running env returns, the current observations, the recurrent carry,
        and the sim's own checkpoint when sim_fns provides 'get_ckpts'
        (rollouts.py:206-215, 300-309)."""
        torch.cuda.synchronize()
        os.makedirs(path, exist_ok=True)
        rank, W = world()
        self.state.save(self.update_idx, os.path.join(path, _ckpt_name(self.update_idx, rank, W)),
                        extra={"rollout": self._rollout_state_dict()})

    def load_ckpt(self, path):  # train.py:48-49
        """A file written by save_ckpt, or its directory (latest update)."""
        torch.cuda.synchronize()
        path = _ckpt_file(path, *world())
        self.state, self.update_idx = self.state.load(path)
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if "rollout" in sd:
            self._load_rollout_state(sd["rollout"])
        torch.cuda.synchronize()
        # captured graphs hold launch arguments taken from the host state they
        # were captured with (the update RNG key, a torch-path preprocess's
        # estimate tensors): the next updates run eagerly once, then capture again
        self._segments = None
        self._eager_iters = 0
        return self

    def _rollout_state_dict(self):
        r = self.rollout
        out = {"counters": r.counters.cpu(), "env_returns": r.env_returns.cpu(),
               "cur_obs": _to_cpu(r.cur_obs), "rnn_states": _to_cpu(r.rnn_states)}
        get = getattr(self, "_sim_get_ckpts", None)
        if get is not None:
            out["sim"] = _to_cpu(get())
        return out

    def _load_rollout_state(self, sd):
        r = self.rollout
        r.counters.copy_(sd["counters"])
        r.env_returns.copy_(sd["env_returns"])
        _copy_into(r.cur_obs, sd["cur_obs"])
        _copy_into(r.rnn_states, sd["rnn_states"])
        load = getattr(self, "_sim_load_ckpts", None)
        if load is not None and sd.get("sim") is not None:
            load(sd["sim"])


def _ckpt_name(update_idx, rank=0, world_size=1):
    """<update_idx>.pt on one rank; <update_idx>.r<rank>.pt per rank of a
    multi-rank job (each rank's file carries its own env shard, rollout
    state and the policies placed on it)."""
    return f"{update_idx}.pt" if world_size == 1 else f"{update_idx}.r{rank}.pt"


def _ckpt_file(path, rank=0, world_size=1):
    """A checkpoint file, or in a directory this rank's latest one."""
    if os.path.isdir(path):
        pat = re.compile(r"^(\d+)\.pt$" if world_size == 1 else rf"^(\d+)\.r{rank}\.pt$")
        ids = [int(m.group(1)) for m in map(pat.match, os.listdir(path)) if m]
        if not ids:
            raise FileNotFoundError(f"no checkpoint of rank {rank}/{world_size} in {path}")
        path = os.path.join(path, _ckpt_name(max(ids), rank, world_size))
    return path


def _to_cpu(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: _to_cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_to_cpu(v) for v in x]
    return x


def _copy_into(dst, src):
    """Copy a saved tree into the live device tensors (same structure)."""
    if isinstance(dst, torch.Tensor):
        dst.copy_(src)
    elif isinstance(dst, dict):
        for k in dst:
            _copy_into(dst[k], src[k])
    elif isinstance(dst, (list, tuple)):
        for d, s_ in zip(dst, src):
            _copy_into(d, s_)


def init_training(dev, cfg: TrainConfig, sim_fns: Dict[str, Callable], policy: Policy,
                  init_sim_ctrl=None, user_hooks: TrainHooks = TrainHooks(),
                  restore_ckpt: Optional[str] = None, profile_port: Optional[int] = None,
                  use_graph: bool = True) -> TrainingManager:
    """train.py:131-146 / 268-391."""
    if not torch.cuda.is_available():
        raise RuntimeError("madrona_learn (MI355X build) needs a ROCm GPU; there is no CPU path")
    device = torch.device(dev) if not isinstance(dev, torch.device) else dev
    if device.type != "cuda":
        raise ValueError(f"device must be a GPU, got {device}")
    torch.cuda.set_device(device)
    if cfg.hlgauss_critic:
        raise NotImplementedError(
            "hlgauss_critic (HLGaussDist, models.py:177-315) is outside the fused path; the "
            "scalar DenseLayerCritic and the DreamerV3Critic two-hot critic are supported")
    num_policies = 1
    if cfg.pbt is not None:
        pbt = cfg.pbt
        if pbt.self_play_portion != 1.0 or pbt.past_play_portion != 0.0 or \
                pbt.cross_play_portion != 0.0:
            raise NotImplementedError(
                "populations run the self-play split (pbt.py:130-133); past/cross-play "
                "matchmaking (pbt.py:135-247) is outside the fused path (past policies are "
                "kept as snapshots, pbt_past_update)")
        num_policies = int(pbt.num_train_policies)
    # policy placement: which train policies this rank holds, and the ranks it
    # shares gradients with (dist.policy_placement)
    policy_ids, dp = policy_placement(num_policies)
    dp.enable_native(device)  # RCCL on the compute stream (inside the captured graph)
    rank, W = world()

    # Global semantics (the reference's meaning of the config, cfg.py:68-96):
    # num_worlds counts the worlds of the whole job; rank r simulates worlds
    # [r*num_worlds/W, (r+1)*num_worlds/W) through ITS sim_fns, and the
    # global minibatch_size is split evenly over the ranks that train a
    # policy (PPO.prepare).  At W = 1 this is the single-device reference.
    if cfg.num_worlds % W != 0:
        raise ValueError(f"num_worlds={cfg.num_worlds} does not split over {W} ranks")
    sim_batch = cfg.num_agents_per_world * (cfg.num_worlds // W)
    rollout_cfg = RolloutConfig.setup(
        num_current_policies=len(policy_ids), num_past_policies=0, num_teams=1,
        team_size=cfg.num_agents_per_world, sim_batch_size=sim_batch, actions_cfg=cfg.actions,
        self_play_portion=1.0, cross_play_portion=0.0, past_play_portion=0.0,
        static_play_portion=0.0, reward_gamma=cfg.gamma,
        custom_policy_ids=cfg.custom_policy_ids, policy_dtype=cfg.compute_dtype)
    rollout_key = _split_seed(cfg.seed, 1)
    rnn_states = policy.actor_critic.init_recurrent_state(sim_batch)
    rollout_state = RolloutState.create(rollout_cfg, sim_fns, rollout_key, rnn_states,
                                        init_sim_ctrl, device=device)

    generic_why = _fused_tree_problem(policy, rollout_state, sim_batch, cfg)
    if generic_why is not None:
        # a tree (or preprocess) the fused kernels do not implement: torch
        # autograd over the user's modules, HIP kernels around them (generic.py)
        return _init_training_torch(device, cfg, policy, rollout_state, user_hooks, dp, rank, W,
                                    num_policies, sim_batch, sim_fns, restore_ckpt, profile_port,
                                    generic_why, policy_ids=list(policy_ids),
                                    use_graph=use_graph)
    prefix = policy.actor_critic.backbone.prefix
    from .rollouts import obs_to_matrix
    obs0 = obs_to_matrix(prefix(rollout_state.cur_obs, train=False), sim_batch)
    arch = compile_arch(policy.actor_critic, obs0.shape[1], cfg.compute_dtype)
    # the loss follows cfg.dreamer_v3_critic (ppo.py:169-218) and the stored
    # values the critic module (rollouts.py:383-384, 601-605): they must agree
    if bool(cfg.dreamer_v3_critic) != (arch.critic_bins > 1):
        raise ValueError(
            f"TrainConfig.dreamer_v3_critic={cfg.dreamer_v3_critic} but the policy's critic is "
            f"{type(policy.actor_critic.critic).__name__}: use DreamerV3Critic with "
            "dreamer_v3_critic=True (the reference default) or DenseLayerCritic with False")
    preprocess = policy.obs_preprocess
    obs_key = None
    if preprocess is not None:
        preprocess.fused_cast_dtype(cfg.compute_dtype)
        from .observations import ObservationsEMANormalizer
        if isinstance(preprocess, ObservationsEMANormalizer):
            # (with a prefix, _fused_tree_problem sent the policy to the torch path)
            o = rollout_state.cur_obs
            obs_key = next(iter(o)) if isinstance(o, dict) else None
    # one PolicyState / PolicyTrainState per train policy (_make_policies,
    # train_state.py:439-488: independent init and optimizer RNG per policy)
    pss, tss, algos = [], [], []
    for pid in policy_ids:
        algo = cfg.algo.setup()
        rng = np.random.default_rng(int(cfg.seed) if num_policies == 1
                                    else [int(cfg.seed), int(pid)])
        ps = PolicyState(policy.actor_critic, arch, preprocess, device, rng, obs_key=obs_key)
        dp.broadcast_(ps.params)
        ps.sync_weights()
        ts = PolicyTrainState(cfg, algo.init_hyperparams(cfg), ps,
                              _split_seed(cfg.seed, 2 + 16 * pid))
        ts.policy_id = pid
        pss.append(ps)
        tss.append(ts)
        algos.append(algo)
    # ActorCritic.rollout / update / critic_only / actor_only of the user's
    # tree now run on the (first) training policy's parameters
    policy.actor_critic.bind(pss[0])
    value_norm = None
    if cfg.normalize_values:
        # EMANormalizer.init_estimates per train policy (moving_avg.py:56-76,
        # train_state.py:307-316): mu 0, inv_sigma 1, sigma 1, biased sums 0, N 0
        value_norm = torch.zeros((len(tss), 8), dtype=torch.float32, device=device)
        value_norm[:, 1] = 1.0
        value_norm[:, 2] = 1.0
        vcount = torch.zeros(len(tss), dtype=torch.int32, device=device)
        for i, ts in enumerate(tss):
            ts.value_norm_est, ts.value_norm_count = value_norm[i], vcount[i:i + 1]
    tsm = TrainStateManager(policy_states=pss[0] if len(pss) == 1 else pss,
                            train_states=tss[0] if len(tss) == 1 else tss, pbt_rng=None,
                            user_state=user_hooks.init_user_state(), value_norm=value_norm)
    if cfg.pbt is not None:
        # the population key and the initial hyperparameter draw (train.py:320-351)
        from .pbt import new_pbt_rng, sample_initial_hyperparams
        tsm.pbt_rng = new_pbt_rng(cfg.seed)
        sample_initial_hyperparams(cfg, tsm)
        if cfg.pbt.num_past_policies > 0:
            from .pbt import init_past_policies
            init_past_policies(cfg, tsm)
    start = 0
    ckpt_rollout = None
    if restore_ckpt is not None:
        # train.py:353-354: the train state; the minibatch RNG position (the
        # epoch counter) is restored with it, like the reference's advanced
        # update_prng_key
        path = _ckpt_file(restore_ckpt, rank, W)
        tsm, start = tsm.load(path)
        ckpt_rollout = torch.load(path, map_location="cpu", weights_only=True).get("rollout")
        if ckpt_rollout is not None:
            rollout_state.counters[1].copy_(ckpt_rollout["counters"][1])

    rollout_mgr = RolloutManager(cfg, rollout_state, pss, env_offset=rank * sim_batch)
    rollout_mgr.get_episode_scores = policy.get_episode_scores
    names = algos[0].add_metrics(cfg, [])
    names = rollout_mgr.add_metrics(cfg, names)
    names = user_hooks.add_metrics(names)
    metrics = TrainingMetrics(names, cfg.metrics_buffer_size, device, num_policies=len(pss))
    for p, (ps, ts, algo) in enumerate(zip(pss, tss, algos)):
        algo.prepare(cfg, ps, ts, rollout_mgr.view(p), dp, policy_idx=p,
                     start_states=rollout_mgr.start_states(p) if ps.recurrent else None)
    print(cfg)
    mgr = TrainingManager(tsm, rollout_state, metrics, cfg, rollout_mgr, algos, user_hooks, dp,
                          update_idx=start, use_graph=use_graph, profile_port=profile_port)
    mgr._sim_get_ckpts = sim_fns.get("get_ckpts")
    mgr._sim_load_ckpts = sim_fns.get("load_ckpts")
    return mgr


def _fused_tree_problem(policy, rollout_state, sim_batch, cfg):
    """None when the fused kernels implement the policy (tree and
    preprocess), else why not (the torch path then trains it).  Only the
    fused path's own limits route a policy to the torch path (an fp16
    compute dtype, a tree or preprocess it does not implement, the
    normaliser-before-prefix order); any other error -- e.g. an even
    DreamerV3Critic num_bins, or a bug inside a user's prefix -- propagates."""
    from .rollouts import obs_to_matrix
    ac = policy.actor_critic
    if cfg.compute_dtype == torch.float16:
        return "fp16 compute dtype (DynamicScale, ppo.py:276-291)"
    bb = getattr(ac, "backbone", None)
    prefix = getattr(bb, "prefix", None)
    if prefix is None:
        return f"{type(bb).__name__} has no shared prefix (actor_critic.py:247-303)"
    x = prefix(rollout_state.cur_obs, train=False)
    if isinstance(x, dict) and len(x) != 1:
        return f"the prefix returns {len(x)} observations (the fused kernels take one matrix)"
    obs0 = obs_to_matrix(x, sim_batch)
    try:
        compile_arch(ac, obs0.shape[1], cfg.compute_dtype)
        if policy.obs_preprocess is not None:
            policy.obs_preprocess.fused_cast_dtype(cfg.compute_dtype)
    except NotImplementedError as e:
        return f"NotImplementedError: {e}"
    from .actor_critic import _identity_prefix
    from .observations import ObservationsEMANormalizer
    if isinstance(policy.obs_preprocess, ObservationsEMANormalizer) and \
            prefix is not _identity_prefix:
        # the reference normalises the raw observations and runs the prefix on
        # the result (rollouts.py:838-840, actor_critic.py:226-229); the fused
        # rollout kernel normalises the prefix's output
        return "ObservationsEMANormalizer with a BackboneShared prefix (normaliser before prefix)"
    return None


def _init_training_torch(device, cfg, policy, rollout_state, user_hooks, dp, rank, W,
                         num_policies, sim_batch, sim_fns, restore_ckpt, profile_port, why,
                         policy_ids=(0,), use_graph=True):
    """init_training for a tree outside the fused kernels (generic.py): the
    user's torch modules train under autograd (captured in HIP graphs after
    one eager update, TrainingManager._update_torch), with
    sampling, post-step, GAE, advantage statistics, action_stats and the
    optimizer on the HIP kernels.  A population (cfg.pbt, self-play split)
    gets one copy of the tree per train policy this rank holds, each with its
    own initialisation, optimizer state and update RNG (_make_policies,
    train_state.py:439-488; the reference vmaps algo.update over the policy
    axis, train.py:165-174), trained one after the other."""
    import copy
    import sys
    from .generic import TorchPolicyState, TorchPPO, TorchTrainState, _has_state
    from .models import action_groups
    P = len(policy_ids)
    if num_policies > 1:
        if _has_state(policy.obs_preprocess):
            raise NotImplementedError(
                "a population on the torch path with a stateful ObservationsPreprocess (its "
                "per-policy state is not part of the PBT policy copies here)")
        if any(True for _ in _leaves(policy.actor_critic.init_recurrent_state(1))):
            raise NotImplementedError("a recurrent population on the torch path")
    print(f"[madrona_learn] policy tree outside the fused kernels ({why}): training it with "
          "torch autograd (HIP sampling / GAE / statistics / optimizer)", file=sys.stderr)
    buckets = [b for _, g in action_groups(cfg.actions) for b in g]
    pss, tss, algos = [], [], []
    # policy 0 keeps the user's modules (and cfg.seed: single-policy runs are
    # unchanged); the others train copies taken before any of them creates
    # its (lazily initialised) parameters, each then initialised with its own
    # seed like the reference's per-policy init keys (train_state.py:439-488)
    acs = [policy.actor_critic] + [copy.deepcopy(policy.actor_critic) for _ in policy_ids[1:]]
    for i, pid in enumerate(policy_ids):
        ac = acs[i]
        seed = cfg.seed if num_policies == 1 else \
            int(np.random.SeedSequence([int(cfg.seed), int(pid)]).generate_state(1)[0] & 0x7FFFFFFF)
        obs_p = rollout_state.cur_obs if P == 1 else _obs_cols(rollout_state.cur_obs, P, i)
        ps = TorchPolicyState(ac, policy.obs_preprocess, device, obs_p, cfg.compute_dtype,
                              buckets, seed)
        if bool(cfg.dreamer_v3_critic) != (ps.critic_bins > 1):
            raise ValueError(f"TrainConfig.dreamer_v3_critic={cfg.dreamer_v3_critic} does not "
                             f"match the policy's critic ({ps.critic_bins} output bins)")
        dp.broadcast_(ps.params)
        algo = TorchPPO(cfg.algo.setup())
        ts = TorchTrainState(cfg, algo.init_hyperparams(cfg), ps,
                             _split_seed(cfg.seed, 2 + 16 * pid))
        ts.policy_id = pid
        pss.append(ps)
        tss.append(ts)
        algos.append(algo)
    value_norm = None
    if cfg.normalize_values:
        # EMANormalizer.init_estimates (moving_avg.py:56-76), the fused path's
        # record layout: mu 0, inv_sigma 1, sigma 1, biased sums 0, N 0
        value_norm = torch.zeros((P, 8), dtype=torch.float32, device=device)
        value_norm[:, 1] = 1.0
        value_norm[:, 2] = 1.0
        vcount = torch.zeros(P, dtype=torch.int32, device=device)
        for i, ts in enumerate(tss):
            ts.value_norm_est, ts.value_norm_count = value_norm[i], vcount[i:i + 1]
    tsm = TrainStateManager(policy_states=pss[0] if P == 1 else pss,
                            train_states=tss[0] if P == 1 else tss, pbt_rng=None,
                            user_state=user_hooks.init_user_state(), value_norm=value_norm)
    if cfg.pbt is not None:
        # the population key and the initial hyperparameter draw (train.py:320-351)
        from .pbt import new_pbt_rng, sample_initial_hyperparams
        tsm.pbt_rng = new_pbt_rng(cfg.seed)
        sample_initial_hyperparams(cfg, tsm)
        if cfg.pbt.num_past_policies > 0:
            from .pbt import init_past_policies
            init_past_policies(cfg, tsm)
    start = 0
    if restore_ckpt is not None:
        path = _ckpt_file(restore_ckpt, rank, W)
        tsm, start = tsm.load(path)
        ckpt_rollout = torch.load(path, map_location="cpu", weights_only=True).get("rollout")
        if ckpt_rollout is not None:
            rollout_state.counters[1].copy_(ckpt_rollout["counters"][1])
    rollout_mgr = RolloutManager(cfg, rollout_state, pss, env_offset=rank * sim_batch)
    rollout_mgr.get_episode_scores = policy.get_episode_scores
    names = algos[0].add_metrics(cfg, [])
    names = rollout_mgr.add_metrics(cfg, names)
    names = user_hooks.add_metrics(names)
    metrics = TrainingMetrics(names, cfg.metrics_buffer_size, device, num_policies=P)
    for i, (ps, ts, algo) in enumerate(zip(pss, tss, algos)):
        algo.prepare(cfg, ps, ts, rollout_mgr.view(i), dp, policy_idx=i)
        algo.store = rollout_mgr.store
        algo.col0 = i * rollout_mgr.B
    print(cfg)
    # HIP graphs (TrainingManager._update_torch: the whole update, else the
    # PPO update only); fp16 (DynamicScale reads the gradient norm on the
    # host) stays eager
    mgr = TrainingManager(tsm, rollout_state, metrics, cfg, rollout_mgr, algos, user_hooks, dp,
                          update_idx=start,
                          use_graph=use_graph and all(ts.scaler is None for ts in tss),
                          profile_port=profile_port)
    mgr._torch_path = True  # whole-update capture, falling back to the update only
    mgr._sim_get_ckpts = sim_fns.get("get_ckpts")
    mgr._sim_load_ckpts = sim_fns.get("load_ckpts")
    return mgr


def _leaves(x):
    if isinstance(x, torch.Tensor):
        yield x
    elif isinstance(x, dict):
        for v in x.values():
            yield from _leaves(v)
    elif isinstance(x, (list, tuple)):
        for v in x:
            yield from _leaves(v)


def _obs_cols(obs, P, i):
    """Policy i's env columns of the observations (sample for its init)."""
    n = (next(iter(obs.values())) if isinstance(obs, dict) else obs).shape[0] // P
    if isinstance(obs, dict):
        return {k: v[i * n:(i + 1) * n] for k, v in obs.items()}
    return obs[i * n:(i + 1) * n]


def stop_training(training_mgr: TrainingManager):  # train.py:148-153
    torch.cuda.synchronize()


def train(dev, cfg: TrainConfig, sim_fns, policy: Policy, init_sim_ctrl=None,
          user_hooks: TrainHooks = TrainHooks(), restore_ckpt=None, log_every=0,
          use_graph=True, callback=None):
    """Convenience loop: cfg.num_updates iterations of update_iter."""
    mgr = init_training(dev, cfg, sim_fns, policy, init_sim_ctrl, user_hooks, restore_ckpt,
                        use_graph=use_graph)
    for i in range(cfg.num_updates):
        mgr = mgr.update_iter()
        if log_every and (i + 1) % log_every == 0 and mgr.dp.rank == 0:
            print(f"update {mgr.update_idx}")
            mgr.metrics.pretty_print()
        if callback is not None:
            callback(mgr)
    stop_training(mgr)
    return mgr
