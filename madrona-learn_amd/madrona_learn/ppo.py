"""PPO (mirrors src/madrona_learn/ppo.py).

``PPO.update_program`` restates ``_ppo`` (ppo.py:366-488) for the default
minibatch mode: per epoch a fresh permutation of the C*B sequences
(ppo.py:445-458), then for every minibatch one native call that runs the
forward, loss and backward to a flat gradient (ppo.py:109-281), the data
parallel gradient all-reduce, and one native optimizer step
(ppo.py:283-338).  It is a generator: it yields ('allreduce', tensor) at
every collective so the caller can run it eagerly or capture the compute
between collectives into HIP graphs.
"""

from dataclasses import dataclass
from typing import Union

import torch

from . import _native as nat
from .algo_common import AlgoBase, HyperParams
from .cfg import AlgoConfig, ParamExplore

__all__ = ["PPOConfig"]

PPO_METRICS = ["Loss", "Action Obj", "Value Loss", "Value Errors", "Entropy"]


@dataclass(frozen=True)
class PPOConfig(AlgoConfig):  # ppo.py:24-39
    num_epochs: int
    minibatch_size: int
    clip_coef: float
    value_loss_coef: float
    entropy_coef: Union[float, ParamExplore, dict]
    max_grad_norm: float
    clip_value_loss: bool = False
    huber_value_loss: bool = False

    def name(self):
        return "ppo"

    def setup(self):
        return PPO()


@dataclass(frozen=True)
class PPOHyperParams(HyperParams):  # ppo.py:42-46
    clip_coef: float = 0.2
    value_loss_coef: float = 0.5
    entropy_coef: object = 0.0
    max_grad_norm: float = 0.5


def _base(x):
    return x.base if isinstance(x, ParamExplore) else x


class PPO(AlgoBase):  # ppo.py:49-106
    # mlearn_ppo_hparams.step_kernel of every minibatch launch: 0 the library's
    # choice (mlearn_ppo_step_kernel), 1 the feature split, 2 the row split
    # (A/B runs; 2 raises where the row split does not apply)
    step_kernel = 0
    # mlearn_ppo_hparams.wgrad_form (ABI 22): 0 the library's choice (the
    # LDS-DMA pipeline), 1 register-staged, 2 LDS-DMA; bit-identical (A/B runs)
    wgrad_form = 0

    def init_hyperparams(self, cfg):
        if cfg.dreamer_v3_critic or cfg.hlgauss_critic:
            assert not cfg.algo.clip_value_loss
            assert not cfg.algo.huber_value_loss
            assert not cfg.normalize_values
        return PPOHyperParams(
            lr=_base(cfg.lr), gamma=cfg.gamma, gae_lambda=cfg.gae_lambda,
            normalize_values=cfg.normalize_values,
            value_normalizer_decay=cfg.value_normalizer_decay,
            max_advantage_est_decay=cfg.max_advantage_est_decay,
            clip_coef=cfg.algo.clip_coef, value_loss_coef=cfg.algo.value_loss_coef,
            entropy_coef=cfg.algo.entropy_coef, max_grad_norm=cfg.algo.max_grad_norm)

    def make_optimizer(self, hyper_params):
        # optax.chain(clip_by_global_norm, adam) (ppo.py:84-90): implemented natively
        return ("clip_by_global_norm+adam", hyper_params.max_grad_norm, hyper_params.lr)

    def add_metrics(self, cfg, names):
        return list(names) + PPO_METRICS

    # ------------------------------------------------------------------
    def prepare(self, cfg, policy_state, train_state, view, dp, policy_idx=0, start_states=None):
        """Allocate the per-update buffers once (graph-capture safe).  ``view``
        is the rollout view of this policy's env columns; ``dp`` the data
        parallel group that trains this policy; ``policy_idx`` its slot in the
        rank's metrics; ``start_states`` the device pointers of this policy's
        rnn_start_states (recurrent policies)."""
        algo = cfg.algo
        if cfg.filter_advantages or cfg.importance_sample_trajectories:
            raise NotImplementedError(
                "filter_advantages / importance_sample_trajectories (ppo.py:374-435) are "
                "non-default modes outside the fused path")
        C = cfg.num_bptt_chunks
        self.bptt = cfg.steps_per_update // C
        # minibatch_size is GLOBAL (sequences per optimizer step of this
        # policy, ppo.py:437-443); the dp.world_size ranks that train the
        # policy each contribute an equal slice of every global minibatch
        self.num_seq = C * view.N                     # this rank's sequences
        G = dp.world_size
        if int(algo.minibatch_size) % G != 0:
            raise ValueError(f"minibatch_size {algo.minibatch_size} does not split over the "
                             f"{G} ranks training this policy")
        self.mb = int(algo.minibatch_size) // G       # this rank's slice
        if self.num_seq % self.mb != 0:               # ppo.py:439 (num_seq*G % minibatch_size)
            raise ValueError(f"{self.num_seq * G} sequences not divisible by minibatch_size "
                             f"{algo.minibatch_size}")
        self.num_mb = self.num_seq // self.mb
        self.E = int(algo.num_epochs)
        dev = policy_state.device
        self.perm = torch.zeros((self.E, self.num_seq), dtype=torch.int32, device=dev)
        self.adv_part = torch.zeros((self.E, self.num_mb * 66), dtype=torch.float64, device=dev)
        self.adv_stats = torch.zeros((self.E, self.num_mb, 2), dtype=torch.float32, device=dev)
        self.adv_sums = torch.zeros((self.E, 2 * self.num_mb), dtype=torch.float64, device=dev)
        rows = self.mb * self.bptt
        self.lstm = policy_state.lstm_desc
        if self.lstm is not None:
            if start_states is None:
                raise ValueError("a recurrent policy needs the rollout's rnn_start_states")
            if self.mb % 32 != 0 or rows % 64 != 0:
                raise NotImplementedError(
                    "recurrent fused path: minibatch_size must be a multiple of 32 sequences "
                    "and minibatch_size * bptt_len a multiple of 64")
            self.start_h, self.start_c = (nat.c_void_p(x) for x in start_states)
            nbytes = nat.lib().mlearn_lstm_ppo_workspace_bytes(policy_state.desc, self.lstm,
                                                               rows, self.mb)
        else:
            nbytes = nat.lib().mlearn_ppo_workspace_bytes(policy_state.desc, rows)
        self.ws = torch.zeros(int(nbytes), dtype=torch.uint8, device=dev)
        self.view = view
        self.policy_idx = policy_idx
        K = policy_state.arch.num_groups
        hp = nat.PPOHparams()
        hp.clip_coef = float(algo.clip_coef)
        hp.value_loss_coef = float(algo.value_loss_coef)
        # action groups = the keys of cfg.actions (ppo.py:221-239): each key's
        # surrogate and entropy are means over its own sub-actions, summed over
        # the keys, each entropy with its key's coefficient -> per sub-action
        # weights K / K_key (mlearn_ppo_hparams.obj_weight)
        from .models import action_groups
        groups = action_groups(cfg.actions)
        if sum(len(b) for _, b in groups) != K or \
                tuple(x for _, b in groups for x in b) != tuple(policy_state.arch.buckets):
            raise ValueError(f"TrainConfig.actions {groups} does not match the actor's head "
                             f"{policy_state.arch.buckets}")
        ec = algo.entropy_coef
        j = 0
        for name, b in groups:
            c = ec[name] if isinstance(ec, dict) else ec
            c = float(_base(c))
            for _ in b:
                hp.obj_weight[j] = K / len(b)
                hp.entropy_coef[j] = c * K / len(b)
                j += 1
        # ppo.py:134-143: the surrogate's "advantages" are the advantages
        # (z-scored if normalize_advantages), or with compute_advantages=False
        # the returns (z-scored if normalize_returns); the rollout view then
        # points its advantage column at the returns (RolloutManager.view)
        if cfg.compute_advantages:
            hp.normalize_advantages = 1 if cfg.normalize_advantages else 0
        else:
            if cfg.normalize_values:
                raise NotImplementedError(
                    "compute_advantages=False with normalize_values: the returns' bootstrap "
                    "would need the inverted critic (rollouts.py:726-738, 771-775)")
            hp.normalize_advantages = 1 if cfg.normalize_returns else 0
        hp.clip_value_loss = 1 if algo.clip_value_loss else 0
        hp.huber_value_loss = 1 if algo.huber_value_loss else 0
        hp.loss_scale = 1.0 / dp.world_size
        hp.step_kernel = int(self.step_kernel)
        hp.wgrad_form = int(self.wgrad_form)
        # single-rank training: the gradient reduction also emits the partial
        # sums of squares clip_by_global_norm needs, so the optimizer step skips
        # its own pass over the gradient (under DP the norm is of the
        # all-reduced gradient and the optimizer computes it)
        if dp.world_size == 1:
            nparts = int(nat.lib().mlearn_grad_sumsq_parts(policy_state.layout["total"]))
            self.gsq = torch.zeros(nparts, dtype=torch.float64, device=dev)
            hp.grad_sumsq_out = self.gsq.data_ptr()
            train_state.optim_desc.grad_sumsq_part = self.gsq.data_ptr()
            train_state.optim_desc.grad_sumsq_nparts = nparts
        # value normaliser (normalize_values, ppo.py:190-211): the returns'
        # per-minibatch sums join the advantage sums' collective; one chain
        # launch per epoch turns them into per-minibatch estimate records
        self.vnorm = bool(cfg.normalize_values)
        hp.normalize_values = 1 if self.vnorm else 0
        if self.vnorm:
            self.vn_est = train_state.value_norm_est
            self.vn_count = train_state.value_norm_count
            self.vn_decay = float(cfg.value_normalizer_decay)
            self.ret_part = torch.zeros_like(self.adv_part)
            self.vn_rec = torch.zeros((self.E, self.num_mb, 8), dtype=torch.float32, device=dev)
            self.adv_sums = torch.zeros((self.E, 4 * self.num_mb), dtype=torch.float64, device=dev)
        self.hp = hp
        self.dp = dp
        self.count = float(self.mb * dp.world_size * self.bptt)

    def update_program(self, cfg, policy_state, train_state, rollout_data, user_metrics_cb,
                       metrics, epoch_ctr):
        L = nat.lib()
        strm = nat.stream_handle()
        k0, k1 = train_state.update_prng_key
        # epoch permutations + advantage statistics for every minibatch of the update
        for e in range(self.E):
            nat.check(L.mlearn_minibatch_perm(k0, k1, nat.ptr(epoch_ctr), e, self.dp.rank,
                                              self.num_seq, nat.ptr(self.perm[e]), strm), "perm")
            nat.check(L.mlearn_adv_stats(self.view, nat.ptr(self.perm[e]), self.num_mb, self.mb,
                                         nat.ptr(self.adv_part[e]), strm), "adv_stats")
            if self.vnorm:
                nat.check(L.mlearn_return_stats(self.view, nat.ptr(self.perm[e]), self.num_mb,
                                                self.mb, nat.ptr(self.ret_part[e]), strm),
                          "return_stats")
        n2 = 2 * self.num_mb
        if self.dp.world_size > 1:
            # one collective for every epoch's per-minibatch advantage (and return) sums
            for e in range(self.E):
                self.adv_sums[e, :n2].copy_(self.adv_part[e, :n2])
                if self.vnorm:
                    self.adv_sums[e, n2:].copy_(self.ret_part[e, :n2])
            if self.dp.comm is not None:
                self.dp.native_all_reduce_sum_(self.adv_sums)
            else:
                yield ("allreduce", self.adv_sums)
            for e in range(self.E):
                self.adv_part[e, :n2].copy_(self.adv_sums[e, :n2])
                if self.vnorm:
                    self.ret_part[e, :n2].copy_(self.adv_sums[e, n2:])
        for e in range(self.E):
            nat.check(L.mlearn_adv_stats_finish(nat.ptr(self.adv_part[e]), self.num_mb,
                                                self.count, nat.ptr(self.adv_stats[e]), strm),
                      "adv_stats_finish")
        if self.vnorm:
            # the estimates move minibatch by minibatch, epochs in order (ppo.py:346)
            for e in range(self.E):
                nat.check(L.mlearn_value_norm_chain(
                    nat.ptr(self.ret_part[e]), nat.ptr(self.adv_stats[e]), self.num_mb,
                    self.count, self.vn_decay, 1e-5, nat.ptr(self.vn_est), nat.ptr(self.vn_count),
                    nat.ptr(self.vn_rec[e]), strm), "value_norm_chain")
        loss_out = metrics.slots("Loss", 5, policy=self.policy_idx)
        for e in range(self.E):
            for m in range(self.num_mb):
                seqs = self.perm[e, m * self.mb:(m + 1) * self.mb]
                # TrainingMetrics.record writes every minibatch's metrics into the
                # same buffer slot (metrics.py:161-181, advanced once per update):
                # only the last minibatch's survive, so only it reduces them
                last = e == self.E - 1 and m == self.num_mb - 1
                lo = nat.ptr(loss_out) if last else None
                stats = self.vn_rec[e, m] if self.vnorm else self.adv_stats[e, m]
                if self.lstm is not None:
                    nat.check(L.mlearn_lstm_ppo_minibatch_grad(
                        policy_state.desc, self.lstm, self.view, self.start_h, self.start_c,
                        nat.ptr(seqs), self.mb, nat.ptr(stats), self.hp,
                        nat.ptr(train_state.grads), lo, nat.ptr(self.ws), strm),
                        "lstm_ppo_minibatch_grad")
                else:
                    nat.check(L.mlearn_ppo_minibatch_grad(
                        policy_state.desc, self.view, nat.ptr(seqs), self.mb,
                        nat.ptr(stats), self.hp, nat.ptr(train_state.grads),
                        lo, nat.ptr(self.ws), strm), "ppo_minibatch_grad")
                if self.dp.world_size > 1:
                    if self.dp.comm is not None:
                        self.dp.native_all_reduce_sum_(train_state.grads)
                    else:
                        yield ("allreduce", train_state.grads)
                train_state.optimizer_step(policy_state)
                metrics = user_metrics_cb(metrics, e, {"sequence_ids": seqs}, policy_state,
                                          train_state)
        return metrics

    def advance_epochs(self, epoch_ctr):
        """Move the device epoch counter past this update's epochs (once per
        update, after every policy's update_program)."""
        nat.check(nat.lib().mlearn_counters_add(nat.ptr(epoch_ctr), 1,
                                                (nat.c_uint64 * 1)(self.E),
                                                nat.stream_handle()), "epoch counter")
