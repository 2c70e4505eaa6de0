"""Population-based training ops (mirrors src/madrona_learn/pbt.py:273-722
and the initial hyperparameter draw of train.py:320-351).

* ``pbt_explore_hyperparams`` (pbt.py:473-562): per ``ParamExplore`` train
  hyperparameter (lr, entropy_coef) and reward hyperparameter, resample it in
  [base*min_scale, base*max_scale] (linear, log10 or ln) with probability
  ``resample_chance``, otherwise perturb it by a uniform factor in
  [perturb_rnd_min, perturb_rnd_max) (clipped if clip_perturb).  As in the
  reference, the optimizer keeps the learning rate it was built with
  (train_state.py:388-389) and the loss reads cfg.algo.entropy_coef
  (ppo.py:231-239): exploration changes the recorded hyperparameters.
* ``pbt_update_fitness`` (pbt.py:382-470): per policy EMA (decay 0.9999) of
  the scores of the episodes that ended this step.
* ``pbt_cull_update`` (pbt.py:609-682): the ``num_cull_policies`` least fit
  train policies take the state of the most fit ones when the one-sided test
  of _check_overwrite (pbt.py:565-600) passes, keeping their own minibatch
  RNG key, then explore the copied hyperparameters (resample chance 0.2).
  Policies of a population are placed over the ranks (dist.policy_placement,
  one per GPU in config P): a copy between ranks is a point-to-point
  transfer of the policy's tensors (RCCL send/recv over xGMI, gloo on CPU);
  the compute weight images are rebuilt on the receiving GPU.
* ``pbt_past_update`` (pbt.py:684-722): past-policy snapshots.  The
  num_past_policies past slots (``TrainStateManager.past_list``, replicated on
  every rank, initialised from train policy j mod P as train_state.py:489-498
  tiles them) hold a policy state without optimizer state; each call picks a
  uniform train policy and overwrites the least fit past slot with it when
  _check_overwrite passes.  Past policies are snapshots only: past-play
  matchmaking (pbt.py:135-247) is outside the fused path, so no env plays
  them and their fitness stays what was copied.

RNG: jax.random's threefry splits are replaced by Philox4x32-10 counters
(the C ABI's ``mlearn_philox4x32_host``): the population key is
``TrainStateManager.pbt_rng`` = int64 [k0, k1, op counter]; op c draws for
population slot s and stream q (0 lr, 1 entropy, 2 + i reward
hyperparameter i) the words of counter {c, s, q, 0}: word 0 decides
resample vs perturb, word 1 is the value's uniform; pbt_past_update's
source pick uses slot 0, stream 0x7fffffff.  Uniforms are
``u32_to_unit`` (csrc/common.h).  oracle/pbt_ref.py restates all of it.
"""

import dataclasses
import math
from typing import Any, Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _native as nat
from .cfg import ParamExplore

EMA_DECAY = 0.9999  # pbt.py:415
CULL_RESAMPLE_CHANCE = 0.2  # pbt.py:637-638


# ---------------------------------------------------------------------------
# RNG
# ---------------------------------------------------------------------------
def philox_host(ctrs, k0, k1):
    c = np.ascontiguousarray(np.asarray(ctrs, dtype=np.uint32).reshape(-1, 4))
    out = np.empty_like(c)
    nat.check(nat.lib().mlearn_philox4x32_host(c.ctypes.data, int(k0) & 0xFFFFFFFF,
                                               int(k1) & 0xFFFFFFFF, out.ctypes.data,
                                               c.shape[0]), "philox_host")
    return out


def u32_to_unit(x):
    """(x >> 8 | 1) * 2^-24: a float32 in (0, 1) (csrc/common.h)."""
    return np.float32(((int(x) >> 8) | 1) * 5.9604644775390625e-08)


def new_pbt_rng(seed):
    """TrainStateManager.pbt_rng: int64 [k0, k1, op counter] (host tensor)."""
    ss = np.random.SeedSequence([int(seed) & 0xFFFFFFFF, 3])
    w = ss.generate_state(2, dtype=np.uint32)
    return torch.tensor([int(w[0]), int(w[1]), 0], dtype=torch.int64)


def _split(pbt_rng):
    """The next op counter of the population key (random.split)."""
    op = int(pbt_rng[2].item())
    pbt_rng[2] += 1
    return int(pbt_rng[0].item()), int(pbt_rng[1].item()), op


def _draws(key, op, slot, stream):
    w = philox_host([[op & 0xFFFFFFFF, slot & 0xFFFFFFFF, stream & 0xFFFFFFFF, 0]], *key)[0]
    return u32_to_unit(w[0]), u32_to_unit(w[1])


# ---------------------------------------------------------------------------
# hyperparameter exploration
# ---------------------------------------------------------------------------
def explore_param(u_resample, u_param, param, pe: ParamExplore, resample_chance):
    """explore_param (pbt.py:480-523) in float32 given its two uniforms."""
    f = np.float32
    lo = f(pe.base * pe.min_scale)
    hi = f(pe.base * pe.max_scale)
    if u_resample < f(resample_chance):
        if pe.log10_scale:
            ls, hs = f(math.log10(lo)), f(math.log10(hi))
        elif pe.ln_scale:
            ls, hs = f(math.log(lo)), f(math.log(hi))
        else:
            ls, hs = lo, hi
        s = f(ls + (hs - ls) * f(u_param))  # random.uniform(minval, maxval)
        if pe.log10_scale:
            s = f(f(10.0) ** s)
        elif pe.ln_scale:
            s = f(np.exp(s))
        return s
    pmin, pmax = f(pe.perturb_rnd_min), f(pe.perturb_rnd_max)
    v = f(f(param) * f(pmin + (pmax - pmin) * f(u_param)))
    if pe.clip_perturb:
        v = f(min(max(v, lo), hi))
    return v


def pbt_explore_hyperparams(cfg, explore_rng, policy_state, train_state, resample_chance):
    """pbt.py:473-562.  explore_rng = (k0, k1, op, slot)."""
    k0, k1, op, slot = explore_rng
    key = (k0, k1)
    rh = getattr(policy_state, "reward_hyper_params", None)
    if rh is not None:
        vals = rh.detach().cpu().numpy().astype(np.float32)
        for i, (_, pe) in enumerate(cfg.pbt.reward_hyper_params_explore.items()):
            ur, up = _draws(key, op, slot, 2 + i)
            vals[i] = explore_param(ur, up, vals[i], pe, resample_chance)
        rh.copy_(torch.from_numpy(vals))
    hp = train_state.hyper_params
    if isinstance(cfg.lr, ParamExplore):
        ur, up = _draws(key, op, slot, 0)
        hp = dataclasses.replace(hp, lr=float(explore_param(ur, up, hp.lr, cfg.lr,
                                                            resample_chance)))
    ec = cfg.algo.entropy_coef
    if isinstance(ec, ParamExplore):
        ur, up = _draws(key, op, slot, 1)
        hp = dataclasses.replace(hp, entropy_coef=float(
            explore_param(ur, up, _scalar(hp.entropy_coef), ec, resample_chance)))
    train_state.hyper_params = hp
    return policy_state, train_state


def _scalar(x):
    return x.base if isinstance(x, ParamExplore) else float(x)


def sample_initial_hyperparams(cfg, tsm):
    """train.py:320-351: every train policy draws its hyperparameters
    (resample chance 1) from one split of the population key; slot = the
    policy's global id, so every rank draws the same values for it."""
    k0, k1, op = _split(tsm.pbt_rng)
    for ps, ts in zip(tsm.policy_list, tsm.train_list):
        pbt_explore_hyperparams(cfg, (k0, k1, op, ts.policy_id), ps, ts, 1.0)
    return tsm


# ---------------------------------------------------------------------------
# fitness
# ---------------------------------------------------------------------------
class MovingEpisodeScore:  # train_state.py:24-27
    def __init__(self, device):
        self.mean = torch.zeros(1, dtype=torch.float32, device=device)
        self.var = torch.zeros(1, dtype=torch.float32, device=device)
        self.N = torch.zeros(1, dtype=torch.int32, device=device)

    def tensors(self):
        return [self.mean, self.var, self.N]


def pbt_update_fitness(policy_columns, episode_scores, dones, team_size=1):
    """pbt.py:382-470 for the self-play split: ``policy_columns`` = [(score,
    col0, ncols)] per local policy (its MovingEpisodeScore and agent
    columns), ``episode_scores`` f32 per match ([N / team_size]:
    get_episode_scores_fn of each match's episode result) or per agent ([N],
    agent 0 of each match counts), ``dones`` [N] per agent.  As the reference
    (pbt.py:390-396), only agent 0 of every match counts: dones reshaped to
    [matches, team_size], column 0.  Device tensor ops only (graph-capturable)."""
    ts = int(team_size)
    dn = dones.reshape(-1)
    d = dn.reshape(-1, ts)[:, 0].bool()
    x = episode_scores.reshape(-1).float()
    if ts > 1 and x.numel() == dn.numel():
        x = x.reshape(-1, ts)[:, 0]
    if x.numel() != d.numel():
        raise ValueError(f"episode scores: {x.numel()} values for {d.numel()} matches")
    nmax = torch.iinfo(torch.int32).max
    for sc, c0, n in policy_columns:
        if c0 % ts or n % ts:
            raise ValueError("a policy's agent columns must hold whole matches")
        v = d[c0 // ts:(c0 + n) // ts]
        xs = x[c0 // ts:(c0 + n) // ts]
        xn = v.sum().to(torch.int32)
        xnf = xn.float()
        cnt = torch.clamp(xnf, min=1.0)
        xm = torch.where(v, xs, 0.0).sum() / cnt
        dev = torch.where(v, xs - xm, 0.0)
        xv = torch.where(xn > 1, (dev * dev).sum() / torch.clamp(xnf - 1.0, min=1.0), 0.0)
        md = xm - sc.mean
        cw = torch.expm1(xnf * math.log(EMA_DECAY)) + 1.0
        xw = 1.0 - cw
        cur = sc.N
        new_n = torch.where(xn > nmax - cur, torch.full_like(cur, nmax), cur + xn)
        mdv = torch.where(cur > 0, (cur.float() / (new_n - 1).float().clamp(min=1.0)) *
                          (cw * xw) * md * md, torch.zeros_like(sc.var))
        upd = xn > 0
        sc.mean.copy_(torch.where(upd, cw * sc.mean + xw * xm, sc.mean))
        sc.var.copy_(torch.where(upd, cw * sc.var + xw * xv + mdv, sc.var))
        sc.N.copy_(torch.where(upd, new_n, sc.N))


def check_overwrite(cfg, mean, var, N, src, dst):
    """_check_overwrite (pbt.py:565-600), episode-score form: one-sided test
    of the score difference, overwrite when p < 0.20 (float32)."""
    f = np.float32
    with np.errstate(divide="ignore", invalid="ignore"):
        s2 = f(var[src]) / f(N[src]) + f(var[dst]) / f(N[dst])
        t = (f(mean[src]) - f(mean[dst])) / np.sqrt(f(s2))
    # t = +/-inf (both variances 0, N > 0, different means) gives p = 0 / 1 as
    # in the reference's 1 - cdf(t); only t = NaN (N = 0) never overwrites
    # (math.erf maps +/-inf to +/-1 and propagates NaN)
    p = f(1.0) - f(0.5 * (1.0 + math.erf(float(t) / math.sqrt(2.0))))
    return bool(p < f(0.20))


# ---------------------------------------------------------------------------
# policy copies between ranks
# ---------------------------------------------------------------------------
def _bundle(ps, ts):
    """Every tensor of a population member that a cull overwrites, plus its
    hyperparameters packed as a float64 tensor."""
    t = [ps.params]
    if ps.obs_est is not None:
        t += [ps.obs_est, ps.obs_count]
    t += ps.episode_score.tensors()
    t += [ts.adam_m, ts.adam_v, ts.step]
    if ts.value_norm_est is not None:
        t += [ts.value_norm_est, ts.value_norm_count]
    return t


def _hp_tensor(ts, device):
    hp = ts.hyper_params
    ec = hp.entropy_coef
    ec = float("nan") if isinstance(ec, dict) else _scalar(ec)  # per-key dicts are not explored
    return torch.tensor([hp.lr, ec], dtype=torch.float64, device=device)


def _set_hp(ts, vec):
    lr, ec = (float(x) for x in vec.cpu().tolist())
    rep = {"lr": lr}
    if not math.isnan(ec):
        rep["entropy_coef"] = ec
    ts.hyper_params = dataclasses.replace(ts.hyper_params, **rep)


def _holders(pid, P, W):
    """Global ranks holding train policy pid (dist.policy_placement)."""
    if P % W == 0:
        return [pid // (P // W)]
    G = W // P
    return list(range(pid * G, (pid + 1) * G))


def copy_policy(tsm, src_pid, dst_pid, P):
    """dst's policy/train state := src's (its own update_prng_key kept),
    locally or from src's first holder to every holder of dst."""
    rank, W = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    local = {ts.policy_id: (ps, ts) for ps, ts in zip(tsm.policy_list, tsm.train_list)}
    root = _holders(src_pid, P, W)[0]
    for r in _holders(dst_pid, P, W):
        if r == root:
            if rank == r:
                sps, sts = local[src_pid]
                dps, dts = local[dst_pid]
                for a, b in zip(_bundle(dps, dts), _bundle(sps, sts)):
                    a.copy_(b)
                dts.hyper_params = sts.hyper_params
                dps.sync_weights()
        elif rank == root:
            sps, sts = local[src_pid]
            for t in _bundle(sps, sts) + [_hp_tensor(sts, sps.params.device)]:
                dist.send(t.contiguous(), r)
        elif rank == r:
            dps, dts = local[dst_pid]
            for t in _bundle(dps, dts):
                dist.recv(t, root)
            hv = _hp_tensor(dts, dps.params.device)
            dist.recv(hv, root)
            _set_hp(dts, hv)
            dps.sync_weights()


def gather_fitness(tsm, P):
    """(mean, var, N) float64 numpy arrays over all P train policies, the same
    on every rank (one all-reduce).  A policy held by one rank reports its
    MovingEpisodeScore as is.  Under data parallelism (G = W / P holders,
    each scoring the episodes of its own env shard) the holders' estimates
    are pooled — N = sum N_g, mean = sum N_g m_g / N, var = sum N_g (v_g +
    (m_g - mean)^2) / N — so the fitness covers all of the policy's envs
    as the reference's does (pbt.py:382-470 over every env of the policy)."""
    rank, W = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    dev = tsm.policy_list[0].params.device
    buf = torch.zeros((P, 6), dtype=torch.float64, device=dev)
    for ps, ts in zip(tsm.policy_list, tsm.train_list):
        e = ps.episode_score
        m, v, n = e.mean[0].double(), e.var[0].double(), e.N[0].double()
        if _holders(ts.policy_id, P, W)[0] == rank:
            buf[ts.policy_id, 0], buf[ts.policy_id, 1], buf[ts.policy_id, 2] = m, v, n
        buf[ts.policy_id, 3] += n  # pooled sums over every holder
        buf[ts.policy_id, 4] += n * m
        buf[ts.policy_id, 5] += n * (v + m * m)
    if W > 1:
        dist.all_reduce(buf)
    h = buf.cpu().numpy()
    mean, var, N = h[:, 0].copy(), h[:, 1].copy(), h[:, 2].copy()
    for pid in range(P):
        if len(_holders(pid, P, W)) > 1 and h[pid, 3] > 0:
            N[pid] = h[pid, 3]
            mean[pid] = h[pid, 4] / N[pid]
            var[pid] = max(h[pid, 5] / N[pid] - mean[pid] * mean[pid], 0.0)
    return mean, var, N


def cull_plan(cfg, mean, var, N, P, num_cull):
    """[(dst, src, overwrite)]: the num_cull least fit train policies (stable
    argsort of the fitness, pbt.py:618-622) against the most fit ones."""
    order = np.argsort(np.asarray(mean, np.float32)[:P], kind="stable")
    bottom, top = order[:num_cull], order[P - num_cull:]
    return [(int(d), int(s), check_overwrite(cfg, mean, var, N, int(s), int(d)))
            for d, s in zip(bottom, top)]


def pbt_cull_update(cfg, tsm, num_cull_policies: int):
    """pbt.py:609-682.  Returns the (updated) TrainStateManager and the
    [(dst, src, overwritten)] plan (the reference prints it)."""
    P = int(cfg.pbt.num_train_policies)
    assert 2 * num_cull_policies <= P
    mean, var, N = gather_fitness(tsm, P)
    plan = cull_plan(cfg, mean, var, N, P, num_cull_policies)
    k0, k1, op = _split(tsm.pbt_rng)
    # every copy reads the pre-cull state of its source (top and bottom are disjoint)
    for i, (dst, src, ok) in enumerate(plan):
        if not ok:
            continue
        copy_policy(tsm, src, dst, P)
        for ps, ts in zip(tsm.policy_list, tsm.train_list):
            if ts.policy_id == dst:
                pbt_explore_hyperparams(cfg, (k0, k1, op, i), ps, ts, CULL_RESAMPLE_CHANCE)
    return tsm, plan


# ---------------------------------------------------------------------------
# past-policy snapshots
# ---------------------------------------------------------------------------
class PastPolicy:
    """Past slot ``policy_id`` (the reference's policy_states[P + j]): the
    policy state of a train policy at the time it was saved — parameters,
    observation-normaliser estimates, fitness — without optimizer state."""

    def __init__(self, policy_id, like):
        self.policy_id = int(policy_id)
        self.params = torch.zeros_like(like.params)
        self.obs_est = None if like.obs_est is None else torch.zeros_like(like.obs_est)
        self.obs_count = None if like.obs_est is None else torch.zeros_like(like.obs_count)
        self.episode_score = MovingEpisodeScore(like.params.device)

    def tensors(self):
        t = [self.params]
        if self.obs_est is not None:
            t += [self.obs_est, self.obs_count]
        return t + self.episode_score.tensors()

    def state_dict(self):
        return {"policy_id": self.policy_id, "tensors": [x.detach().cpu() for x in self.tensors()]}

    def load_state_dict(self, sd):
        for a, b in zip(self.tensors(), sd["tensors"]):
            a.copy_(b)


def _policy_tensors(ps):
    t = [ps.params]
    if ps.obs_est is not None:
        t += [ps.obs_est, ps.obs_count]
    return t + ps.episode_score.tensors()


def snapshot_policy(tsm, src_pid, past, P, fitness=None):
    """past := train policy src_pid's policy state on every rank (a broadcast
    from src's first holder).  ``fitness`` = the (mean, var, N) arrays of
    gather_fitness: the slot's MovingEpisodeScore takes src's POOLED estimate,
    so that under data parallelism (G > 1 holders, each scoring its own env
    shard) the past slots compare with the pooled train fitness on the same
    footing in pbt_past_update (not the first holder's shard alone)."""
    rank, W = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    root = _holders(src_pid, P, W)[0]
    if rank == root:
        local = {ts.policy_id: ps for ps, ts in zip(tsm.policy_list, tsm.train_list)}
        for a, b in zip(past.tensors(), _policy_tensors(local[src_pid])):
            a.copy_(b)
    if W > 1:
        for t in past.tensors():
            dist.broadcast(t, root)
    if fitness is not None:
        mean, var, N = fitness
        e = past.episode_score
        e.mean.fill_(float(mean[src_pid]))
        e.var.fill_(float(var[src_pid]))
        e.N.fill_(int(round(float(N[src_pid]))))


def init_past_policies(cfg, tsm):
    """TrainStateManager.past_list: num_past_policies snapshots, slot j a copy
    of train policy j mod P's initial state (train_state.py:489-498)."""
    P, Q = int(cfg.pbt.num_train_policies), int(cfg.pbt.num_past_policies)
    like = tsm.policy_list[0]
    tsm.past_list = []
    fit = gather_fitness(tsm, P) if Q else None
    for j in range(Q):
        pp = PastPolicy(P + j, like)
        snapshot_policy(tsm, j % P, pp, P, fitness=fit)
        tsm.past_list.append(pp)
    return tsm


def past_update_plan(key, op, mean, var, N, P, Q):
    """(src, dst, overwrite) of pbt_past_update; mean / var / N cover the P
    train then the Q past policies."""
    u, _ = _draws(key, op, 0, 0x7FFFFFFF)
    src = min(int(np.float32(u) * np.float32(P)), P - 1)  # random.randint(0, P)
    dst = P + int(np.argmin(np.asarray(mean, np.float32)[P:P + Q]))  # jnp.argmin: first minimum
    with np.errstate(divide="ignore", invalid="ignore"):
        return src, dst, check_overwrite(cfg=None, mean=mean, var=var, N=N, src=src, dst=dst)


def pbt_past_update(cfg, tsm):
    """pbt.py:684-722: a uniform train policy overwrites the least fit past
    slot when the one-sided test passes.  The plan is kept in
    ``tsm.last_past_update`` (the reference prints it)."""
    if cfg.pbt.num_past_policies == 0:
        return tsm
    P, Q = int(cfg.pbt.num_train_policies), int(cfg.pbt.num_past_policies)
    if len(getattr(tsm, "past_list", None) or []) != Q:
        raise ValueError(f"TrainStateManager holds no {Q} past policies (init_past_policies)")
    k0, k1, op = _split(tsm.pbt_rng)
    fit = gather_fitness(tsm, P)
    mean, var, N = fit
    e = [p.episode_score for p in tsm.past_list]  # pooled when they were taken
    mean = np.concatenate([mean, [float(x.mean[0]) for x in e]])
    var = np.concatenate([var, [float(x.var[0]) for x in e]])
    N = np.concatenate([N, [float(x.N[0]) for x in e]])
    src, dst, ok = past_update_plan((k0, k1), op, mean, var, N, P, Q)
    if ok:
        snapshot_policy(tsm, src, tsm.past_list[dst - P], P, fitness=fit)
    tsm.last_past_update = (src, dst, ok)
    return tsm
