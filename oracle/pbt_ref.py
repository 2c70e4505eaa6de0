"""CPU restatement of the population ops (TEST INFRASTRUCTURE ONLY: imported
by tests/, never by the product).

Follows src/madrona_learn/pbt.py of the reference:
  explore_param               pbt.py:480-523 (float32, like jnp)
  pbt_explore_hyperparams     pbt.py:526-562 (lr / entropy / reward streams)
  pbt_update_fitness          pbt.py:382-470 (EMA decay 0.9999)
  _check_overwrite            pbt.py:565-600 (one-sided test, p < 0.20)
  pbt_cull_update             pbt.py:609-682 (argsort, bottom <- top)
  pbt_past_update             pbt.py:684-722 (random train source -> least fit past slot)
  past snapshots' initial     train_state.py:489-498 (past j = train j mod P, tiled)
with the RNG contract of madrona_learn/pbt.py (Philox4x32-10 counters
{op, slot, stream, 0} on the population key replacing jax.random.split /
uniform; the reference's threefry streams cannot be reproduced without JAX:
parity unpinned against executed reference output, pinned to the restated
formulas and the Random123 Philox known-answer vectors).
"""

import math

import numpy as np
from scipy.stats import norm

from . import native

f32 = np.float32


def unit(w):
    """u32_to_unit (csrc/common.h)."""
    return f32(((int(w) >> 8) | 1) * 5.9604644775390625e-08)


def draws(k0, k1, op, slot, stream):
    w = native.philox(np.array([[op, slot, stream, 0]], np.uint32), k0, k1)[0]
    return unit(w[0]), unit(w[1])


def explore_param(u_resample, u_param, param, pe, resample_chance):
    """pe: dict with base, min_scale, max_scale, log10_scale, ln_scale,
    clip_perturb, perturb_rnd_min, perturb_rnd_max (cfg.py:27-46)."""
    lo = f32(pe["base"] * pe["min_scale"])
    hi = f32(pe["base"] * pe["max_scale"])
    should_resample = u_resample < f32(resample_chance)  # uniform(0, 1) < chance
    if should_resample:
        if pe.get("log10_scale"):
            a, b = f32(math.log10(lo)), f32(math.log10(hi))
        elif pe.get("ln_scale"):
            a, b = f32(math.log(lo)), f32(math.log(hi))
        else:
            a, b = lo, hi
        sampled = f32(a + (b - a) * u_param)  # random.uniform(minval=a, maxval=b)
        if pe.get("log10_scale"):
            sampled = f32(f32(10.0) ** sampled)
        elif pe.get("ln_scale"):
            sampled = f32(np.exp(sampled))
        return sampled
    pmin, pmax = f32(pe.get("perturb_rnd_min", 0.8)), f32(pe.get("perturb_rnd_max", 1.2))
    perturbed = f32(f32(param) * f32(pmin + (pmax - pmin) * u_param))
    if pe.get("clip_perturb"):
        perturbed = f32(min(max(perturbed, lo), hi))
    return perturbed


def explore_hyperparams(key, op, slot, hp, explore, resample_chance):
    """hp: {'lr', 'entropy_coef', 'reward': [..]}; explore: {'lr': pe or
    None, 'entropy_coef': pe or None, 'reward': [pe, ...]}."""
    out = dict(hp)
    k0, k1 = key
    if explore.get("reward"):
        vals = [f32(x) for x in hp["reward"]]
        for i, pe in enumerate(explore["reward"]):
            ur, up = draws(k0, k1, op, slot, 2 + i)
            vals[i] = explore_param(ur, up, vals[i], pe, resample_chance)
        out["reward"] = vals
    if explore.get("lr") is not None:
        ur, up = draws(k0, k1, op, slot, 0)
        out["lr"] = float(explore_param(ur, up, hp["lr"], explore["lr"], resample_chance))
    if explore.get("entropy_coef") is not None:
        ur, up = draws(k0, k1, op, slot, 1)
        out["entropy_coef"] = float(explore_param(ur, up, hp["entropy_coef"],
                                                  explore["entropy_coef"], resample_chance))
    return out


def update_fitness(mean, var, N, scores, valid, ema_decay=0.9999):
    """update_policy_episode_score (pbt.py:395-466) of one policy."""
    x = np.asarray(scores, np.float32)[np.asarray(valid, bool)]
    xN = x.size
    if xN == 0:
        return f32(mean), f32(var), int(N)
    xm = f32(x.mean(dtype=np.float32))
    xv = f32(x.var(ddof=1, dtype=np.float32)) if xN > 1 else f32(0)
    md = f32(xm - f32(mean))
    cw = f32(np.expm1(f32(xN) * f32(np.log(ema_decay)))) + f32(1)
    xw = f32(1) - cw
    nmax = np.iinfo(np.int32).max
    newN = nmax if xN > nmax - N else N + xN
    mdv = f32(N / f32(newN - 1)) * (cw * xw) * md * md if N > 0 else f32(0)
    return f32(cw * f32(mean) + xw * xm), f32(cw * f32(var) + xw * xv + mdv), int(newN)


def check_overwrite(mean, var, N, src, dst):
    s2 = f32(var[src]) / f32(N[src]) + f32(var[dst]) / f32(N[dst])
    t = (f32(mean[src]) - f32(mean[dst])) / np.sqrt(f32(s2))
    p = 1 - norm.cdf(t)
    return bool(p < 0.20)


def cull_plan(mean, var, N, num_train, num_cull):
    """[(dst, src, overwrite)] of pbt_cull_update."""
    order = np.argsort(np.asarray(mean, np.float32)[:num_train], kind="stable")
    bottom, top = order[:num_cull], order[num_train - num_cull:]
    with np.errstate(divide="ignore", invalid="ignore"):
        return [(int(d), int(s), check_overwrite(mean, var, N, s, d))
                for d, s in zip(bottom, top)]


def past_update_plan(k0, k1, op, mean, var, N, num_train, num_past):
    """(src, dst, overwrite) of pbt_past_update (pbt.py:684-722): the source
    is a uniform train policy (random.randint(0, num_train), here counter
    {op, 0, 0x7fffffff, 0} word 0 -> floor(u * num_train)), the destination
    the least fit past policy (jnp.argmin: the first minimum), overwritten
    when _check_overwrite passes.  mean / var / N cover train then past
    policies."""
    u, _ = draws(k0, k1, op, 0, 0x7FFFFFFF)
    src = min(int(f32(u) * f32(num_train)), num_train - 1)
    past = np.asarray(mean, np.float32)[num_train:num_train + num_past]
    dst = num_train + int(np.argmin(past))
    with np.errstate(divide="ignore", invalid="ignore"):
        return src, dst, check_overwrite(mean, var, N, src, dst)


def initial_past_sources(num_train, num_past):
    """Train policy whose initial state past slot j copies (the tile of
    train_state.py:489-498)."""
    return [j % num_train for j in range(num_past)]
