"""NumPy restatement of the reference's batched-PPO iteration.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Every function cites the
reference file:line (relative to shacklettbp/madrona-learn src/madrona_learn/)
whose arithmetic it restates.  Third-party arithmetic the reference calls is
restated from its published definition (flax 0.8.1 LayerNorm / Dense, optax
0.1.9 clip_by_global_norm / adam / l2_loss / huber_loss, jax.nn.logsumexp /
softmax); the replaced RNG (jax.random threefry) is documented in DESIGN.md.

Modes
  'f64'   float64 arithmetic, no rounding (accuracy reference)
  'f32'   float32 values at every reference dtype boundary
  'bf16'  compute_dtype=bfloat16: values rounded to bf16 (RNE) where the
          reference's flax modules emit bf16 (Dense outputs, LayerNorm
          outputs, head outputs, bf16 cotangents at Dense boundaries)
Arithmetic runs in ``ad`` (float64 by default; float32 for the timed CPU
baseline).
"""

import numpy as np

from . import native

LN_EPS = 1e-6  # flax.linen.LayerNorm default epsilon (flax 0.8.1)
ADAM_B1, ADAM_B2, ADAM_EPS = 0.9, 0.999, 1e-8  # optax.adam defaults (optax 0.1.9)


# ---------------------------------------------------------------------------
# dtype helpers
# ---------------------------------------------------------------------------
def round_bf16(x):
    """float32 -> bfloat16 (round to nearest even) -> float32."""
    x = np.asarray(x, dtype=np.float32)
    u = x.view(np.uint32)
    # uint32 arithmetic: only NaN patterns can wrap, and those are kept as is
    r = (u + (np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1)))) & np.uint32(0xFFFF0000)
    out = r.view(np.float32)
    return np.where(np.isnan(x), x, out)


def round_fp16_significand(x):
    """float32 -> the float16 significand (10 bits, round to nearest even)
    with float32's exponent range.  The fp16 compute dtype trains under
    DynamicScale (ppo.py:276-291): the loss is scaled by 2^k before the
    backward, which keeps the backward's cotangents inside fp16's normal
    range, where rounding to fp16 and back equals rounding the significand
    (a power-of-two scale commutes with it); the forward's values are O(1).
    So the fp16 rounding points are emulated without fp16's range limits
    (the scale's own overflow handling is oracle/dynamic_scale_ref.py's)."""
    x = np.asarray(x, dtype=np.float32)
    u = x.view(np.uint32)
    r = (u + (np.uint32(0xFFF) + ((u >> np.uint32(13)) & np.uint32(1)))) & np.uint32(0xFFFFE000)
    out = r.view(np.float32)
    return np.where(np.isfinite(x), out, x)


def rnd(x, mode, ad=np.float64):
    """Round to the compute dtype of `mode` ("f64": none; "f32"; "bf16";
    "fp16": round_fp16_significand) and return in the arithmetic dtype ad."""
    if mode == "f64":
        return np.asarray(x, dtype=ad)
    x32 = np.asarray(x, dtype=np.float32)
    if mode == "bf16":
        x32 = round_bf16(x32)
    elif mode == "fp16":
        x32 = round_fp16_significand(x32)
    return x32.astype(ad)


# ---------------------------------------------------------------------------
# returns / advantages
# ---------------------------------------------------------------------------
def gae_f32(rewards, values, dones, bootstrap, gamma, lam):
    """compute_advantages (algo_common.py:84-130) + returns = adv + values
    (rollouts.py:761-769), in float32 with the reference's operation order
    (no fused multiply-add): bit-exact twin of the HIP kernel.

    gamma / lam are the config's Python floats.  The constant gamma * lambda
    is their double-precision product rounded to f32 once (algo_common.py:120
    multiplies the Python floats first, rollouts.py:406; JAX's weak typing
    then rounds to the f32 advantage dtype), NOT f32(gamma) * f32(lambda)."""
    r = np.asarray(rewards, np.float32)
    v = np.asarray(values, np.float32)
    d = np.asarray(dones).astype(bool)
    T = r.shape[0]
    g = np.float32(gamma)
    gl = np.float32(float(gamma) * float(lam))
    nv = np.asarray(bootstrap, np.float32).copy()
    na = np.zeros_like(nv)
    adv = np.empty_like(r)
    for i in range(T - 1, -1, -1):
        nv = np.where(d[i], np.float32(0), nv)
        na = np.where(d[i], np.float32(0), na)
        td = (r[i] + g * nv) - v[i]
        a = td + gl * na
        adv[i] = a
        nv = v[i]
        na = a
    return adv, adv + v


def gae(rewards, values, dones, bootstrap, gamma, lam, ad=np.float64):
    """Same recurrence in `ad` precision (accuracy reference)."""
    r = np.asarray(rewards, ad)
    v = np.asarray(values, ad)
    d = np.asarray(dones).astype(bool)
    nv = np.asarray(bootstrap, ad).copy()
    na = np.zeros_like(nv)
    adv = np.empty_like(r)
    for i in range(r.shape[0] - 1, -1, -1):
        nv = np.where(d[i], 0, nv)
        na = np.where(d[i], 0, na)
        a = r[i] + gamma * nv - v[i] + gamma * lam * na
        adv[i] = a
        nv, na = v[i], a
    return adv, adv + v


def discounted_returns_f32(rewards, dones, bootstrap, gamma):
    """compute_returns (algo_common.py:45-81), float32 operation order."""
    r = np.asarray(rewards, np.float32)
    d = np.asarray(dones).astype(bool)
    g = np.float32(gamma)
    nr = np.asarray(bootstrap, np.float32).copy()
    out = np.empty_like(r)
    for i in range(r.shape[0] - 1, -1, -1):
        nr = np.where(d[i], np.float32(0), nr)
        nr = r[i] + g * nr
        out[i] = nr
    return out


def zscore(x):
    """zscore_data (algo_common.py:133-140): population variance, clamp 1e-5."""
    x = np.asarray(x, np.float64)
    mean, var = x.mean(), x.var()
    return (x - mean) / np.sqrt(max(var, 1e-5)), mean, var


# ---------------------------------------------------------------------------
# parameters
# ---------------------------------------------------------------------------
def param_layout(obs_dim, hidden, num_layers, num_logits, critic_bins=1):
    """Flat layout shared with the HIP library (mlearn_param_count).
    critic_bins = 1: DenseLayerCritic; odd > 1: DreamerV3Critic bins."""
    H, A1 = hidden, num_logits + critic_bins
    off, lay = 0, {"W": [], "s": [], "b": []}
    for l in range(num_layers):
        fin = obs_dim if l == 0 else H
        lay["W"].append((off, (fin, H)))
        off += fin * H
        lay["s"].append((off, (H,)))
        off += H
        lay["b"].append((off, (H,)))
        off += H
    lay["Wh"] = (off, (H, A1))
    off += H * A1
    lay["bh"] = (off, (A1,))
    off += A1
    lay["total"] = off
    lay["critic_bins"] = critic_bins
    return lay


def unflatten(flat, lay, ad=np.float64):
    flat = np.asarray(flat, ad)
    P = {"W": [], "s": [], "b": []}
    for k in ("W", "s", "b"):
        for o, shp in lay[k]:
            P[k].append(flat[o:o + int(np.prod(shp))].reshape(shp).copy())
    for k in ("Wh", "bh"):
        o, shp = lay[k]
        P[k] = flat[o:o + int(np.prod(shp))].reshape(shp).copy()
    P["CB"] = lay.get("critic_bins", 1)
    return P


def flatten(P, lay):
    out = np.zeros(lay["total"], np.float64)
    for k in ("W", "s", "b"):
        for (o, shp), v in zip(lay[k], P[k]):
            out[o:o + v.size] = v.reshape(-1)
    for k in ("Wh", "bh"):
        o, shp = lay[k]
        out[o:o + P[k].size] = P[k].reshape(-1)
    return out


# ---------------------------------------------------------------------------
# actor-critic forward (models.py:46-56, 99-154; actor_critic.py:74-128)
# ---------------------------------------------------------------------------
def trunk(P, x, mode, ad=np.float64):
    """MLP trunk (models.py:99-119): Dense no-bias -> LayerNorm -> ReLU per
    layer.  Returns (last activation [M,H], cache)."""
    h = rnd(x, mode, ad)
    cache = {"in": [], "z": [], "mean": [], "rstd": [], "a": []}
    for l in range(len(P["W"])):
        W = rnd(P["W"][l], mode, ad)
        z = rnd(h @ W, mode, ad)                                    # Dense output dtype
        mean = z.mean(-1, keepdims=True)
        var = np.maximum((z * z).mean(-1, keepdims=True) - mean * mean, 0)  # fast variance
        rstd = 1.0 / np.sqrt(var + LN_EPS)
        y = (z - mean) * (rstd * P["s"][l].astype(ad)) + P["b"][l].astype(ad)
        a = np.maximum(rnd(y, mode, ad), 0)                         # LayerNorm dtype, ReLU
        cache["in"].append(h)
        cache["z"].append(z)
        cache["mean"].append(mean)
        cache["rstd"].append(rstd)
        cache["a"].append(a)
        h = a
    return h, cache


def head_outputs(P, h, mode, ad=np.float64):
    """DenseLayerDiscreteActor (models.py:122-139) + DenseLayerCritic
    (142-154) or DreamerV3Critic (157-174) on the backbone features: Dense
    with bias, outputs upcast to f32.  Returns (logits [M,A], critic) with
    critic = value [M] (scalar critic) or the bin logits [M, CB]."""
    Wh = rnd(P["Wh"], mode, ad)
    out = rnd(rnd(h @ Wh, mode, ad) + rnd(P["bh"], mode, ad), mode, ad)  # Dense + bias
    CB = P.get("CB", 1)
    A = Wh.shape[1] - CB
    return out[:, :A], (out[:, A] if CB == 1 else out[:, A:A + CB])


def value_estimate(crit):
    """_compute_value_estimate (rollouts.py:601-605): the scalar critic, or
    SymExpTwoHotDistribution.mean() of the bin logits."""
    crit = np.asarray(crit)
    return crit if crit.ndim == 1 else twohot_mean(crit)


def heads(P, h, mode, ad=np.float64):
    """head_outputs with the critic reduced to its value estimate:
    (logits [M,A], value [M])."""
    logits, crit = head_outputs(P, h, mode, ad)
    return logits, value_estimate(crit)


def forward(P, x, mode, ad=np.float64):
    """MLP trunk + actor logits + critic.

    Returns (logits [M,A] f32-valued, value estimate [M], cache); the raw
    critic output is cache['crit']."""
    h, cache = trunk(P, x, mode, ad)
    logits, crit = head_outputs(P, h, mode, ad)
    cache["crit"] = crit
    return logits, value_estimate(crit), cache


# ---------------------------------------------------------------------------
# SymExpTwoHotDistribution (dists.py:119-208; the DreamerV3 critic)
# ---------------------------------------------------------------------------
def twohot_bins(nb):
    """_compute_bins (dists.py:128-141) in f32: half = symexp(linspace(-14, 0,
    nb//2 + 1)) with jnp.linspace's interpolation form start * (1 - i/div) +
    stop * i/div and the endpoint set to stop (third-party jax, restated);
    symexp = sign(x) expm1(|x|) (utils.py:39-40); bins = [half,
    -half[:-1][::-1]]."""
    assert nb % 2 == 1 and nb > 1
    nh = nb // 2
    i = np.arange(nh + 1, dtype=np.float32)
    step = (i / np.float32(nh)).astype(np.float32)
    x = (np.float32(-14.0) * (np.float32(1.0) - step)).astype(np.float32)
    x[-1] = 0.0
    half = (np.sign(x) * np.expm1(np.abs(x).astype(np.float64))).astype(np.float32)
    return np.concatenate([half, -half[:-1][::-1]]).astype(np.float32)


def _softmax(x):
    e = np.exp(x - x.max(-1, keepdims=True))
    return e / e.sum(-1, keepdims=True)


def twohot_mean(logits):
    """SymExpTwoHotDistribution.mean (dists.py:143-169): symmetric sum of the
    mirrored halves so that it is exactly 0 at initialisation."""
    logits = np.asarray(logits)
    nb = logits.shape[-1]
    bins = twohot_bins(nb).astype(logits.dtype)
    probs = _softmax(logits)
    mid = (nb - 1) // 2
    p1, p2, p3 = probs[..., :mid], probs[..., mid:mid + 1], probs[..., mid + 1:]
    b1, b2, b3 = bins[:mid], bins[mid:mid + 1], bins[mid + 1:]
    return (p2 * b2).sum(-1) + ((p1 * b1)[..., ::-1] + (p3 * b3)).sum(-1)


def twohot_weights(nb, targets, dtype=np.float64):
    """Two-hot target weights of two_hot_cross_entropy_loss (dists.py:171-203)
    as the reference writes them: lower index = #(bins <= t) - 1, upper =
    nb - #(bins > t), both clipped; lower weight = |b_lo - t| / (|b_lo - t| +
    |b_up - t|) and upper = |b_up - t| / (...) (1/2 each when the clipped
    indices coincide).  Returns [M, nb]."""
    bins = twohot_bins(nb).astype(dtype)
    t = np.asarray(targets, dtype)[:, None]
    lo = np.clip((bins[None, :] <= t).sum(-1) - 1, 0, nb - 1)
    up = np.clip(nb - (bins[None, :] > t).sum(-1), 0, nb - 1)
    same = lo == up
    tt = t[:, 0]
    dl = np.where(same, 1.0, np.abs(bins[lo] - tt))
    du = np.where(same, 1.0, np.abs(bins[up] - tt))
    tot = dl + du
    W = np.zeros((t.shape[0], nb), dtype)
    rows = np.arange(t.shape[0])
    np.add.at(W, (rows, lo), dl / tot)
    np.add.at(W, (rows, up), du / tot)
    return W


def twohot_ce(logits, targets):
    """two_hot_cross_entropy_loss (dists.py:171-208): -sum(two_hot * log_softmax).
    Returns (loss [M], d loss / d logits [M, nb])."""
    logits = np.asarray(logits)
    W = twohot_weights(logits.shape[-1], targets, logits.dtype)
    m = logits.max(-1, keepdims=True)
    lse = m + np.log(np.exp(logits - m).sum(-1, keepdims=True))
    loss = -(W * (logits - lse)).sum(-1)
    grad = W.sum(-1, keepdims=True) * _softmax(logits) - W
    return loss, grad


def log_softmax_groups(logits, buckets):
    """Per-group log_softmax / softmax / entropy (dists.py:54-77)."""
    res = []
    off = 0
    for nb in buckets:
        sl = logits[:, off:off + nb]
        mx = sl.max(-1, keepdims=True)
        lse = mx + np.log(np.exp(sl - mx).sum(-1, keepdims=True))
        lp = sl - lse
        p = np.exp(sl - mx) / np.exp(sl - mx).sum(-1, keepdims=True)
        ent = -(p * lp).sum(-1)
        res.append((off, nb, lp, p, ent))
        off += nb
    return res


def action_stats(logits, buckets, actions):
    """DiscreteActionDistributions.action_stats (dists.py:54-77)."""
    res = log_softmax_groups(np.asarray(logits, np.float64), buckets)
    M = logits.shape[0]
    rows = np.arange(M)
    logp = np.stack([lp[rows, actions[:, g]] for g, (_, _, lp, _, _) in enumerate(res)], -1)
    ent = np.stack([e for (_, _, _, _, e) in res], -1)
    return logp, ent


def sample_actions(logits, buckets, gumbel):
    """DiscreteActionDistributions.sample (dists.py:26-44) with the replaced
    RNG: argmax(logit + Gumbel noise) per group in float32, first index on ties."""
    lg = np.asarray(logits, np.float32)
    noisy = lg + np.asarray(gumbel, np.float32)
    acts = []
    off = 0
    for nb in buckets:
        acts.append(np.argmax(noisy[:, off:off + nb], axis=-1))
        off += nb
    a = np.stack(acts, -1).astype(np.int32)
    logp, _ = action_stats(lg, buckets, a)
    return a, logp


# ---------------------------------------------------------------------------
# PPO loss and its gradient (ppo.py:129-281)
# ---------------------------------------------------------------------------
def _dmin(a, b):
    """JAX's balanced derivative of minimum(a, b) w.r.t. a (0.5 on ties)."""
    return np.where(a < b, 1.0, np.where(a == b, 0.5, 0.0))


def objective_key(hp):
    """ppo.py:134-143: the surrogate uses the advantages, or with
    compute_advantages=False the returns."""
    return "advantages" if hp.get("compute_advantages", True) else "returns"


def objective_normalized(hp):
    """normalize_advantages (compute_advantages) / normalize_returns (not)."""
    if hp.get("compute_advantages", True):
        return hp.get("normalize_advantages", True)
    return hp.get("normalize_returns", True)


def ppo_loss_dhead(logits, V, batch, hp, buckets, adv_stats=None, loss_scale=1.0,
                   ad=np.float64):
    """PPO loss (ppo.py:129-262) and d loss / d head outputs [M, A+1]
    (logits then value), unrounded.  batch: actions [M,K], log_probs [M,K],
    advantages [M], returns [M], values [M]."""
    M = logits.shape[0]
    K = len(buckets)
    acts = np.asarray(batch["actions"])
    old = np.asarray(batch["log_probs"], ad)
    adv = np.asarray(batch[objective_key(hp)], ad)
    R = np.asarray(batch["returns"], ad)
    if objective_normalized(hp):
        if adv_stats is None:
            mean, var = adv.mean(), adv.var()
        else:
            mean, var = adv_stats
        adv = (adv - mean) / np.sqrt(max(var, 1e-5))
    clip = hp["clip_coef"]
    lo, hi = 1.0 - clip, 1.0 + clip
    inv_s = 1.0 / M
    # action groups = the keys of cfg.actions (ppo.py:221-239): each key's
    # surrogate and entropy are means over its own [M, K_key] sub-actions,
    # summed over the keys, with the key's entropy coefficient
    groups = hp.get("action_groups") or [(K, hp["entropy_coef"])]
    assert sum(n for n, _ in groups) == K
    key_of = np.repeat(np.arange(len(groups)), [n for n, _ in groups])
    dlog = np.zeros((M, logits.shape[1]), ad)
    objs, ents = [], []
    action_loss, entropy_loss = 0.0, 0.0
    rows = np.arange(M)
    for g, (off, nb, lp, p, ent) in enumerate(log_softmax_groups(logits, buckets)):
        n_key, ce = groups[key_of[g]]
        inv_sk = 1.0 / (M * n_key)
        a = acts[:, g]
        ratio = np.exp(lp[rows, a] - old[:, g])
        s1 = adv * ratio
        y = np.maximum(ratio, lo)
        cr = np.minimum(y, hi)
        s2 = adv * cr
        obj = np.minimum(s1, s2)
        dclip = np.where(ratio > lo, 1.0, np.where(ratio == lo, 0.5, 0.0)) * \
            np.where(y < hi, 1.0, np.where(y == hi, 0.5, 0.0))
        w1 = _dmin(s1, s2)
        dobj = w1 * adv + (1 - w1) * adv * dclip
        g_lp = -inv_sk * dobj * ratio
        onehot = np.zeros((M, nb), ad)
        onehot[rows, a] = 1.0
        d = g_lp[:, None] * (onehot - p) + ce * inv_sk * p * (lp + ent[:, None])
        dlog[:, off:off + nb] = d * loss_scale
        objs.append(obj)
        ents.append(ent)
        action_loss -= obj.sum() * inv_sk
        entropy_loss -= ce * ent.sum() * inv_sk
    obj = np.stack(objs, -1)
    ent = np.stack(ents, -1)
    if np.asarray(V).ndim == 2:
        # DreamerV3Critic (ppo.py:169-177): two-hot cross entropy of the
        # returns, value errors from mean(); no clip / huber (ppo.py:54-57)
        crit = np.asarray(V, ad)
        vl, dcrit = twohot_ce(crit, R)
        dV = hp["value_loss_coef"] * inv_s * dcrit * loss_scale
        loss = action_loss + hp["value_loss_coef"] * vl.mean() + entropy_loss
        metrics = {
            "Loss": loss, "Action Obj": obj, "Value Loss": vl,
            "Value Errors": np.abs(twohot_mean(crit) - R), "Entropy": ent,
        }
        return loss, np.concatenate([dlog, dV], -1), metrics
    # value normaliser (normalize_values, ppo.py:190-211): hp["value_norm"] =
    # (mu', inv_sigma' after this minibatch's update, mu, sigma before it)
    vn = hp.get("value_norm")
    tgt = R
    if vn is not None:
        f = np.float32
        tgt = ((np.asarray(batch["returns"], f) - f(vn[0])) * f(vn[1])).astype(ad)
    vpred, dvp = V, np.ones_like(V)
    if hp.get("clip_value_loss", False):
        ov = np.asarray(batch["values"], ad)
        yy = np.maximum(V, ov - clip)
        vpred = np.minimum(yy, ov + clip)
        dvp = np.where(V > ov - clip, 1.0, np.where(V == ov - clip, 0.5, 0.0)) * \
            np.where(yy < ov + clip, 1.0, np.where(yy == ov + clip, 0.5, 0.0))
    e = vpred - tgt
    if hp.get("huber_value_loss", False):
        ae = np.abs(e)
        quad = np.minimum(ae, 1.0)
        vl = 0.5 * quad * quad + (ae - quad)
        dvl = np.where(ae < 1.0, e, np.sign(e))
    else:
        vl = 0.5 * e * e
        dvl = e
    dV = hp["value_loss_coef"] * inv_s * dvl * dvp * loss_scale
    loss = action_loss + hp["value_loss_coef"] * vl.mean() + entropy_loss
    metrics = {
        "Loss": loss, "Action Obj": obj, "Value Loss": vl,
        "Value Errors": np.abs((V if vn is None else V * vn[3] + vn[2]) - R), "Entropy": ent,
    }
    return loss, np.concatenate([dlog, dV[:, None]], -1), metrics


def trunk_backward(P, cache, da, G, mode, ad=np.float64):
    """Backward through the MLP trunk from d loss / d (last activation):
    ReLU, LayerNorm (flax fast variance), Dense; fills G['W'], G['s'], G['b']."""
    for l in range(len(P["W"]) - 1, -1, -1):
        z, mean, rstd = cache["z"][l], cache["mean"][l], cache["rstd"][l]
        gam, bet = P["s"][l].astype(ad), P["b"][l].astype(ad)
        xh = (z - mean) * rstd
        y = (z - mean) * (rstd * gam) + bet
        dy = np.where(rnd(y, mode, ad) > 0, da, 0.0)
        G["s"][l] = (dy * xh).sum(0)
        G["b"][l] = dy.sum(0)
        dxh = dy * gam
        dz = rstd * (dxh - dxh.mean(-1, keepdims=True) - xh * (dxh * xh).mean(-1, keepdims=True))
        dz = rnd(dz, mode, ad)
        G["W"][l] = cache["in"][l].T @ dz
        if l > 0:
            da = dz @ rnd(P["W"][l], mode, ad).T
    return G


def ppo_loss_grads(P, batch, hp, buckets, mode="f64", adv_stats=None, loss_scale=1.0,
                   ad=np.float64):
    """Loss (ppo.py:129-262) and d loss / d params (jax.value_and_grad) by
    hand-written backprop.  batch: obs [M,D], actions [M,K], log_probs [M,K],
    advantages [M], returns [M], values [M] (all rows of one minibatch)."""
    logits, V, cache = forward(P, batch["obs"], mode, ad)
    loss, dhead, metrics = ppo_loss_dhead(logits, cache["crit"], batch, hp, buckets, adv_stats,
                                          loss_scale,
                                          ad)
    # ---- backward ----
    dhead = rnd(dhead, mode, ad)                     # cotangent in the compute dtype
    G = {"W": [None] * len(P["W"]), "s": [None] * len(P["W"]), "b": [None] * len(P["W"])}
    aL = cache["a"][-1]
    G["Wh"] = aL.T @ dhead
    G["bh"] = dhead.sum(0)
    da = dhead @ rnd(P["Wh"], mode, ad).T
    trunk_backward(P, cache, da, G, mode, ad)
    return loss, G, metrics, {"logits": logits, "value": V}


# ---------------------------------------------------------------------------
# optimizer (ppo.py:84-90, 283-338; optax 0.1.9)
# ---------------------------------------------------------------------------
def clip_by_global_norm(g, max_norm):
    gn = np.sqrt((g * g).sum())
    if gn < max_norm:
        return g, gn
    return (g / gn) * max_norm, gn


def adam_step(p, g, m, v, count, lr, b1=ADAM_B1, b2=ADAM_B2, eps=ADAM_EPS):
    """optax.scale_by_adam + scale(-lr) + apply_updates; count = step before."""
    m = (1 - b1) * g + b1 * m
    v = (1 - b2) * (g * g) + b2 * v
    c = count + 1
    mhat = m / (1 - b1 ** c)
    vhat = v / (1 - b2 ** c)
    u = mhat / (np.sqrt(vhat) + eps)
    return p + (-lr) * u, m, v


def project(P, init_norms):
    """normalize_params (ppo.py:303-310) + normalize_layernorms (312-338)."""
    for l in range(len(P["W"])):
        W = P["W"][l]
        P["W"][l] = (init_norms[l] * W) / np.sqrt((W * W).sum())
        s, b = P["s"][l], P["b"][l]
        f = np.sqrt(s.shape[-1] / (np.dot(b, b) + np.dot(s, s)))
        P["s"][l] = f * s
        P["b"][l] = f * b
    return P


def optimizer_step(flat_p, flat_g, m, v, count, lay, init_norms, lr, max_grad_norm):
    g, gn = clip_by_global_norm(flat_g, max_grad_norm)
    p, m, v = adam_step(flat_p, g, m, v, count, lr)
    P = project(unflatten(p, lay), init_norms)
    return flatten(P, lay), m, v, gn


def grads_to_flat(G, lay):
    return flatten(G, lay)


# ---------------------------------------------------------------------------
# minibatching (ppo.py:437-482, rollouts.py:319-329)
# ---------------------------------------------------------------------------
def _feistel4(x, half, k0, k1, rank, epoch):
    mask = np.uint32((1 << half) - 1)
    L, R = x >> np.uint32(half), x & mask
    for rd in range(4):
        ctr = np.stack([R + np.uint32(rd << 24), np.full(len(R), rank, np.uint32),
                        np.full(len(R), epoch & 0xFFFFFFFF, np.uint32),
                        np.full(len(R), epoch >> 32, np.uint32)], -1)
        f = native.philox(ctr, k0, k1)[:, 0]
        L, R = R, L ^ (f & mask)
    return (L << np.uint32(half)) | R


def epoch_permutation(k0, k1, epoch, rank, n):
    """random.permutation restated as a keyed bijection (see DESIGN.md RNG):
    4-round balanced Feistel network on [0, 2^b) with Philox round functions,
    restricted to [0, n) by cycle walking (misc.hip perm_kernel)."""
    b = 2
    while (1 << b) < n:
        b += 1
    b += b & 1
    x = np.arange(n, dtype=np.uint32)
    x = _feistel4(x, b // 2, k0, k1, rank, epoch)
    out = x >= n
    while out.any():
        x[out] = _feistel4(x[out], b // 2, k0, k1, rank, epoch)
        out = x >= n
    return x.astype(np.int32)


def minibatch_rows(seq_ids, N, bptt):
    """Store rows (t*N + b) of the minibatch, time-major [T/C, mb] like
    RolloutData.minibatch + swapaxes (rollouts.py:319-329)."""
    seq = np.asarray(seq_ids, np.int64)
    c, b = seq // N, seq % N
    tl = np.arange(bptt)[:, None]
    return ((c[None, :] * bptt + tl) * N + b[None, :]).reshape(-1)


def gather_minibatch(store, rows):
    T, N = store["rewards"].shape
    flat = lambda x: np.asarray(x).reshape(T * N, *np.asarray(x).shape[2:])
    return {
        "obs": flat(store["obs"])[rows],
        "actions": flat(store["actions"])[rows],
        "log_probs": flat(store["log_probs"])[rows],
        "advantages": flat(store["advantages"])[rows],
        "returns": flat(store["returns"])[rows],
        "values": flat(store["values"])[rows],
    }


def ppo_update(flat_p, opt, stores, hp, buckets, lay, init_norms, *, num_epochs, minibatch_size,
               bptt, key, epoch_base, mode="f64", lr, max_grad_norm, ad=np.float64,
               value_norm=None, value_norm_decay=0.99999):
    """_ppo (ppo.py:366-488) for the default minibatch mode, over one or more
    data-parallel ranks (stores[r] = rank r's [T][N] store).  Each optimizer
    step uses the union of the ranks' minibatches: advantage statistics of the
    union, gradient = mean over ranks of the local-mean gradients (equal
    sizes: the union mean).  Returns (params, opt, last-minibatch metrics)."""
    world = len(stores)
    T, N = stores[0]["rewards"].shape
    nseq = (T // bptt) * N
    nmb = nseq // minibatch_size
    m, v, count = opt
    metrics = None
    for e in range(num_epochs):
        perms = [epoch_permutation(key[0], key[1], epoch_base + e, r, nseq) for r in range(world)]
        for mb_i in range(nmb):
            batches = []
            for r in range(world):
                ids = perms[r][mb_i * minibatch_size:(mb_i + 1) * minibatch_size]
                batches.append(gather_minibatch(stores[r], minibatch_rows(ids, N, bptt)))
            alladv = np.concatenate([np.asarray(b[objective_key(hp)], np.float64)
                                     for b in batches])
            stats = (alladv.mean(), alladv.var())
            hp_mb = hp
            if value_norm is not None:
                # normalize_and_update_estimates on the union minibatch's returns
                # (ppo.py:209-211; moving_avg.py:183-192), state carried (ppo.py:346)
                allret = np.concatenate([np.asarray(b["returns"], np.float64) for b in batches])
                z = np.zeros(1, np.float32)
                new = ema_update_estimates(value_norm, ema_update_input_stats(
                    (z, z), 0, allret[:, None]), value_norm_decay, 1e-5)
                hp_mb = dict(hp, value_norm=(float(new["mu"][0]), float(new["inv_sigma"][0]),
                                             float(value_norm["mu"][0]),
                                             float(value_norm["sigma"][0])))
                value_norm.update(new)
            P = unflatten(flat_p, lay, ad)
            gsum = None
            for b in batches:
                loss, G, met, _ = ppo_loss_grads(P, b, hp_mb, buckets, mode, adv_stats=stats,
                                                 loss_scale=1.0 / world, ad=ad)
                gf = flatten(G, lay)
                gsum = gf if gsum is None else gsum + gf
                if metrics is None or b is batches[0]:
                    metrics = met
            flat_p, m, v, _ = optimizer_step(flat_p, gsum, m, v, count, lay, init_norms, lr,
                                             max_grad_norm)
            count += 1
    return flat_p, (m, v, count), metrics


# ---------------------------------------------------------------------------
# rollout (rollouts.py:829-978) with the synthetic env
# ---------------------------------------------------------------------------
# ---------------------------------------------------------------------------
# ObservationsEMANormalizer / EMANormalizer (observations.py:70-132,
# moving_avg.py:48-196), f32 like the reference
# ---------------------------------------------------------------------------
def ema_init(D):
    """init_estimates (moving_avg.py:56-76)."""
    z = np.zeros(D, np.float32)
    return {"mu": z.copy(), "inv_sigma": np.ones(D, np.float32), "sigma": np.ones(D, np.float32),
            "mu_biased": z.copy(), "sigma_sq_biased": z.copy(), "N": 0}


def ema_invert(est, x):
    """EMANormalizer.invert (moving_avg.py:87-95) in f32: x * sigma + mu."""
    f = np.float32
    return (np.asarray(x, f) * est["sigma"].astype(f) + est["mu"].astype(f)).astype(f)


def ema_normalize(est, x, mode):
    """normalize (moving_avg.py:78-86) in f32, then the cast to the compute dtype."""
    x = np.asarray(x, np.float32)
    y = ((x - est["mu"]) * est["inv_sigma"]).astype(np.float32)
    return rnd(y, mode)


def ema_update_input_stats(cur, t, x):
    """update_input_stats (moving_avg.py:107-130) with num_prev_updates = t."""
    a_mean, a_var = cur
    x = np.asarray(x, np.float64)
    b_mean = x.mean(0)
    b_var = ((x - b_mean) ** 2).mean(0)
    b_mean, b_var = b_mean.astype(np.float32), b_var.astype(np.float32)
    delta = (b_mean - a_mean).astype(np.float32)
    b_w = np.float32(1.0) / np.float32(t + 1)
    a_w = np.float32(1.0) - b_w
    ab_mean = (a_mean + delta * b_w).astype(np.float32)
    ab_var = (a_w * a_var + b_w * b_var + np.square(delta) * a_w * b_w).astype(np.float32)
    return ab_mean, ab_var


def ema_update_estimates(est, stats, decay, eps):
    """update_estimates (moving_avg.py:132-180)."""
    x_mean, x_var = stats
    f = np.float32
    mean_delta = (x_mean - est["mu"]).astype(f)
    oma = f(decay)
    alpha = f(1.0) - oma
    N, nN = est["N"], est["N"] + 1
    mu_b = (oma * est["mu_biased"] + alpha * x_mean).astype(f)
    s2_b = (oma * est["sigma_sq_biased"] + alpha * x_var +
            (f(N) / f(nN)) * (oma * alpha) * np.square(mean_delta)).astype(f)
    bc = f(-1.0) / f(np.expm1(f(nN) * f(np.log(oma))))
    mu = (mu_b * bc).astype(f)
    s2 = (s2_b * bc).astype(f)
    inv = (f(1.0) / np.sqrt(np.maximum(s2, f(eps)))).astype(f)
    return {"mu": mu, "inv_sigma": inv, "sigma": (f(1.0) / inv).astype(f), "mu_biased": mu_b,
            "sigma_sq_biased": s2_b, "N": nN}


def rollout(flat_p, lay, env, T, buckets, key, step_base, mode="f32", gamma=0.99,
            env_returns=None, ad=np.float64, actions_override=None, policy_fn=None,
            obs_norm=None):
    """rollout_loop restated: per step policy forward + Gumbel-max sample,
    store, env step, env-return bookkeeping; then the bootstrap critic.
    actions_override[t] (e.g. the GPU's actions) drives the env instead of
    the oracle's own samples (used to replay a GPU trajectory exactly).
    policy_fn(obs) -> (actions, log_probs, values) replaces the MLP policy
    (integer fake-policy KAT, tests/test_rollout_kat.py).  obs_norm = (est,
    decay, eps) applies ObservationsEMANormalizer with the estimates est and
    returns the updated estimates as out['obs_est'] (rollouts.py:670-678,
    train.py:193-204)."""
    if policy_fn is not None:
        return _rollout_fake(policy_fn, env, T, gamma, env_returns)
    N = env.N
    if isinstance(flat_p, (list, tuple)):
        # a population: policy p acts for env columns [p*B, (p+1)*B), the
        # self-play split of pbt_init_matchmaking (pbt.py:130-133)
        Ps = [unflatten(fp, lay, ad) for fp in flat_p]
        B = N // len(Ps)

        def forward_all(x):
            outs = [forward(Pp, x[p * B:(p + 1) * B], mode, ad) for p, Pp in enumerate(Ps)]
            return (np.concatenate([o[0] for o in outs]), np.concatenate([o[1] for o in outs]),
                    None)
    else:
        P = unflatten(flat_p, lay, ad)

        def forward_all(x):
            return forward(P, x, mode, ad)
    A = int(sum(buckets))
    K = len(buckets)
    store = {k: [] for k in ("obs", "actions", "log_probs", "values", "rewards", "dones")}
    store["logits"] = []
    er = np.zeros(N, np.float32) if env_returns is None else env_returns
    trace = []
    obs = env.obs.copy()
    prep = (lambda o: rnd(o, mode, ad)) if obs_norm is None else \
        (lambda o: ema_normalize(obs_norm[0], o, mode).astype(ad))
    ostats = (np.zeros(env.D, np.float32), np.zeros(env.D, np.float32))
    for t in range(T):
        x = prep(obs)
        if obs_norm is not None:
            ostats = ema_update_input_stats(ostats, t, obs)
        logits, V, _ = forward_all(x)
        gum = native.gumbel_table(key[0], key[1], step_base + t, env.eoff, N, A)
        acts, logp = sample_actions(logits.astype(np.float32), buckets, gum)
        if actions_override is not None:
            acts = np.asarray(actions_override[t], np.int32)
            logp, _ = action_stats(logits, buckets, acts)
        store["obs"].append(x.astype(np.float32))
        store["actions"].append(acts)
        store["log_probs"].append(logp.astype(np.float32))
        store["values"].append(V.astype(np.float32))
        store["logits"].append(logits.astype(np.float32))
        obs, rew, done = env.step(acts)
        er = (rew + np.float32(gamma) * er).astype(np.float32)
        trace.append(er.copy())
        store["rewards"].append(rew)
        store["dones"].append(done)
        er = np.where(done.astype(bool), np.float32(0), er).astype(np.float32)
    _, boot, _ = forward_all(prep(obs))
    out = _finish_store(store, boot, trace)
    if obs_norm is not None:
        out["obs_est"] = ema_update_estimates(obs_norm[0], ostats, obs_norm[1], obs_norm[2])
    return out, er


def _finish_store(store, boot, trace):
    out = {k: np.stack(v) for k, v in store.items()}
    out["bootstrap"] = np.asarray(boot).astype(np.float32)
    out["env_returns_trace"] = np.stack(trace)
    return out


def _rollout_fake(policy_fn, env, T, gamma, env_returns):
    """Same store / bookkeeping order as rollout() with a pluggable policy
    (rollouts.py:829-978: infer -> store -> sim step -> done bookkeeping)."""
    store = {k: [] for k in ("obs", "actions", "log_probs", "values", "rewards", "dones")}
    er = np.zeros(env.N, np.float32) if env_returns is None else env_returns
    trace = []
    obs = env.obs.copy()
    for t in range(T):
        acts, logp, V = policy_fn(obs)
        store["obs"].append(obs.copy())
        store["actions"].append(acts)
        store["log_probs"].append(logp)
        store["values"].append(V)
        obs, rew, done = env.step(acts)
        er = (rew + np.float32(gamma) * er).astype(np.float32)
        trace.append(er.copy())
        store["rewards"].append(rew)
        store["dones"].append(done)
        er = np.where(done.astype(bool), np.float32(0), er).astype(np.float32)
    _, _, boot = policy_fn(obs)
    return _finish_store(store, boot, trace), er



