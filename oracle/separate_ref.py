"""NumPy restatement of the PPO update for a BackboneSeparate policy
(actor_critic.py:247-303: separate actor and critic encoders over the same
observations), as the torch path of init_training trains it
(madrona_learn/generic.py).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Built from the pieces of
ppo_ref (the MLP trunk and its backward, the PPO loss and its d / d head
outputs, clip + Adam), with the projections of ppo.py:303-338 over both
trunks.  Parameters are a dict of named arrays (the torch module names).
"""

import numpy as np

from . import ppo_ref as ref


def _enc(named, which, L):
    pre = f"backbone.{which}_encoder.net"
    return {"W": [named[f"{pre}.dense.{l}.kernel"] for l in range(L)],
            "s": [named[f"{pre}.norms.{l}.scale"] for l in range(L)],
            "b": [named[f"{pre}.norms.{l}.bias"] for l in range(L)]}


def _head(h, W, b, mode, ad):
    """Dense with bias, outputs in f32 (models.py:122-154), as head_outputs."""
    return ref.rnd(ref.rnd(h @ ref.rnd(W, mode, ad), mode, ad) + ref.rnd(b, mode, ad), mode, ad)


def forward(named, x, L, mode, ad=np.float64):
    """(logits [M,A], value [M], caches) of BackboneSeparate(MLP, MLP) with
    DenseLayerDiscreteActor / DenseLayerCritic."""
    Pa, Pc = _enc(named, "actor", L), _enc(named, "critic", L)
    ha, ca = ref.trunk(Pa, x, mode, ad)
    hc, cc = ref.trunk(Pc, x, mode, ad)
    logits = _head(ha, named["actor.impl.kernel"], named["actor.impl.bias"], mode, ad)
    V = _head(hc, named["critic.impl.kernel"], named["critic.impl.bias"], mode, ad)[:, 0]
    return logits, V, (Pa, Pc, ha, hc, ca, cc)


def loss_grads(named, batch, hp, buckets, L, mode="f64", adv_stats=None, ad=np.float64):
    """Loss (ppo.py:129-262) and d loss / d every named parameter."""
    logits, V, (Pa, Pc, ha, hc, ca, cc) = forward(named, batch["obs"], L, mode, ad)
    loss, dhead, met = ref.ppo_loss_dhead(logits, V, batch, hp, buckets, adv_stats, 1.0, ad)
    dhead = ref.rnd(dhead, mode, ad)
    A = logits.shape[1]
    dla, dv = dhead[:, :A], dhead[:, A:]
    G = {"actor.impl.kernel": ha.T @ dla, "actor.impl.bias": dla.sum(0),
         "critic.impl.kernel": hc.T @ dv, "critic.impl.bias": dv.sum(0)}
    for which, P, cache, da in (
            ("actor", Pa, ca, dla @ ref.rnd(named["actor.impl.kernel"], mode, ad).T),
            ("critic", Pc, cc, dv @ ref.rnd(named["critic.impl.kernel"], mode, ad).T)):
        Gt = {"W": [None] * L, "s": [None] * L, "b": [None] * L}
        ref.trunk_backward(P, cache, da, Gt, mode, ad)
        pre = f"backbone.{which}_encoder.net"
        for l in range(L):
            G[f"{pre}.dense.{l}.kernel"] = Gt["W"][l]
            G[f"{pre}.norms.{l}.scale"] = Gt["s"][l]
            G[f"{pre}.norms.{l}.bias"] = Gt["b"][l]
    return loss, G, met


def project(named, init_norms, L):
    """normalize_params (ppo.py:303-310) on both trunks' kernels (the heads
    live under actor / critic: no initial norm) and normalize_layernorms
    (ppo.py:312-338) on both trunks' LayerNorms."""
    for which in ("actor", "critic"):
        pre = f"backbone.{which}_encoder.net"
        for l in range(L):
            k = f"{pre}.dense.{l}.kernel"
            W = named[k]
            named[k] = (init_norms[k] * W) / np.sqrt((W * W).sum())
            s, b = named[f"{pre}.norms.{l}.scale"], named[f"{pre}.norms.{l}.bias"]
            f = np.sqrt(s.shape[-1] / (np.dot(b, b) + np.dot(s, s)))
            named[f"{pre}.norms.{l}.scale"] = f * s
            named[f"{pre}.norms.{l}.bias"] = f * b
    return named


def ppo_update(named, order, store, hp, buckets, L, init_norms, *, num_epochs, minibatch_size,
               bptt, key, epoch_base, mode, lr, max_grad_norm, ad=np.float64, value_norm=None,
               value_norm_decay=0.99999):
    """_ppo (ppo.py:366-488): the same minibatch plan as ppo_ref.ppo_update;
    the optimizer runs over the flat vector in `order` (the parameter names in
    the torch arena's order).  `store` is one rank's [T][N] store or a list of
    them (data parallelism: each optimizer step over the union of the ranks'
    minibatches -- union advantage statistics, gradient = sum over ranks of
    the rank-local gradients of the loss scaled by 1 / world).  value_norm
    (normalize_values, ppo.py:190-211): the EMANormalizer estimates
    (ppo_ref.ema_init), moved minibatch by minibatch as in
    ppo_ref.ppo_update."""
    stores = store if isinstance(store, (list, tuple)) else [store]
    world = len(stores)
    store = stores[0]
    T, N = store["rewards"].shape
    nseq = (T // bptt) * N
    nmb = nseq // minibatch_size
    flat = np.concatenate([np.asarray(named[k], ad).reshape(-1) for k in order])
    shapes = [np.asarray(named[k]).shape for k in order]
    sizes = [int(np.prod(s)) for s in shapes]

    def unflat(v):
        out, o = {}, 0
        for k, s, n in zip(order, shapes, sizes):
            out[k] = v[o:o + n].reshape(s)
            o += n
        return out

    m, v = np.zeros_like(flat), np.zeros_like(flat)
    count = 0
    met = None
    for e in range(num_epochs):
        perms = [ref.epoch_permutation(key[0], key[1], epoch_base + e, r, nseq)
                 for r in range(world)]
        for i in range(nmb):
            bs = [ref.gather_minibatch(stores[r], ref.minibatch_rows(
                perms[r][i * minibatch_size:(i + 1) * minibatch_size], N, bptt))
                for r in range(world)]
            adv = np.concatenate([np.asarray(b[ref.objective_key(hp)], np.float64) for b in bs])
            hp_mb = hp
            if value_norm is not None:  # as ppo_ref.ppo_update (ppo.py:209-211, 346)
                allret = np.concatenate([np.asarray(b["returns"], np.float64) for b in bs])
                z = np.zeros(1, np.float32)
                new = ref.ema_update_estimates(value_norm, ref.ema_update_input_stats(
                    (z, z), 0, allret[:, None]), value_norm_decay, 1e-5)
                hp_mb = dict(hp, value_norm=(float(new["mu"][0]), float(new["inv_sigma"][0]),
                                             float(value_norm["mu"][0]),
                                             float(value_norm["sigma"][0])))
                value_norm.update(new)
            g = None
            for r, b in enumerate(bs):
                _, G, m_r = loss_grads(unflat(flat), b, hp_mb, buckets, L, mode,
                                       (adv.mean(), adv.var()), ad)
                gr = np.concatenate([np.asarray(G[k], ad).reshape(-1) for k in order]) / world
                g = gr if g is None else g + gr
                if r == 0:
                    met = m_r
            g, _ = ref.clip_by_global_norm(g, max_grad_norm)
            flat, m, v = ref.adam_step(flat, g, m, v, count, lr)
            count += 1
            P = project(unflat(flat), init_norms, L)
            flat = np.concatenate([np.asarray(P[k], ad).reshape(-1) for k in order])
    return unflat(flat), met
