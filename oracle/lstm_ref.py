"""NumPy restatement of the recurrent (LSTM) policy path.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates, from the
reference (paths relative to shacklettbp/madrona-learn src/madrona_learn/):
  * RecurrentBackboneEncoder (actor_critic.py:156-199): MLP trunk -> LSTM;
    the heads read the LSTM output;
  * LSTM / MultiLayerLSTMCell (rnn.py:10-111) with one layer, whose cell is
    flax 0.8.1 nn.OptimizedLSTMCell (third-party, restated from its published
    definition): input kernels Wi [in, 4H] without bias, hidden kernels
    Wh [H, 4H] with bias, gate blocks (i, f, g, o) concatenated along the
    output axis; i, f, o = sigmoid, g = tanh; c' = f*c + i*g; h' = o*tanh(c');
    output = h'.  Initialisers: orthogonal per gate block, bias 0 (rnn.py:30-36);
  * the rollout carry (rollouts.py:898-901, 942): state cleared where the env
    step reports done; the state at the start of every BPTT chunk is saved as
    rnn_start_states (rollouts.py:533-537);
  * LSTM.sequence (rnn.py:81-111): nn.scan over the chunk from the start state,
    clearing the carry AFTER step t where dones[t] (sequence_breaks = the
    minibatch's dones, actor_critic.py:98-128, ppo.py:123);
  * weight-norm projection of every backbone `kernel` leaf, which for the
    LSTM is each of the 8 gate kernels ii..io, hi..ho separately
    (ppo.py:303-310, train_state.py:413-423).

Precision contract (shared with the HIP kernels; the reference's bf16
rounding points inside the cell are XLA fusion decisions no reference test
pins): gate pre-activations = x@Wi + h@Wh + bias accumulated in f32 (one
rounding point fewer than two separately rounded Dense outputs); gate
activations, c' and h' rounded to the compute dtype; backward: gate
pre-activation cotangents rounded to the compute dtype, the recurrent h / c
cotangents carried in f32, d features rounded to the compute dtype.

Parameter layout: the MLP layout of ppo_ref.param_layout padded to a multiple
of 64 floats, then Wi [H][4H], Wh [H][4H], bias [4H] (mlearn_lstm_param_*).
"""

import numpy as np

from . import native
from . import ppo_ref as ref
from .ppo_ref import rnd

GATES = ("i", "f", "g", "o")


def param_layout(obs_dim, hidden, num_layers, num_logits, critic_bins=1):
    lay = ref.param_layout(obs_dim, hidden, num_layers, num_logits, critic_bins)
    H = hidden
    off = (lay["total"] + 63) // 64 * 64
    lay["lstm_off"] = off
    lay["Wi"] = (off, (H, 4 * H))
    off += 4 * H * H
    lay["Wr"] = (off, (H, 4 * H))
    off += 4 * H * H
    lay["bl"] = (off, (4 * H,))
    off += 4 * H
    lay["total"] = off
    return lay


def unflatten(flat, lay, ad=np.float64):
    P = ref.unflatten(flat, lay, ad)
    flat = np.asarray(flat, ad)
    for k in ("Wi", "Wr", "bl"):
        o, shp = lay[k]
        P[k] = flat[o:o + int(np.prod(shp))].reshape(shp).copy()
    return P


def flatten(P, lay):
    out = ref.flatten(P, lay)  # MLP offsets are unchanged; padding stays zero
    for k in ("Wi", "Wr", "bl"):
        o, shp = lay[k]
        out[o:o + P[k].size] = P[k].reshape(-1)
    return out


def kernel_norms(P):
    """Initial Frobenius norms of every projected kernel, in the order of the
    native init_norms array: trunk W_l, then Wi gate blocks (i, f, g, o), then
    Wh gate blocks (train_state.py:413-423)."""
    H = P["Wr"].shape[0]
    n = [np.linalg.norm(W) for W in P["W"]]
    for k in ("Wi", "Wr"):
        for g in range(4):
            n.append(np.linalg.norm(P[k][:, g * H:(g + 1) * H]))
    return np.array(n)


def init_params(rng, obs_dim, hidden, num_layers, buckets):
    """Reference initialisers (models.py orthogonal(sqrt 2) trunk, 0.01 actor,
    1.0 critic; rnn.py:30-36 orthogonal per LSTM gate, zero bias), restated
    with the product's orthogonal routine."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)),
                                    "madrona-learn_amd"))
    from madrona_learn.models import orthogonal
    A = int(sum(buckets))
    lay = param_layout(obs_dim, hidden, num_layers, A)
    P = {"W": [], "s": [], "b": []}
    for l in range(num_layers):
        fin = obs_dim if l == 0 else hidden
        P["W"].append(orthogonal(np.sqrt(2))(rng, (fin, hidden)).astype(np.float64))
        P["s"].append(np.ones(hidden))
        P["b"].append(np.zeros(hidden))
    P["Wh"] = np.concatenate([orthogonal(0.01)(rng, (hidden, A)),
                              orthogonal(1.0)(rng, (hidden, 1))], 1).astype(np.float64)
    P["bh"] = np.zeros(A + 1)
    P["Wi"] = np.concatenate([orthogonal(1.0)(rng, (hidden, hidden)) for _ in range(4)], 1)
    P["Wr"] = np.concatenate([orthogonal(1.0)(rng, (hidden, hidden)) for _ in range(4)], 1)
    P["Wi"] = P["Wi"].astype(np.float64)
    P["Wr"] = P["Wr"].astype(np.float64)
    P["bl"] = np.zeros(4 * hidden)
    return lay, P


# ---------------------------------------------------------------------------
# cell
# ---------------------------------------------------------------------------
def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm_cell(P, x, h, c, mode, ad=np.float64):
    """OptimizedLSTMCell step (rnn.py:28-41).  x, h, c are compute-dtype
    valued; returns (h', c', gates (i, f, g, o))."""
    H = h.shape[1]
    pre = x @ rnd(P["Wi"], mode, ad) + h @ rnd(P["Wr"], mode, ad) + P["bl"].astype(ad)
    i = rnd(_sigmoid(pre[:, :H]), mode, ad)
    f = rnd(_sigmoid(pre[:, H:2 * H]), mode, ad)
    g = rnd(np.tanh(pre[:, 2 * H:3 * H]), mode, ad)
    o = rnd(_sigmoid(pre[:, 3 * H:]), mode, ad)
    c2 = rnd(f * c + i * g, mode, ad)
    h2 = rnd(o * np.tanh(c2), mode, ad)
    return h2, c2, (i, f, g, o)


def policy_step(P, obs, h, c, mode, ad=np.float64):
    """ActorCritic.rollout with a RecurrentBackboneEncoder (actor_critic.py:
    74-96, 173-177): trunk -> LSTM -> heads.  Returns (logits, V, h', c')."""
    F, _ = ref.trunk(P, obs, mode, ad)
    h2, c2, _ = lstm_cell(P, F, h, c, mode, ad)
    logits, V = ref.heads(P, h2, mode, ad)
    return logits, V, h2, c2


# ---------------------------------------------------------------------------
# rollout (rollouts.py:829-978) with a recurrent policy
# ---------------------------------------------------------------------------
def rollout(flat_p, lay, env, T, bptt, buckets, key, step_base, state, mode="f32", gamma=0.99,
            env_returns=None, ad=np.float64, actions_override=None):
    """rollout_loop with the recurrent carry.  state = (h, c) [N,H] at the
    start (already cleared where the previous step was done).  Returns
    (store incl. start_h / start_c [C,N,H], final state, env returns)."""
    P = unflatten(flat_p, lay, ad)
    N = env.N
    A = int(sum(buckets))
    h, c = (np.asarray(s, ad) for s in state)
    store = {k: [] for k in ("obs", "actions", "log_probs", "values", "rewards", "dones",
                             "logits")}
    start_h, start_c = [], []
    er = np.zeros(N, np.float32) if env_returns is None else env_returns
    trace = []
    obs = env.obs.copy()
    for t in range(T):
        if t % bptt == 0:  # collect_state.save(rnn_start_states) (rollouts.py:528-531)
            start_h.append(h.copy())
            start_c.append(c.copy())
        x = rnd(obs, mode, ad)
        logits, V, h2, c2 = policy_step(P, x, h, c, mode, ad)
        gum = native.gumbel_table(key[0], key[1], step_base + t, env.eoff, N, A)
        acts, logp = ref.sample_actions(logits.astype(np.float32), buckets, gum)
        if actions_override is not None:
            acts = np.asarray(actions_override[t], np.int32)
            logp, _ = ref.action_stats(logits, buckets, acts)
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
        m = done.astype(bool)[:, None]  # rnn_reset_fn (rollouts.py:942)
        h = np.where(m, 0.0, h2)
        c = np.where(m, 0.0, c2)
    # bootstrap critic (rollouts.py:607-635): the carry is not advanced
    _, boot, _, _ = policy_step(P, rnd(obs, mode, ad), h, c, mode, ad)
    out = ref._finish_store(store, boot, trace)
    out["start_h"] = np.stack(start_h)
    out["start_c"] = np.stack(start_c)
    return out, (h, c), er


# ---------------------------------------------------------------------------
# PPO loss + BPTT gradients of one minibatch
# ---------------------------------------------------------------------------
def ppo_loss_grads(P, batch, hp, buckets, mode="f64", adv_stats=None, loss_scale=1.0,
                   ad=np.float64):
    """ActorCritic.update (actor_critic.py:98-128) with RecurrentBackbone-
    Encoder.sequence (actor_critic.py:179-199) + LSTM.sequence (rnn.py:92-111),
    the PPO loss (ppo.py:129-262) and its gradient by hand-written BPTT.
    batch rows are time-major (row = t*mb + m): obs [M,D], actions, log_probs,
    advantages, returns, values, dones [M]; start_h / start_c [mb,H]."""
    H = P["Wr"].shape[0]
    h0 = np.asarray(batch["start_h"], ad)
    c0 = np.asarray(batch["start_c"], ad)
    mb = h0.shape[0]
    M = np.asarray(batch["obs"]).shape[0]
    bptt = M // mb
    F, cache = ref.trunk(P, batch["obs"], mode, ad)
    done = np.asarray(batch["dones"]).astype(bool).reshape(bptt, mb)
    hin, cin = h0, c0
    rec = []
    Hout = np.zeros((M, H), ad)
    for t in range(bptt):
        Ft = F[t * mb:(t + 1) * mb]
        h2, c2, gates = lstm_cell(P, Ft, hin, cin, mode, ad)
        rec.append((hin, cin, c2, gates))
        Hout[t * mb:(t + 1) * mb] = h2
        m = done[t][:, None]
        hin = np.where(m, 0.0, h2)
        cin = np.where(m, 0.0, c2)
    logits, crit = ref.head_outputs(P, Hout, mode, ad)
    V = ref.value_estimate(crit)
    loss, dhead, metrics = ref.ppo_loss_dhead(logits, crit, batch, hp, buckets, adv_stats,
                                              loss_scale, ad)
    dhead = rnd(dhead, mode, ad)
    G = {"W": [None] * len(P["W"]), "s": [None] * len(P["W"]), "b": [None] * len(P["W"])}
    G["Wh"] = Hout.T @ dhead
    G["bh"] = dhead.sum(0)
    dHout = rnd(dhead @ rnd(P["Wh"], mode, ad).T, mode, ad)
    # BPTT (reverse scan)
    Wcat = np.concatenate([rnd(P["Wi"], mode, ad), rnd(P["Wr"], mode, ad)], 0)  # [2H, 4H]
    dh_c = np.zeros((mb, H), ad)
    dc_c = np.zeros((mb, H), ad)
    dF = np.zeros((M, H), ad)
    dG = np.zeros((M, 4 * H), ad)
    Hin = np.zeros((M, H), ad)
    for t in range(bptt - 1, -1, -1):
        hin_t, cin_t, c_t, (i, f, g, o) = rec[t]
        m = done[t][:, None]
        dh = dHout[t * mb:(t + 1) * mb] + np.where(m, 0.0, dh_c)
        dcn = np.where(m, 0.0, dc_c)
        tc = np.tanh(c_t)
        do = dh * tc
        dc = dcn + dh * o * (1.0 - tc * tc)
        di = dc * g
        dgg = dc * i
        df = dc * cin_t
        dc_c = dc * f
        dGt = np.concatenate([di * i * (1.0 - i), df * f * (1.0 - f), dgg * (1.0 - g * g),
                              do * o * (1.0 - o)], 1)
        dGt = rnd(dGt, mode, ad)
        dX = dGt @ Wcat.T
        dF[t * mb:(t + 1) * mb] = rnd(dX[:, :H], mode, ad)
        dh_c = dX[:, H:]
        dG[t * mb:(t + 1) * mb] = dGt
        Hin[t * mb:(t + 1) * mb] = hin_t
    G["Wi"] = F.T @ dG
    G["Wr"] = Hin.T @ dG
    G["bl"] = dG.sum(0)
    ref.trunk_backward(P, cache, dF, G, mode, ad)
    return loss, G, metrics, {"logits": logits, "value": V, "dG": dG, "dF": dF, "Hout": Hout}


# ---------------------------------------------------------------------------
# optimizer with the LSTM segment
# ---------------------------------------------------------------------------
def project(P, init_norms):
    """ppo_ref.project + the 8 LSTM gate kernels, each to its initial norm."""
    L = len(P["W"])
    P = ref.project(P, init_norms[:L])
    H = P["Wr"].shape[0]
    j = L
    for k in ("Wi", "Wr"):
        for g in range(4):
            W = P[k][:, g * H:(g + 1) * H]
            P[k][:, g * H:(g + 1) * H] = (init_norms[j] * W) / np.sqrt((W * W).sum())
            j += 1
    return P


def optimizer_step(flat_p, flat_g, m, v, count, lay, init_norms, lr, max_grad_norm):
    g, gn = ref.clip_by_global_norm(flat_g, max_grad_norm)
    p, m, v = ref.adam_step(flat_p, g, m, v, count, lr)
    P = project(unflatten(p, lay), init_norms)
    return flatten(P, lay), m, v, gn


def gather_minibatch(store, seq_ids, bptt):
    """RolloutData.minibatch (rollouts.py:319-329) for the recurrent store:
    rows time-major [bptt, mb], plus the sequences' start states."""
    T, N = store["rewards"].shape
    rows = ref.minibatch_rows(seq_ids, N, bptt)
    b = ref.gather_minibatch(store, rows)
    b["dones"] = np.asarray(store["dones"]).reshape(T * N)[rows]
    seq = np.asarray(seq_ids, np.int64)
    b["start_h"] = store["start_h"][seq // N, seq % N]
    b["start_c"] = store["start_c"][seq // N, seq % N]
    return b


def ppo_update(flat_p, opt, stores, hp, buckets, lay, init_norms, *, num_epochs, minibatch_size,
               bptt, key, epoch_base, mode="f64", lr, max_grad_norm, ad=np.float64):
    """ppo_ref.ppo_update for the recurrent policy."""
    world = len(stores)
    T, N = stores[0]["rewards"].shape
    nseq = (T // bptt) * N
    nmb = nseq // minibatch_size
    m, v, count = opt
    metrics = None
    for e in range(num_epochs):
        perms = [ref.epoch_permutation(key[0], key[1], epoch_base + e, r, nseq)
                 for r in range(world)]
        for mb_i in range(nmb):
            batches = [gather_minibatch(stores[r],
                                        perms[r][mb_i * minibatch_size:(mb_i + 1) * minibatch_size],
                                        bptt) for r in range(world)]
            alladv = np.concatenate([np.asarray(b["advantages"], np.float64) for b in batches])
            stats = (alladv.mean(), alladv.var())
            P = unflatten(flat_p, lay, ad)
            gsum = None
            for b in batches:
                loss, G, met, _ = ppo_loss_grads(P, b, hp, buckets, mode, adv_stats=stats,
                                                 loss_scale=1.0 / world, ad=ad)
                gf = flatten(G, lay)
                gsum = gf if gsum is None else gsum + gf
                if metrics is None or b is batches[0]:
                    metrics = met
            flat_p, m, v, _ = optimizer_step(flat_p, gsum, m, v, count, lay, init_norms, lr,
                                             max_grad_norm)
            count += 1
    return flat_p, (m, v, count), metrics
