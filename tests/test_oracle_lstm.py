"""The LSTM oracle (oracle/lstm_ref.py): its hand-written BPTT equals fp64
autograd of the same restated forward (RecurrentBackboneEncoder.sequence,
actor_critic.py:179-199 + LSTM.sequence, rnn.py:81-111, with carries cleared
after done steps), closed-form cell cases, and the recurrent rollout carry
(rollouts.py:528-537, 898-901, 942) on the oracle env."""

import numpy as np
import pytest
import torch

from oracle import lstm_ref as lref
from oracle import native
from oracle import ppo_ref as ref
from tests.test_oracle_grads import BUCKETS


def torch_loss(P, batch, hp, buckets, adv_stats):
    x = torch.tensor(batch["obs"], dtype=torch.float64)
    h = x
    for l in range(len(P["W"])):
        z = h @ P["W"][l]
        mean = z.mean(-1, keepdim=True)
        var = torch.clamp((z * z).mean(-1, keepdim=True) - mean * mean, min=0)
        y = (z - mean) * (torch.rsqrt(var + ref.LN_EPS) * P["s"][l]) + P["b"][l]
        h = torch.relu(y)
    F = h
    H = P["Wr"].shape[0]
    mb = batch["start_h"].shape[0]
    bptt = F.shape[0] // mb
    hc = torch.tensor(batch["start_h"], dtype=torch.float64)
    cc = torch.tensor(batch["start_c"], dtype=torch.float64)
    done = torch.tensor(np.asarray(batch["dones"]).reshape(bptt, mb).astype(bool))
    outs = []
    for t in range(bptt):
        pre = F[t * mb:(t + 1) * mb] @ P["Wi"] + hc @ P["Wr"] + P["bl"]
        i, f = torch.sigmoid(pre[:, :H]), torch.sigmoid(pre[:, H:2 * H])
        g, o = torch.tanh(pre[:, 2 * H:3 * H]), torch.sigmoid(pre[:, 3 * H:])
        c2 = f * cc + i * g
        h2 = o * torch.tanh(c2)
        outs.append(h2)
        m = done[t][:, None]
        hc = torch.where(m, torch.zeros_like(h2), h2)
        cc = torch.where(m, torch.zeros_like(c2), c2)
    Hout = torch.cat(outs, 0)
    out = Hout @ P["Wh"] + P["bh"]
    A = out.shape[1] - 1
    logits, V = out[:, :A], out[:, A]
    adv = torch.tensor(batch["advantages"], dtype=torch.float64)
    mean, var = adv_stats
    adv = (adv - mean) / np.sqrt(max(var, 1e-5))
    acts = torch.tensor(batch["actions"], dtype=torch.int64)
    old = torch.tensor(batch["log_probs"], dtype=torch.float64)
    objs, ents = [], []
    off = 0
    for gi, nb in enumerate(buckets):
        sl = logits[:, off:off + nb]
        lp = sl - torch.logsumexp(sl, -1, keepdim=True)
        ent = -(torch.softmax(sl, -1) * lp).sum(-1)
        ratio = torch.exp(lp.gather(1, acts[:, gi:gi + 1])[:, 0] - old[:, gi])
        c = hp["clip_coef"]
        objs.append(torch.minimum(adv * ratio, adv * torch.clamp(ratio, 1 - c, 1 + c)))
        ents.append(ent)
        off += nb
    R = torch.tensor(batch["returns"], dtype=torch.float64)
    vl = 0.5 * (V - R) ** 2
    return (-torch.stack(objs, -1).mean() + hp["value_loss_coef"] * vl.mean()
            - hp["entropy_coef"] * torch.stack(ents, -1).mean())


def _batch(rng, D, H, mb, bptt, done_p=0.2):
    M = mb * bptt
    acts = np.stack([rng.integers(0, b, M) for b in BUCKETS], -1)
    return {"obs": rng.standard_normal((M, D)), "actions": acts,
            "log_probs": rng.standard_normal((M, 6)) * 0.3 - 1.5,
            "advantages": rng.standard_normal(M) + 0.2, "returns": rng.standard_normal(M),
            "values": rng.standard_normal(M), "dones": rng.random(M) < done_p,
            "start_h": rng.standard_normal((mb, H)) * 0.5,
            "start_c": rng.standard_normal((mb, H)) * 0.5}


@pytest.mark.parametrize("H,L,mb,bptt", [(32, 2, 8, 6), (16, 1, 5, 9)])
def test_bptt_matches_autograd(H, L, mb, bptt):
    rng = np.random.default_rng(H * 7 + L)
    D = 24
    lay, P = lref.init_params(rng, D, H, L, BUCKETS)
    flat = lref.flatten(P, lay) + rng.standard_normal(lay["total"]) * 0.05
    P = lref.unflatten(flat, lay)
    for l in range(L):
        P["s"][l] = 1.0 + 0.3 * rng.standard_normal(H)
    batch = _batch(rng, D, H, mb, bptt)
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01}
    stats = (batch["advantages"].mean(), batch["advantages"].var())
    loss, G, _, _ = lref.ppo_loss_grads(P, batch, hp, BUCKETS, "f64", adv_stats=stats)
    TP = {k: ([torch.tensor(x, requires_grad=True) for x in v] if isinstance(v, list)
              else torch.tensor(v, requires_grad=True)) for k, v in P.items() if k != "CB"}
    tl = torch_loss(TP, batch, hp, BUCKETS, stats)
    tl.backward()
    np.testing.assert_allclose(loss, tl.item(), rtol=1e-12)
    for k in ("W", "s", "b"):
        for l in range(L):
            np.testing.assert_allclose(G[k][l], TP[k][l].grad.numpy(), rtol=1e-7, atol=1e-12)
    for k in ("Wh", "bh", "Wi", "Wr", "bl"):
        np.testing.assert_allclose(G[k], TP[k].grad.numpy(), rtol=1e-7, atol=1e-12)


def test_cell_closed_form():
    """Zero weights: every gate is sigmoid(b) / tanh(b); c' = f c + i g."""
    H = 4
    P = {"Wi": np.zeros((3, 4 * H)), "Wr": np.zeros((H, 4 * H)),
         "bl": np.concatenate([np.full(H, 0.5), np.full(H, -1.0), np.full(H, 2.0),
                               np.full(H, 0.0)])}
    c = np.array([[0.3, -0.2, 1.0, 0.0]])
    h2, c2, (i, f, g, o) = lref.lstm_cell(P, np.ones((1, 3)), np.ones((1, H)), c, "f64")
    si, sf, tg, so = 1 / (1 + np.exp(-0.5)), 1 / (1 + np.exp(1.0)), np.tanh(2.0), 0.5
    np.testing.assert_allclose(c2, sf * c + si * tg, rtol=1e-14)
    np.testing.assert_allclose(h2, so * np.tanh(sf * c + si * tg), rtol=1e-14)


def test_rollout_carry_and_start_states():
    """Start states are the (cleared) carries at every chunk start; a done env
    starts its next step from zeros; the bootstrap does not advance the carry."""
    rng = np.random.default_rng(4)
    N, D, H, T, bptt = 16, 16, 16, 8, 4
    lay, P = lref.init_params(rng, D, H, 1, BUCKETS)
    flat = lref.flatten(P, lay)
    env = native.Env(N, D, 3, 4, 0)
    env.reset()
    z = np.zeros((N, H))
    store, (h, c), _ = lref.rollout(flat, lay, env, T, bptt, BUCKETS, (1, 2), 0, (z, z),
                                    mode="f64")
    assert store["start_h"].shape == (T // bptt, N, H)
    assert np.all(store["start_h"][0] == 0)
    # replay step by step
    env2 = native.Env(N, D, 3, 4, 0)
    env2.reset()
    hh, cc = z, z
    PP = lref.unflatten(flat, lay)
    for t in range(T):
        if t % bptt == 0:
            np.testing.assert_array_equal(store["start_h"][t // bptt], hh)
            np.testing.assert_array_equal(store["start_c"][t // bptt], cc)
        _, _, h2, c2 = lref.policy_step(PP, store["obs"][t].astype(np.float64), hh, cc, "f64")
        d = store["dones"][t].astype(bool)[:, None]
        hh, cc = np.where(d, 0.0, h2), np.where(d, 0.0, c2)
    np.testing.assert_array_equal(h, hh)
    np.testing.assert_array_equal(c, cc)
    assert store["dones"].any()
