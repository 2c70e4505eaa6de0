"""The oracle's hand-written PPO backward equals fp64 autograd of the same
restated forward (torch on CPU) — pins the gradient derivation that the HIP
backward kernels mirror (ppo.py:129-281 under jax.value_and_grad)."""

import numpy as np
import pytest
import torch

from oracle import ppo_ref as ref

BUCKETS = [4, 8, 5, 5, 2, 2]


def torch_loss(P, batch, hp, buckets, adv_stats):
    x = torch.tensor(batch["obs"], dtype=torch.float64)
    h = x
    for l in range(len(P["W"])):
        z = h @ P["W"][l]
        mean = z.mean(-1, keepdim=True)
        var = torch.clamp((z * z).mean(-1, keepdim=True) - mean * mean, min=0)
        y = (z - mean) * (torch.rsqrt(var + ref.LN_EPS) * P["s"][l]) + P["b"][l]
        h = torch.relu(y)
    out = h @ P["Wh"] + P["bh"]
    CB = P.get("CB", 1) if isinstance(P.get("CB", 1), int) else 1
    A = out.shape[1] - CB
    logits, V = out[:, :A], (out[:, A] if CB == 1 else out[:, A:])
    adv = torch.tensor(batch["advantages"], dtype=torch.float64)
    mean, var = adv_stats
    adv = (adv - mean) / np.sqrt(max(var, 1e-5))
    acts = torch.tensor(batch["actions"], dtype=torch.int64)
    old = torch.tensor(batch["log_probs"], dtype=torch.float64)
    objs, ents = [], []
    off = 0
    for g, nb in enumerate(buckets):
        sl = logits[:, off:off + nb]
        lp = sl - torch.logsumexp(sl, -1, keepdim=True)
        ent = -(torch.softmax(sl, -1) * lp).sum(-1)
        ratio = torch.exp(lp.gather(1, acts[:, g:g + 1])[:, 0] - old[:, g])
        c = hp["clip_coef"]
        obj = torch.minimum(adv * ratio, adv * torch.clamp(ratio, 1 - c, 1 + c))
        objs.append(obj)
        ents.append(ent)
        off += nb
    R = torch.tensor(batch["returns"], dtype=torch.float64)
    if CB == 1:
        vl = 0.5 * (V - R) ** 2
    else:  # two-hot cross entropy with constant target weights (dists.py:171-208)
        W = torch.tensor(ref.twohot_weights(CB, batch["returns"]))
        vl = -(W * torch.log_softmax(V, -1)).sum(-1)
    return (-torch.stack(objs, -1).mean() + hp["value_loss_coef"] * vl.mean()
            - hp["entropy_coef"] * torch.stack(ents, -1).mean())


@pytest.mark.parametrize("H,L,CB", [(64, 2, 1), (32, 3, 1), (16, 1, 1), (32, 2, 63), (16, 1, 7)])
def test_backward_matches_autograd(H, L, CB):
    rng = np.random.default_rng(H + L)
    D, M = 24, 200
    lay = ref.param_layout(D, H, L, sum(BUCKETS), CB)
    flat = rng.standard_normal(lay["total"]) * 0.3
    P = ref.unflatten(flat, lay)
    for l in range(L):
        P["s"][l] = 1.0 + 0.3 * rng.standard_normal(H)
    acts = np.stack([rng.integers(0, b, M) for b in BUCKETS], -1)
    batch = {"obs": rng.standard_normal((M, D)), "actions": acts,
             "log_probs": rng.standard_normal((M, 6)) * 0.3 - 1.5,
             "advantages": rng.standard_normal(M) + 0.2,
             "returns": rng.standard_normal(M) * (30.0 if CB > 1 else 1.0),
             "values": rng.standard_normal(M)}
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01}
    stats = (batch["advantages"].mean(), batch["advantages"].var())
    loss, G, _, _ = ref.ppo_loss_grads(P, batch, hp, BUCKETS, "f64", adv_stats=stats)
    TP = {k: ([torch.tensor(x, requires_grad=True) for x in v] if isinstance(v, list)
              else torch.tensor(v, requires_grad=True)) for k, v in P.items() if k != "CB"}
    TP["CB"] = CB
    tl = torch_loss(TP, batch, hp, BUCKETS, stats)
    tl.backward()
    np.testing.assert_allclose(loss, tl.item(), rtol=1e-12)
    for k in ("W", "s", "b"):
        for l in range(L):
            np.testing.assert_allclose(G[k][l], TP[k][l].grad.numpy(), rtol=1e-8, atol=1e-12)
    np.testing.assert_allclose(G["Wh"], TP["Wh"].grad.numpy(), rtol=1e-8, atol=1e-12)
    np.testing.assert_allclose(G["bh"], TP["bh"].grad.numpy(), rtol=1e-8, atol=1e-12)
