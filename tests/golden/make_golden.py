"""Generates the golden fixtures of tests/test_oracle.py from the fp64 / f32
CPU restatement (oracle/).  The reference itself is not importable here (no
JAX), so these fixtures pin the oracle against regressions; the external
anchors are the Random123 vectors and the closed-form cases in the tests.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import ppo_ref as ref  # noqa: E402

BUCKETS = [4, 8, 5, 5, 2, 2]


def gae():
    rng = np.random.default_rng(1234)
    T, N = 32, 64
    r = rng.standard_normal((T, N)).astype(np.float32)
    v = rng.standard_normal((T, N)).astype(np.float32)
    d = (rng.random((T, N)) < 0.1).astype(np.uint8)
    b = rng.standard_normal(N).astype(np.float32)
    adv, ret = ref.gae_f32(r, v, d, b, 0.99, 0.95)
    np.savez(os.path.join(HERE, "gae_32x64.npz"), rewards=r, values=v, dones=d, bootstrap=b,
             gamma=np.float64(0.99), lam=np.float64(0.95), advantages=adv, returns=ret)


def ppo():
    rng = np.random.default_rng(4321)
    D, H, L = 16, 64, 2
    A = sum(BUCKETS)
    lay = ref.param_layout(D, H, L, A)
    p = rng.standard_normal(lay["total"]) * 0.2
    for o, shp in lay["s"]:
        p[o:o + shp[0]] += 1.0
    M = 4 * 16  # 4 sequences x 16 steps
    P = ref.unflatten(p, lay)
    obs = rng.standard_normal((M, D))
    logits, V, _ = ref.forward(P, obs, "f64")
    acts = np.stack([rng.integers(0, nb, M) for nb in BUCKETS], -1).astype(np.int32)
    lp, _ = ref.action_stats(logits, BUCKETS, acts)
    batch = {"obs": obs, "actions": acts, "log_probs": lp + rng.standard_normal(lp.shape) * 0.1,
             "advantages": rng.standard_normal(M) * 2 + 0.3,
             "returns": V + rng.standard_normal(M), "values": V.copy()}
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
          "normalize_advantages": True}
    loss, G, _, _ = ref.ppo_loss_grads(P, batch, hp, BUCKETS, "f64")
    np.savez(os.path.join(HERE, "ppo_4x16.npz"), D=D, H=H, L=L, buckets=np.array(BUCKETS),
             params=p, loss=np.float64(loss), grads=ref.flatten(G, lay), **batch)


def optim():
    rng = np.random.default_rng(99)
    D, H, L, A = 16, 64, 2, 26
    lay = ref.param_layout(D, H, L, A)
    p0 = rng.standard_normal(lay["total"]) * 0.3
    g = rng.standard_normal(lay["total"]) * 0.05
    m0 = rng.standard_normal(lay["total"]) * 0.01
    v0 = rng.random(lay["total"]) * 1e-3
    init = np.array([3.0, 4.0])
    p1, m1, v1, _ = ref.optimizer_step(p0, g, m0, v0, 5, lay, init, 3e-4, 0.5)
    np.savez(os.path.join(HERE, "optim_step.npz"), D=D, H=H, L=L, A=A, p0=p0, grad=g, m0=m0,
             v0=v0, count=5, init_norms=init, lr=3e-4, max_norm=0.5, p1=p1, m1=m1, v1=v1)


if __name__ == "__main__":
    gae()
    ppo()
    optim()
    print("golden fixtures written to", HERE)
