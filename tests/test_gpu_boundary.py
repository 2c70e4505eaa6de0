"""The reference's callable plugin surface (actor_critic.py:55-128):
ActorCritic.rollout / actor_only / critic_only / update on
  * a recognised tree (fused HIP kernels, lazily compiled PolicyState),
    checked against the oracle forward (models.py:99-154, dists.py:26-77);
  * a recognised recurrent tree (LSTM carry through rollout steps vs the
    update's sequence with breaks, rnn.py:81-111);
  * a user-defined tree (plain torch slow path, distribution math on the
    HIP kernels).
"""

import numpy as np
import pytest
import torch
from torch import nn

from oracle import native as onat
from oracle import ppo_ref as ref

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]


def _ac(dtype, H, recurrent=False):
    import madrona_learn as ml
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
    from madrona_learn.rnn import LSTM
    enc = ml.RecurrentBackboneEncoder(net=MLP(H, 2, dtype), rnn=LSTM(H, 1, dtype)) if recurrent \
        else ml.BackboneEncoder(net=MLP(H, 2, dtype))
    return ml.ActorCritic(backbone=ml.BackboneShared(encoder=enc),
                          actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dtype),
                          critic=DenseLayerCritic(dtype))


@pytest.mark.parametrize("mode,dtype,H", [("f32", torch.float32, 64),
                                          ("bf16", torch.bfloat16, 256)])
def test_recognised_tree_methods(gpu, mode, dtype, H):
    from madrona_learn.dists import PhiloxKey
    N, D = 96, 64
    torch.manual_seed(0)
    ac = _ac(dtype, H)
    obs = torch.randn((N, D), device=gpu)
    key = PhiloxKey(11, 22, step=3, env_offset=5)
    out, st = ac.rollout(key, (), obs)
    ps = ac.policy_state
    assert ps is not None, "recognised tree must take the fused path"
    assert st == ()
    lay = ref.param_layout(D, H, 2, 26)
    P = ref.unflatten(ps.params.cpu().numpy().astype(np.float64), lay)
    logits, V, _ = ref.forward(P, obs.cpu().numpy().astype(np.float64), mode)
    tol = 1e-4 if mode == "f32" else 3e-2
    np.testing.assert_allclose(out["critic"][:, 0].cpu().numpy(), V, rtol=tol, atol=tol)
    acts = out["actions"].cpu().numpy()
    lp, ent = ref.action_stats(logits, BUCKETS, acts)
    np.testing.assert_allclose(out["log_probs"].cpu().numpy(), lp, rtol=tol, atol=tol)
    # Gumbel-max with the oracle's noise table, wherever the margin is clear
    noisy = logits + onat.gumbel_table(11, 22, 3, 5, N, 26)
    off = 0
    for g, nb in enumerate(BUCKETS):
        sl = np.sort(noisy[:, off:off + nb], -1)
        clear = (sl[:, -1] - sl[:, -2]) > 1e-3
        assert np.array_equal(np.argmax(noisy[:, off:off + nb], -1)[clear], acts[clear, g])
        off += nb
    # update on the same rows (T = 2 copies): log-probs of the sampled actions
    # are the rollout's bit for bit, entropies and critic match the oracle
    T = 2
    seq_obs = obs[None].expand(T, N, D).contiguous()
    seq_act = out["actions"][None].expand(T, N, len(BUCKETS)).contiguous()
    breaks = torch.zeros((T, N, 1), dtype=torch.bool, device=gpu)
    upd = ac.update((), breaks, {"actions": seq_act}, seq_obs)
    assert upd["log_probs"].shape == (T, N, len(BUCKETS))
    assert torch.equal(upd["log_probs"][0], out["log_probs"])
    assert torch.equal(upd["log_probs"][1], out["log_probs"])
    assert torch.equal(upd["critic"][0], out["critic"])
    np.testing.assert_allclose(upd["entropies"][1].cpu().numpy(), ent, rtol=tol, atol=tol)
    # actor_only = best() (first-index argmax of the logits), critic_only
    a_only, _ = ac.actor_only((), obs)
    off = 0
    for g, nb in enumerate(BUCKETS):
        sl = np.sort(logits[:, off:off + nb], -1)
        clear = (sl[:, -1] - sl[:, -2]) > 1e-3
        got = a_only["actions"][:, g].cpu().numpy()
        assert np.array_equal(np.argmax(logits[:, off:off + nb], -1)[clear], got[clear])
        off += nb
    c_only, _ = ac.critic_only((), obs)
    assert torch.equal(c_only["critic"], out["critic"])


def test_recognised_recurrent_tree(gpu):
    """Step-by-step rollout with the carry (cleared after episode ends) and
    the update's sequence over the same steps agree bit for bit."""
    from madrona_learn.dists import PhiloxKey
    N, D, H, T = 64, 64, 64, 5
    torch.manual_seed(1)
    ac = _ac(torch.float32, H, recurrent=True)
    obs = torch.randn((T, N, D), device=gpu)
    breaks = (torch.rand((T, N, 1), device=gpu) < 0.3)
    start = ac.init_recurrent_state(N)
    start = ([start[0][0].to(gpu)], [start[1][0].to(gpu)])
    st = start
    lps, vals, acts = [], [], []
    for t in range(T):
        out, st = ac.rollout(PhiloxKey(3, 4, step=t), st, obs[t])
        assert ac.policy_state is not None and ac.policy_state.recurrent
        lps.append(out["log_probs"])
        vals.append(out["critic"])
        acts.append(out["actions"])
        st = ac.clear_recurrent_state(st, breaks[t])
    upd = ac.update(start, breaks, torch.stack(acts), obs)
    for t in range(T):
        assert torch.equal(upd["log_probs"][t], lps[t]), t
        assert torch.equal(upd["critic"][t], vals[t]), t
    assert torch.isfinite(upd["entropies"]).all()


class _TanhNet(nn.Module):
    """A user's own trunk (not an MLP the engine compiles)."""

    def __init__(self, D, H):
        super().__init__()
        self.l1 = nn.Linear(D, H)
        self.l2 = nn.Linear(H, H)

    def forward(self, x, train=False):
        return torch.tanh(self.l2(torch.tanh(self.l1(x))))


class _UserBackbone(nn.Module):
    """A user's own Backbone (actor_critic.py:13-35 protocol), separate
    actor / critic features."""

    def __init__(self, D, H):
        super().__init__()
        self.a = _TanhNet(D, H)
        self.c = _TanhNet(D, H)

    def init_recurrent_state(self, N):
        return ()

    def clear_recurrent_state(self, s, m):
        return ()

    def forward(self, rnn_states, obs, train=False):
        return self.a(obs), self.c(obs), ()

    def actor_only(self, rnn_states, obs, train=False):
        return self.a(obs), ()

    def critic_only(self, rnn_states, obs, train=False):
        return self.c(obs), ()

    def sequence(self, start, ends, obs, train=False):
        flat = obs.reshape(-1, obs.shape[-1])
        return self.a(flat), self.c(flat)


@pytest.mark.parametrize("kind", ["custom_net", "custom_backbone"])
def test_custom_tree_slow_path(gpu, kind):
    import madrona_learn as ml
    from madrona_learn.dists import PhiloxKey
    from madrona_learn.models import DenseLayerCritic, DenseLayerDiscreteActor
    N, D, H, T = 80, 32, 48, 3
    torch.manual_seed(2)
    if kind == "custom_net":
        bb = ml.BackboneShared(encoder=ml.BackboneEncoder(net=_TanhNet(D, H)))
    else:
        bb = _UserBackbone(D, H)
    ac = ml.ActorCritic(backbone=bb,
                        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS),
                                                      torch.float32),
                        critic=DenseLayerCritic(torch.float32)).to(gpu)
    obs = torch.randn((T, N, D), device=gpu)
    out, _ = ac.rollout(PhiloxKey(5, 6), (), obs[0])
    assert ac.policy_state is None, "a user tree must run on the torch slow path"
    assert out["actions"].shape == (N, len(BUCKETS)) and out["critic"].shape == (N, 1)
    with torch.no_grad():
        feats = (bb.encoder.net(obs[0]) if kind == "custom_net" else bb.a(obs[0]))
        logits = ac.actor.impl(feats).double().cpu().numpy()
    lp, ent = ref.action_stats(logits, BUCKETS, out["actions"].cpu().numpy())
    np.testing.assert_allclose(out["log_probs"].detach().cpu().numpy(), lp, rtol=1e-5,
                               atol=1e-5)
    acts = torch.stack([out["actions"]] * T)
    upd = ac.update((), torch.zeros((T, N, 1), dtype=torch.bool, device=gpu), acts, obs)
    assert upd["log_probs"].shape == (T, N, len(BUCKETS))
    np.testing.assert_allclose(upd["log_probs"][0].detach().cpu().numpy(), lp, rtol=1e-5,
                               atol=1e-5)
    np.testing.assert_allclose(upd["entropies"][0].detach().cpu().numpy(), ent, rtol=1e-5,
                               atol=1e-5)
    torch.testing.assert_close(upd["critic"][0], out["critic"])
    # slow-path gradients flow into the user's parameters (torch autograd)
    upd["critic"].sum().backward()
    grads = [p.grad for p in ac.critic.parameters()]
    assert grads and all(g is not None for g in grads)
