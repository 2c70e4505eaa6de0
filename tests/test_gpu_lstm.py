"""GPU parity of the recurrent (LSTM) policy path against the oracle
(oracle/lstm_ref.py): RecurrentBackboneEncoder(MLP, LSTM) rollout step with
the carry (actor_critic.py:156-199, rollouts.py:898-901, 942), the BPTT
minibatch gradient (rnn.py:81-111 + ppo.py:129-281), the optimizer over the
LSTM segment (ppo.py:283-338), and one full PPO iteration (config L shape).

Tolerances as tests/test_gpu_policy.py: f32 — loss within 1e-5 relative,
values / carries / gradients within 1e-4 (1e-3 relative for gradients) of the
fp64 oracle; bf16 — the oracle emulates the compute-dtype rounding points of
the precision contract in oracle/lstm_ref.py, results within 3e-2 of the
largest magnitude and cosine > 0.999.  Start states (the carry entering a
chunk) and cleared carries are bit-exact.
"""

import numpy as np
import pytest
import torch

from oracle import lstm_ref as lref
from oracle import native as onat
from oracle import ppo_ref as ref

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]


def make_actor_critic(hidden, layers, dtype, critic_bins=1):
    import madrona_learn as ml
    from madrona_learn.models import MLP, DenseLayerDiscreteActor
    from madrona_learn.rnn import LSTM
    from tests.test_gpu_policy import make_critic
    return ml.ActorCritic(
        backbone=ml.BackboneShared(encoder=ml.RecurrentBackboneEncoder(
            net=MLP(hidden, layers, dtype), rnn=LSTM(hidden, 1, dtype))),
        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dtype),
        critic=make_critic(critic_bins, dtype))


def make_policy_state(gpu, obs_dim, hidden, layers, dtype, seed=0, critic_bins=1):
    from madrona_learn.train_state import PolicyState, compile_arch
    ac = make_actor_critic(hidden, layers, dtype, critic_bins)
    arch = compile_arch(ac, obs_dim, dtype)
    assert arch.lstm_hidden == hidden
    return PolicyState(ac, arch, None, gpu, np.random.default_rng(seed))


def oracle_layout(ps):
    a = ps.arch
    lay = lref.param_layout(a.obs_dim, a.hidden, a.num_layers, a.num_logits, a.critic_bins)
    assert lay["total"] == ps.layout["total"] and lay["lstm_off"] == ps.layout["lstm_off"]
    return lay


def perturb(ps, seed, scale=0.05):
    """Non-trivial LayerNorm, head and LSTM-bias parameters."""
    rng = np.random.default_rng(seed)
    p = ps.params.cpu().numpy()
    for key in ("s", "b"):
        for o, shp in ps.layout[key]:
            p[o:o + shp[0]] += rng.standard_normal(shp[0]).astype(np.float32) * 0.3
    for key, sc in (("hw", scale), ("hb", 0.1), ("bl", 0.3)):
        o, shp = ps.layout[key]
        n = int(np.prod(shp))
        p[o:o + n] += rng.standard_normal(n).astype(np.float32) * sc
    if ps.arch.critic_bins > 1:  # zero-initialised two-hot critic: make it non-trivial
        o, shp = ps.layout["hw"]
        hw = p[o:o + shp[0] * shp[1]].reshape(shp)
        hw[:, ps.arch.num_logits:] += rng.standard_normal(
            hw[:, ps.arch.num_logits:].shape).astype(np.float32) * 0.3
    ps.params.copy_(torch.from_numpy(p))
    ps.sync_weights()


def _carry(h, c, sh=None, sc=None, commit=1):
    from madrona_learn import _native as nat
    d = nat.LstmCarry()
    d.h, d.c = h.data_ptr(), c.data_ptr()
    if sh is not None:
        d.start_h, d.start_c = sh.data_ptr(), sc.data_ptr()
    d.commit = commit
    return d


def _post(gpu, N, done_np, rng):
    from madrona_learn import _native as nat
    t = {
        "rew": torch.from_numpy(rng.standard_normal(N).astype(np.float32)).to(gpu),
        "dn": torch.from_numpy(done_np.astype(np.uint8)).to(gpu),
        "srew": torch.zeros(N, dtype=torch.float32, device=gpu),
        "sdn": torch.zeros(N, dtype=torch.uint8, device=gpu),
        "er": torch.zeros(N, dtype=torch.float32, device=gpu),
        "tr": torch.zeros(N, dtype=torch.float32, device=gpu),
    }
    d = nat.PostStep()
    d.rewards, d.dones = t["rew"].data_ptr(), t["dn"].data_ptr()
    d.store_rewards, d.store_dones = t["srew"].data_ptr(), t["sdn"].data_ptr()
    d.env_returns, d.env_returns_trace = t["er"].data_ptr(), t["tr"].data_ptr()
    d.gamma = 0.99
    return d, t


CASES = [("f32", torch.float32, 64, 256, 2), ("bf16", torch.bfloat16, 64, 256, 2),
         ("f32", torch.float32, 32, 64, 2), ("bf16", torch.bfloat16, 48, 128, 1)]


@pytest.mark.parametrize("mode,dtype,D,H,L,CB", [c + (1,) for c in CASES] + [
    ("f32", torch.float32, 64, 256, 2, 63), ("bf16", torch.bfloat16, 32, 64, 2, 63)])
def test_lstm_rollout_step(gpu, mode, dtype, D, H, L, CB):
    ps = make_policy_state(gpu, D, H, L, dtype, seed=D + H, critic_bins=CB)
    perturb(ps, 1)
    N = 1000
    rng = np.random.default_rng(3)
    obs = rng.standard_normal((N, D)).astype(np.float32)
    h0 = ref.rnd(rng.standard_normal((N, H)) * 0.5, mode)
    c0 = ref.rnd(rng.standard_normal((N, H)) * 0.5, mode)
    done = rng.random(N) < 0.2
    o = torch.from_numpy(obs).to(gpu)
    hd = torch.from_numpy(h0.astype(np.float32)).to(gpu, dtype)
    cd = torch.from_numpy(c0.astype(np.float32)).to(gpu, dtype)
    hd2, cd2 = hd.clone(), cd.clone()
    sh, sc = torch.zeros_like(hd), torch.zeros_like(cd)
    store = torch.zeros((N, D), dtype=dtype, device=gpu)
    acts = torch.zeros((N, 6), dtype=torch.int32, device=gpu)
    logp = torch.zeros((N, 6), dtype=torch.float32, device=gpu)
    vals = torch.zeros(N, dtype=torch.float32, device=gpu)
    ctr = torch.tensor([100, 0, 0, 0], dtype=torch.int64, device=gpu)
    post, keep = _post(gpu, N, done, rng)
    ps.rollout_step(o, store, acts, logp, vals, (5, 6), ctr[0:1], 7, env_offset=3, post=post,
                    carry=_carry(hd, cd, sh, sc))
    torch.cuda.synchronize()
    # rnn_reset_fn on the previous step's dones, then the cell
    hin = np.where(done[:, None], 0.0, h0)
    cin = np.where(done[:, None], 0.0, c0)
    P = lref.unflatten(ps.params.cpu().numpy(), oracle_layout(ps))
    logits, V, h2, c2 = lref.policy_step(P, ref.rnd(obs, mode), hin, cin, mode)
    assert np.array_equal(sh.float().cpu().numpy(), hin.astype(np.float32))
    assert np.array_equal(sc.float().cpu().numpy(), cin.astype(np.float32))
    assert np.array_equal(store.float().cpu().numpy(), ref.rnd(obs, mode).astype(np.float32))
    assert np.array_equal(keep["sdn"].cpu().numpy(), done.astype(np.uint8))
    tol = 1e-4 if mode == "f32" else 3e-2
    vtol = tol * (1.0 if CB == 1 else max(1.0, float(np.abs(V).max())))
    np.testing.assert_allclose(vals.cpu().numpy(), V, rtol=tol, atol=vtol)
    np.testing.assert_allclose(hd.float().cpu().numpy(), h2, rtol=tol, atol=tol)
    np.testing.assert_allclose(cd.float().cpu().numpy(), c2, rtol=tol, atol=tol)
    gum = onat.gumbel_table(5, 6, 107, 3, N, 26)
    noisy = logits.astype(np.float32) + gum
    exp_acts, _ = ref.sample_actions(logits.astype(np.float32), BUCKETS, gum)
    got = acts.cpu().numpy()
    off = 0
    for g, nb in enumerate(BUCKETS):
        srt = np.sort(noisy[:, off:off + nb], axis=-1)
        clear = (srt[:, -1] - srt[:, -2]) > 1e-3
        assert np.array_equal(got[clear, g], exp_acts[clear, g]), f"group {g}"
        off += nb
    elogp, _ = ref.action_stats(logits, BUCKETS, got)
    np.testing.assert_allclose(logp.cpu().numpy(), elogp, rtol=tol, atol=tol)
    # bootstrap critic: same values, carry cleared but not advanced
    post2, _ = _post(gpu, N, done, rng)
    v2 = torch.zeros(N, dtype=torch.float32, device=gpu)
    ps.critic_only(o, v2, post=post2, carry=_carry(hd2, cd2, commit=0))
    torch.cuda.synchronize()
    assert torch.equal(v2, vals)
    assert np.array_equal(hd2.float().cpu().numpy(), hin.astype(np.float32))
    assert np.array_equal(cd2.float().cpu().numpy(), cin.astype(np.float32))


def _random_store(rng, T, N, D, H, C, ps, mode):
    obs = ref.rnd(rng.standard_normal((T, N, D)), mode).astype(np.float32)
    acts = np.stack([rng.integers(0, b, T * N) for b in BUCKETS], -1).astype(np.int32)
    lp = (rng.standard_normal((T * N, 6)) * 0.3 - 1.6).astype(np.float32)
    V = rng.standard_normal((T, N)).astype(np.float32)
    return {
        "obs": obs,
        "actions": acts.reshape(T, N, 6),
        "log_probs": lp.reshape(T, N, 6),
        "values": V,
        "advantages": (rng.standard_normal((T, N)) * 2 + 0.3).astype(np.float32),
        "returns": (V + rng.standard_normal((T, N))).astype(np.float32),
        "rewards": np.zeros((T, N), np.float32),
        "dones": (rng.random((T, N)) < 0.15).astype(np.uint8),
        "start_h": ref.rnd(rng.standard_normal((C, N, H)) * 0.5, mode).astype(np.float32),
        "start_c": ref.rnd(rng.standard_normal((C, N, H)) * 0.5, mode).astype(np.float32),
    }


def _device_store(gpu, st, dtype, C):
    from madrona_learn.rollouts import RolloutStore
    T, N, D = st["obs"].shape
    H = st["start_h"].shape[2]
    s = RolloutStore(T, N, D, 6, dtype, gpu, num_chunks=C, rnn_hidden=H)
    s.obs.copy_(torch.from_numpy(st["obs"]).to(dtype))
    for k in ("actions", "log_probs", "values", "advantages", "returns", "dones"):
        getattr(s, k).copy_(torch.from_numpy(st[k]))
    s.start_h.copy_(torch.from_numpy(st["start_h"]).to(dtype))
    s.start_c.copy_(torch.from_numpy(st["start_c"]).to(dtype))
    return s


HP = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
      "normalize_advantages": True}


def _hp(nat):
    hp = nat.PPOHparams()
    hp.clip_coef, hp.value_loss_coef = 0.2, 0.5
    for k in range(6):
        hp.entropy_coef[k] = 0.01
    hp.normalize_advantages, hp.loss_scale = 1, 1.0
    return hp


@pytest.mark.parametrize("mode,dtype,D,H,L,CB", [c + (1,) for c in CASES] + [
    ("f32", torch.float32, 64, 256, 2, 63), ("bf16", torch.bfloat16, 32, 64, 2, 63)])
@pytest.mark.parametrize("bptt", [32, 16])
def test_lstm_minibatch_grad(gpu, mode, dtype, D, H, L, CB, bptt):
    from madrona_learn import _native as nat
    ps = make_policy_state(gpu, D, H, L, dtype, seed=H + 1, critic_bins=CB)
    perturb(ps, 9, scale=0.2)
    T, N, mb = 32, 96, 64
    C = T // bptt
    rng = np.random.default_rng(12)
    st = _random_store(rng, T, N, D, H, C, ps, mode)
    if CB > 1:
        st["returns"] = (st["returns"] * 20.0).astype(np.float32)
    s = _device_store(gpu, st, dtype, C)
    seqs = rng.permutation(C * N)[:mb].astype(np.int32)
    batch = lref.gather_minibatch(st, seqs, bptt)
    adv = batch["advantages"].astype(np.float64)
    P = lref.unflatten(ps.params.cpu().numpy(), oracle_layout(ps))
    loss, G, met, _ = lref.ppo_loss_grads(P, batch, HP, BUCKETS, mode)
    gflat = lref.flatten(G, oracle_layout(ps))

    view = s.view(bptt)
    stats = torch.tensor([adv.mean(), 1.0 / np.sqrt(max(adv.var(), 1e-5))], dtype=torch.float32,
                         device=gpu)
    M = mb * bptt
    L_ = nat.lib()
    ws = torch.zeros(int(L_.mlearn_lstm_ppo_workspace_bytes(ps.desc, ps.lstm_desc, M, mb)),
                     dtype=torch.uint8, device=gpu)
    grad = torch.zeros(ps.layout["total"], dtype=torch.float32, device=gpu)
    out = torch.zeros(25, dtype=torch.float32, device=gpu)
    sq = torch.from_numpy(seqs).to(gpu)
    nat.check(L_.mlearn_lstm_ppo_minibatch_grad(
        ps.desc, ps.lstm_desc, view, nat.ptr(s.start_h), nat.ptr(s.start_c), nat.ptr(sq), mb,
        nat.ptr(stats), _hp(nat), nat.ptr(grad), nat.ptr(out), nat.ptr(ws),
        nat.stream_handle()), "lstm minibatch grad")
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    g = grad.cpu().numpy()
    scale = np.abs(gflat).max()
    if mode == "f32":
        np.testing.assert_allclose(o[0], loss, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(g, gflat, rtol=1e-3, atol=1e-4 * scale)
    else:
        np.testing.assert_allclose(o[0], loss, rtol=2e-2, atol=2e-3)
        err = np.abs(g - gflat).max() / scale
        assert err < 3e-2, err
    # every parameter segment on its own (a wrong LSTM block would hide in the global cosine)
    lay = oracle_layout(ps)
    for key in ("Wi", "Wr", "bl", "Wh"):
        off, shp = lay[key]
        n = int(np.prod(shp))
        a, b = g[off:off + n], gflat[off:off + n]
        cos = a @ b / (np.linalg.norm(a) * np.linalg.norm(b))
        assert cos > (0.99999 if mode == "f32" else 0.999), (key, cos)
    np.testing.assert_allclose(o[10], met["Value Loss"].mean(), rtol=2e-2 if mode == "bf16" else 1e-5)
    np.testing.assert_allclose(o[20], met["Entropy"].mean(), rtol=2e-2 if mode == "bf16" else 1e-5)
    assert o[14] == M and o[24] == M * 6


def test_lstm_optimizer_step_and_images(gpu):
    from madrona_learn.frag import from_image
    from madrona_learn.ppo import PPOHyperParams
    from madrona_learn.train_state import PolicyTrainState
    H = 128
    ps = make_policy_state(gpu, 64, H, 2, torch.float32, seed=4)
    perturb(ps, 5)
    hp = PPOHyperParams(lr=3e-4, gamma=0.99, gae_lambda=0.95, normalize_values=False,
                        value_normalizer_decay=0.0, max_advantage_est_decay=0.0, clip_coef=0.2,
                        value_loss_coef=0.5, entropy_coef=0.01, max_grad_norm=0.5)
    ts = PolicyTrainState(None, hp, ps, (1, 2))
    lay = oracle_layout(ps)
    init_norms = ps.init_norms.cpu().numpy().astype(np.float64)
    assert init_norms.size == 2 + 8
    P0 = lref.unflatten(ps.params.cpu().numpy(), lay)
    np.testing.assert_allclose(init_norms, lref.kernel_norms(P0), rtol=1e-6)
    rng = np.random.default_rng(6)
    p = ps.params.cpu().numpy().astype(np.float64)
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    for step in range(3):
        g = (rng.standard_normal(p.size) * (0.01 if step != 1 else 1.0)).astype(np.float32)
        ts.grads.copy_(torch.from_numpy(g))
        ts.optimizer_step(ps)
        p, m, v, _ = lref.optimizer_step(p, g.astype(np.float64), m, v, step, lay, init_norms,
                                         3e-4, 0.5)
    torch.cuda.synchronize()
    got = ps.params.cpu().numpy()
    np.testing.assert_allclose(got, p, rtol=2e-5, atol=2e-6)
    assert int(ts.step.item()) == 3
    # operand images follow the master LSTM weights
    wi, wr = ps.view("wi"), ps.view("wr")
    u = np.arange(H)
    nu = torch.from_numpy(np.concatenate([(u // 32) * 128 + g * 32 + u % 32 for g in range(4)]))
    cols = torch.arange(4 * H)
    for img, W, perm in ((ps.lstm_wi_perm, wi, True), (ps.lstm_wi_nat, wi, False),
                         (ps.lstm_wh_nat, wr, False)):
        logical = from_image(img, 4 * H, H, perm)
        assert torch.equal(logical[nu.to(gpu)], W.t()[cols.to(gpu)])
    wb = from_image(ps.lstm_w_bwd, 2 * H, 4 * H, False)
    assert torch.equal(wb, torch.cat([wi, wr], 0))
    hw = ps.view("hw")
    assert torch.equal(from_image(ps.head_t_nat, 32, H, False)[:hw.shape[1]], hw.t())


def make_cfg(dtype, N=64, T=32, chunks=1, mb=32, epochs=2, seed=5, critic_bins=1):
    import madrona_learn as ml
    return ml.TrainConfig(
        num_worlds=N, num_agents_per_world=1, num_updates=1,
        actions={"actions": ml.DiscreteActionsConfig(BUCKETS)}, steps_per_update=T,
        lr=3e-4, algo=ml.PPOConfig(num_epochs=epochs, minibatch_size=mb, clip_coef=0.2,
                                   value_loss_coef=0.5, entropy_coef={"actions": 0.01},
                                   max_grad_norm=0.5),
        num_bptt_chunks=chunks, gamma=0.99, gae_lambda=0.95, seed=seed, metrics_buffer_size=4,
        dreamer_v3_critic=critic_bins > 1, compute_dtype=dtype)


def _setup(gpu, dtype, N=64, H=64, D=64, chunks=1, mb=32, use_graph=False, critic_bins=1):
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    env = DummyVecEnv(N, D, 6, seed=2, device=gpu)
    cfg = make_cfg(dtype, N=N, chunks=chunks, mb=mb, critic_bins=critic_bins)
    pol = ml.Policy(actor_critic=make_actor_critic(H, 2, dtype, critic_bins),
                    obs_preprocess=ml.ObservationsCaster.create(dtype))
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), pol, use_graph=use_graph)
    return cfg, env, mgr


@pytest.mark.parametrize("mode,dtype,chunks,CB", [("f32", torch.float32, 1, 1),
                                                  ("f32", torch.float32, 2, 1),
                                                  ("bf16", torch.bfloat16, 2, 1),
                                                  ("f32", torch.float32, 2, 63)])
def test_lstm_full_update_matches_oracle(gpu, mode, dtype, chunks, CB):
    cfg, env, mgr = _setup(gpu, dtype, chunks=chunks, critic_bins=CB)
    ps, ts = mgr.state.policy_states, mgr.state.train_states
    lay = oracle_layout(ps)
    p0 = ps.params.cpu().numpy().astype(np.float64)
    T, N, H = cfg.steps_per_update, env.N, 64
    bptt = T // chunks
    oenv = onat.Env(env.N, env.D, env.k0, env.k1, 0)
    oenv.reset()
    mgr.update_iter()
    torch.cuda.synchronize()
    s = mgr.rollout_mgr.store
    g_acts = s.actions.cpu().numpy()
    z = np.zeros((N, H))
    ro, (hT, cT), _ = lref.rollout(p0, lay, oenv, T, bptt, BUCKETS, mgr.rollout.prng_key, 0,
                                   (z, z), mode=mode, gamma=cfg.gamma, actions_override=g_acts)
    assert np.array_equal(s.obs.float().cpu().numpy(), ro["obs"])
    assert np.array_equal(s.rewards.cpu().numpy(), ro["rewards"])
    assert np.array_equal(s.dones.cpu().numpy(), ro["dones"])
    assert ro["dones"].any()
    tol = 1e-4 if mode == "f32" else 3e-2
    np.testing.assert_allclose(s.values.cpu().numpy(), ro["values"], rtol=tol, atol=tol)
    np.testing.assert_allclose(s.bootstrap.cpu().numpy(), ro["bootstrap"], rtol=tol, atol=tol)
    np.testing.assert_allclose(s.log_probs.cpu().numpy(), ro["log_probs"], rtol=tol, atol=tol)
    np.testing.assert_allclose(s.start_h.float().cpu().numpy(), ro["start_h"], rtol=tol, atol=tol)
    np.testing.assert_allclose(s.start_c.float().cpu().numpy(), ro["start_c"], rtol=tol, atol=tol)
    c_states, h_states = mgr.rollout.rnn_states
    np.testing.assert_allclose(h_states[0].float().cpu().numpy(), hT, rtol=tol, atol=tol)
    np.testing.assert_allclose(c_states[0].float().cpu().numpy(), cT, rtol=tol, atol=tol)
    # cleared carries are exact zeros at every chunk start after a done step
    if chunks > 1:
        d = s.dones.cpu().numpy()[bptt - 1].astype(bool)
        assert not s.start_h[1][torch.from_numpy(d).to(gpu)].any()
    adv, ret = ref.gae_f32(s.rewards.cpu().numpy(), s.values.cpu().numpy(),
                           s.dones.cpu().numpy(), s.bootstrap.cpu().numpy(), cfg.gamma,
                           cfg.gae_lambda)
    assert np.array_equal(s.advantages.cpu().numpy(), adv)
    # PPO epochs on the GPU's store (incl. its start states) from the same parameters
    store = {k: v.float().cpu().numpy() if v.dtype == torch.bfloat16 else v.cpu().numpy()
             for k, v in s.as_dict().items()}
    store["start_h"] = s.start_h.float().cpu().numpy()
    store["start_c"] = s.start_c.float().cpu().numpy()
    zeros = np.zeros_like(p0)
    p1, _, _ = lref.ppo_update(
        p0, (zeros, zeros.copy(), 0), [store], HP, BUCKETS, lay,
        ps.init_norms.cpu().numpy().astype(np.float64), num_epochs=2, minibatch_size=32,
        bptt=bptt, key=ts.update_prng_key, epoch_base=0, mode=mode, lr=3e-4, max_grad_norm=0.5)
    got = ps.params.cpu().numpy()
    dr, dg = p1 - p0, got - p0
    cos = dg @ dr / (np.linalg.norm(dg) * np.linalg.norm(dr))
    if mode == "f32":
        np.testing.assert_allclose(got, p1, rtol=1e-4, atol=2e-5)
        assert cos > 0.999
    else:
        from tests.bf16_bound import check_bf16_update
        pf, _, _ = lref.ppo_update(
            p0, (zeros, zeros.copy(), 0), [store], HP, BUCKETS, lay,
            ps.init_norms.cpu().numpy().astype(np.float64), num_epochs=2, minibatch_size=32,
            bptt=bptt, key=ts.update_prng_key, epoch_base=0, mode="f32", lr=3e-4,
            max_grad_norm=0.5)
        check_bf16_update(f"lstm_C{chunks}_CB{CB}", got, p0, p1, pf, lay)
        assert cos > 0.99, cos
    assert int(ts.step.item()) == 2 * (N * chunks // 32)


def test_lstm_graph_replay_matches_eager(gpu):
    _, _, eager = _setup(gpu, torch.bfloat16, chunks=2, use_graph=False)
    _, _, graph = _setup(gpu, torch.bfloat16, chunks=2, use_graph=True)
    for _ in range(3):
        eager.update_iter()
        graph.update_iter()
    torch.cuda.synchronize()
    assert graph._segments is not None
    assert torch.equal(eager.state.policy_states.params, graph.state.policy_states.params)
    assert torch.equal(eager.rollout_mgr.store.actions, graph.rollout_mgr.store.actions)
    assert torch.equal(eager.rollout.rnn_states[1][0], graph.rollout.rnn_states[1][0])

