"""Population (PBT self-play split, config P of SURVEY §8(d)) on the GPU
path: TrainConfig.pbt with 2 train policies on one rank.  Policy p acts for
env columns [p*B, (p+1)*B) (pbt.py:130-133), has its own initial parameters,
optimizer state and minibatch RNG (train_state.py:439-488), and its PPO
update sees only its own columns (the vmap of algo_wrapper, train.py:165-174).
Checked against the oracle: the population rollout replayed on the oracle
env, then one oracle PPO update per policy on that policy's columns."""

import numpy as np
import pytest
import torch

from oracle import native as onat
from oracle import ppo_ref as ref

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]
N, D, H, T, P = 128, 64, 64, 32, 2


def _setup(gpu, dtype=torch.float32, use_graph=False, N=N, H=H, P=P, mb=16):
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from tests.test_gpu_train import make_policy
    env = DummyVecEnv(N, D, 6, seed=3, device=gpu)
    cfg = ml.TrainConfig(
        num_worlds=N, num_agents_per_world=1, num_updates=1,
        actions={"actions": ml.DiscreteActionsConfig(BUCKETS)}, steps_per_update=T,
        lr=3e-4, algo=ml.PPOConfig(num_epochs=2, minibatch_size=mb, clip_coef=0.2,
                                   value_loss_coef=0.5, entropy_coef={"actions": 0.01},
                                   max_grad_norm=0.5),
        num_bptt_chunks=1, gamma=0.99, gae_lambda=0.95, seed=9, metrics_buffer_size=4,
        dreamer_v3_critic=False, compute_dtype=dtype,
        pbt=ml.PBTConfig(num_teams=1, team_size=1, num_train_policies=P, num_past_policies=0,
                         self_play_portion=1.0, cross_play_portion=0.0, past_play_portion=0.0))
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), make_policy(dtype, H), use_graph=use_graph)
    return cfg, env, mgr


@pytest.mark.parametrize("mode,dtype,Np,Hp,Pp,mb", [
    ("f32", torch.float32, 128, 64, 2, 16),
    # config P's population shape: 8 policies, MLP[256,256], bf16 (128 envs each)
    ("bf16", torch.bfloat16, 1024, 256, 8, 32)])
def test_population_update_matches_oracle(gpu, mode, dtype, Np, Hp, Pp, mb):
    N, H, P = Np, Hp, Pp
    cfg, env, mgr = _setup(gpu, dtype, N=N, H=H, P=P, mb=mb)
    pss, tss = mgr.state.policy_list, mgr.state.train_list
    assert len(pss) == P and mgr.rollout_mgr.B == N // P
    p0 = [ps.params.cpu().numpy().astype(np.float64) for ps in pss]
    assert not np.array_equal(p0[0], p0[1]), "population members must init independently"
    assert tss[0].update_prng_key != tss[1].update_prng_key
    oenv = onat.Env(env.N, env.D, env.k0, env.k1, 0)
    oenv.reset()
    mgr.update_iter()
    torch.cuda.synchronize()
    s = mgr.rollout_mgr.store
    lay = ref.param_layout(D, H, 2, 26)
    ro, _ = ref.rollout(p0, lay, oenv, T, BUCKETS, mgr.rollout.prng_key, 0, mode=mode,
                        gamma=cfg.gamma, actions_override=s.actions.cpu().numpy())
    assert np.array_equal(s.rewards.cpu().numpy(), ro["rewards"])
    assert np.array_equal(s.dones.cpu().numpy(), ro["dones"])
    tol = 1e-4 if mode == "f32" else 3e-2
    np.testing.assert_allclose(s.values.cpu().numpy(), ro["values"], rtol=tol, atol=tol)
    np.testing.assert_allclose(s.bootstrap.cpu().numpy(), ro["bootstrap"], rtol=tol,
                               atol=tol)
    np.testing.assert_allclose(s.log_probs.cpu().numpy(), ro["log_probs"], rtol=tol, atol=tol)
    adv, ret = ref.gae_f32(s.rewards.cpu().numpy(), s.values.cpu().numpy(),
                           s.dones.cpu().numpy(), s.bootstrap.cpu().numpy(), cfg.gamma,
                           cfg.gae_lambda)
    assert np.array_equal(s.advantages.cpu().numpy(), adv)
    full = {k: (v.float() if v.dtype == torch.bfloat16 else v).cpu().numpy()
            for k, v in s.as_dict().items()}
    B = N // P
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
          "normalize_advantages": True}
    for p in range(P):
        c = slice(p * B, (p + 1) * B)
        store = {k: (v[:, c] if v.ndim >= 2 else v[c]) for k, v in full.items()}
        z = np.zeros_like(p0[p])
        p1, _, _ = ref.ppo_update(
            p0[p], (z, z.copy(), 0), [store], hp, BUCKETS, lay,
            pss[p].init_norms.cpu().numpy().astype(np.float64), num_epochs=2,
            minibatch_size=mb, bptt=T, key=tss[p].update_prng_key, epoch_base=0, mode=mode,
            lr=3e-4, max_grad_norm=0.5)
        got = pss[p].params.cpu().numpy()
        if mode == "f32":
            np.testing.assert_allclose(got, p1, rtol=1e-4, atol=2e-5)
        else:
            from tests.bf16_bound import check_bf16_update
            pf, _, _ = ref.ppo_update(
                p0[p], (z, z.copy(), 0), [store], hp, BUCKETS, lay,
                pss[p].init_norms.cpu().numpy().astype(np.float64), num_epochs=2,
                minibatch_size=mb, bptt=T, key=tss[p].update_prng_key, epoch_base=0,
                mode="f32", lr=3e-4, max_grad_norm=0.5)
            check_bf16_update(f"pbt_N{N}_H{H}_P{P}_p{p}", got, p0[p], p1, pf, lay)
            dg, dr = got - p0[p], p1 - p0[p]
            cos = dg @ dr / (np.linalg.norm(dg) * np.linalg.norm(dr))
            assert cos > 0.99, (p, cos)
        assert int(tss[p].step.item()) == 2 * (B // mb)
        # per-policy rollout metrics cover that policy's columns only
        last = mgr.metrics.last(policy=p)
        np.testing.assert_allclose(last["Rewards"].mean, store["rewards"].mean(), rtol=1e-5)
        assert last["Advantages"].count == T * B


def test_population_graph_replay_matches_eager(gpu):
    _, _, eager = _setup(gpu, torch.bfloat16, use_graph=False)
    _, _, graph = _setup(gpu, torch.bfloat16, use_graph=True)
    for _ in range(3):
        eager.update_iter()
        graph.update_iter()
    torch.cuda.synchronize()
    assert graph._segments is not None
    for a, b in zip(eager.state.policy_list, graph.state.policy_list):
        assert torch.equal(a.params, b.params)


def test_cull_update_gpu(gpu):
    """pbt_cull_update on a 4-policy population on one GPU: plan and
    hyperparameter draws as the oracle's, the culled policies hold their
    sources' state (weights, optimizer, fitness) and rebuilt compute images,
    keep their own minibatch RNG key, and training continues."""
    import dataclasses
    import madrona_learn as ml
    from madrona_learn import pbt
    from oracle import pbt_ref as oref
    cfg, env, mgr = _setup(gpu, torch.float32, N=256, H=64, P=4, mb=16)
    lr_kw = dict(base=3e-4, min_scale=0.1, max_scale=10.0, log10_scale=True)
    cfg = dataclasses.replace(cfg, lr=ml.ParamExplore(**lr_kw))
    # the initial draw (train.py:320-351), redone on this cfg
    mgr.state.pbt_rng = pbt.new_pbt_rng(cfg.seed)
    pbt.sample_initial_hyperparams(cfg, mgr.state)
    k0, k1 = (int(x) for x in mgr.state.pbt_rng[:2])
    for p, ts in enumerate(mgr.state.train_list):
        ur, up = oref.draws(k0, k1, 0, p, 0)
        assert np.float32(ts.hyper_params.lr) == oref.explore_param(ur, up, 3e-4, lr_kw, 1.0)
    mgr.update_iter()
    torch.cuda.synchronize()
    pss, tss = mgr.state.policy_list, mgr.state.train_list
    fit = [(0.0, 1.0, 40), (-3.0, 1.0, 40), (3.0, 1.0, 40), (0.5, 1.0, 2)]
    for ps, (m, v, n) in zip(pss, fit):
        ps.episode_score.mean.fill_(m)
        ps.episode_score.var.fill_(v)
        ps.episode_score.N.fill_(n)
    before = [(ps.params.clone(), ts.adam_m.clone(), int(ts.step.item()), ts.update_prng_key,
               ts.hyper_params.lr) for ps, ts in zip(pss, tss)]
    mean = np.array([f[0] for f in fit], np.float32)
    var = np.array([f[1] for f in fit], np.float32)
    N = np.array([f[2] for f in fit], np.float64)
    _, plan = pbt.pbt_cull_update(cfg, mgr.state, 2)
    assert plan == oref.cull_plan(mean, var, N, 4, 2)
    obs = torch.randn((64, D), device=gpu)
    for i, (dst, src, ok) in enumerate(plan):
        if not ok:
            assert torch.equal(pss[dst].params, before[dst][0])
            continue
        assert torch.equal(pss[dst].params, before[src][0])
        assert torch.equal(tss[dst].adam_m, before[src][1])
        assert int(tss[dst].step.item()) == before[src][2]
        assert tss[dst].update_prng_key == before[dst][3]
        assert float(pss[dst].episode_score.mean) == fit[src][0]
        ur, up = oref.draws(k0, k1, 1, i, 0)
        assert np.float32(tss[dst].hyper_params.lr) == \
            oref.explore_param(ur, up, before[src][4], lr_kw, 0.2)
        outs = []
        for q in (dst, src):  # same weights -> same rollout outputs (images rebuilt)
            a = torch.empty((64, 6), dtype=torch.int32, device=gpu)
            lp = torch.empty((64, 6), device=gpu)
            v = torch.empty(64, device=gpu)
            pss[q].rollout_step(obs, None, a, lp, v, (1, 2), None, 0)
            outs.append((a, lp, v))
        assert all(torch.equal(x, y) for x, y in zip(*outs))
    assert any(ok for _, _, ok in plan)
    mgr.update_iter()
    torch.cuda.synchronize()
    assert all(torch.isfinite(ps.params).all() for ps in pss)


def test_past_update_gpu(gpu, tmp_path):
    """TrainConfig.pbt with past policies (snapshots, no past play): the
    past slots start as copies of train policy j mod P, pbt_past_update
    follows the oracle's plan and copies the source's policy state into the
    least fit slot, and the past slots survive a checkpoint round trip."""
    import dataclasses
    import madrona_learn as ml
    from madrona_learn import pbt
    from madrona_learn.envs import DummyVecEnv
    from oracle import pbt_ref as oref
    from tests.test_gpu_train import make_policy
    env = DummyVecEnv(128, D, 6, seed=3, device=gpu)
    cfg, _, _ = _setup(gpu, torch.float32, N=128, H=64, P=2, mb=16)
    cfg = dataclasses.replace(cfg, pbt=dataclasses.replace(cfg.pbt, num_past_policies=3))
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), make_policy(torch.float32, 64),
                           use_graph=False)
    pss, past = mgr.state.policy_list, mgr.state.past_list
    assert [p.policy_id for p in past] == [2, 3, 4]
    for j, p in enumerate(past):
        assert torch.equal(p.params, pss[oref.initial_past_sources(2, 3)[j]].params)
    mgr.update_iter()
    torch.cuda.synchronize()
    fit = [(1.0, 1.0, 40), (4.0, 1.0, 40), (0.0, 1.0, 30), (-6.0, 1.0, 30), (0.0, 1.0, 30)]
    for e, (m, v, n) in zip([p.episode_score for p in pss + past], fit):
        e.mean.fill_(m)
        e.var.fill_(v)
        e.N.fill_(n)
    op = int(mgr.state.pbt_rng[2])
    k0, k1 = (int(x) for x in mgr.state.pbt_rng[:2])
    before = [p.params.clone() for p in pss]
    pbt.pbt_past_update(cfg, mgr.state)
    want = oref.past_update_plan(k0, k1, op, np.array([f[0] for f in fit], np.float32),
                                 np.array([f[1] for f in fit], np.float32),
                                 np.array([f[2] for f in fit], np.float64), 2, 3)
    assert mgr.state.last_past_update == want
    src, dst, ok = want
    assert dst == 3 and ok
    assert torch.equal(past[1].params, before[src])
    assert float(past[1].episode_score.mean) == fit[src][0]
    # checkpoint round trip of the past slots
    mgr.save_ckpt(str(tmp_path))
    saved = [p.params.clone() for p in past]
    for p in past:
        p.params.zero_()
    mgr.load_ckpt(str(tmp_path))
    assert all(torch.equal(a.params, b) for a, b in zip(mgr.state.past_list, saved))
