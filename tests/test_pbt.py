"""Population ops on the host (CPU): hyperparameter exploration with the
Philox RNG contract, the fitness EMA and the cull plan against the oracle
restatement (oracle/pbt_ref.py, pbt.py:382-722), and the cross-rank policy
copy of pbt_cull_update over gloo (world 2, one policy per rank)."""

import dataclasses
import os
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import pbt_ref as oref


def _pe(**kw):
    import madrona_learn as ml
    return ml.ParamExplore(**kw)


EXPLORES = [
    dict(base=3e-4, min_scale=0.1, max_scale=10.0, log10_scale=True),
    dict(base=0.01, min_scale=0.5, max_scale=2.0, ln_scale=True),
    dict(base=0.5, min_scale=0.5, max_scale=1.5),
    dict(base=0.5, min_scale=0.9, max_scale=1.1, clip_perturb=True, perturb_rnd_min=0.5,
         perturb_rnd_max=1.5),
]


@pytest.mark.parametrize("chance", [0.0, 0.2, 1.0])
@pytest.mark.parametrize("e", range(len(EXPLORES)))
def test_explore_param_matches_oracle(chance, e):
    from madrona_learn import pbt
    kw = EXPLORES[e]
    pe = _pe(**kw)
    for op in range(4):
        for slot in range(3):
            ur, up = pbt._draws((0x1234, 0x5678), op, slot, 0)
            our, oup = oref.draws(0x1234, 0x5678, op, slot, 0)
            assert (ur, up) == (our, oup)
            got = pbt.explore_param(ur, up, 0.37, pe, chance)
            want = oref.explore_param(our, oup, 0.37, kw, chance)
            assert np.float32(got) == np.float32(want)
            lo, hi = np.float32(kw["base"] * kw["min_scale"]), np.float32(kw["base"] * kw["max_scale"])
            if chance == 1.0 or kw.get("clip_perturb"):
                assert lo * 0.999 <= got <= hi * 1.001


def test_explore_hyperparams_streams():
    """lr, entropy and reward hyperparameters use their own streams."""
    import madrona_learn as ml
    from madrona_learn import pbt
    from madrona_learn.ppo import PPOHyperParams
    lr_pe, ec_pe = _pe(**EXPLORES[0]), _pe(**EXPLORES[2])
    cfg = types.SimpleNamespace(lr=lr_pe, algo=types.SimpleNamespace(entropy_coef=ec_pe),
                                pbt=types.SimpleNamespace(reward_hyper_params_explore={
                                    "a": _pe(**EXPLORES[1]), "b": _pe(**EXPLORES[3])}))
    ts = types.SimpleNamespace(hyper_params=PPOHyperParams(
        lr=3e-4, gamma=0.99, gae_lambda=0.95, normalize_values=False, value_normalizer_decay=0.99,
        max_advantage_est_decay=0.99, entropy_coef=0.5))
    ps = types.SimpleNamespace(reward_hyper_params=torch.tensor([0.01, 0.5]))
    pbt.pbt_explore_hyperparams(cfg, (7, 9, 3, 5), ps, ts, 0.2)
    want = oref.explore_hyperparams((7, 9), 3, 5, {"lr": 3e-4, "entropy_coef": 0.5,
                                                   "reward": [0.01, 0.5]},
                                    {"lr": EXPLORES[0], "entropy_coef": EXPLORES[2],
                                     "reward": [EXPLORES[1], EXPLORES[3]]}, 0.2)
    assert np.float32(ts.hyper_params.lr) == np.float32(want["lr"])
    assert np.float32(ts.hyper_params.entropy_coef) == np.float32(want["entropy_coef"])
    assert np.array_equal(ps.reward_hyper_params.numpy(), np.array(want["reward"], np.float32))


def test_fitness_ema_matches_oracle():
    from madrona_learn import pbt
    rng = np.random.default_rng(0)
    N, B = 96, 32
    scores = [pbt.MovingEpisodeScore("cpu") for _ in range(3)]
    state = [(np.float32(0), np.float32(0), 0) for _ in range(3)]
    for step in range(20):
        res = torch.from_numpy(rng.standard_normal(N).astype(np.float32))
        dn = torch.from_numpy(rng.random(N) < (0.0 if step == 3 else 0.15))
        pbt.pbt_update_fitness([(scores[p], p * B, B) for p in range(3)], res, dn)
        for p in range(3):
            sl = slice(p * B, (p + 1) * B)
            state[p] = oref.update_fitness(*state[p], res.numpy()[sl], dn.numpy()[sl])
    for p in range(3):
        np.testing.assert_allclose(scores[p].mean.item(), state[p][0], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(scores[p].var.item(), state[p][1], rtol=1e-4, atol=1e-7)
        assert scores[p].N.item() == state[p][2]


@pytest.mark.parametrize("team", [2, 4])
@pytest.mark.parametrize("per_agent", [False, True])
def test_fitness_counts_agent_zero_of_each_match(team, per_agent):
    """pbt.py:390-396: dones reshaped to [matches, team_size] and only agent 0
    of a match counts; episode scores are per match (or per agent, agent 0
    taken).  A match ending counts once, not team_size times."""
    from madrona_learn import pbt
    rng = np.random.default_rng(7)
    M, P = 48, 2                      # matches, policies (contiguous self-play split)
    N, Bm = M * team, M // P          # agents, matches per policy
    scores = [pbt.MovingEpisodeScore("cpu") for _ in range(P)]
    state = [(np.float32(0), np.float32(0), 0) for _ in range(P)]
    for step in range(12):
        match_done = rng.random(M) < 0.3
        dn = np.repeat(match_done, team)           # every agent of a match ends together
        dn[1::team] = rng.random(M) < 0.5          # other agents' flags must not matter
        dn[::team] = match_done
        res = rng.standard_normal(M).astype(np.float32)
        x = np.repeat(res, team) if per_agent else res
        pbt.pbt_update_fitness([(scores[p], p * Bm * team, Bm * team) for p in range(P)],
                               torch.from_numpy(x), torch.from_numpy(dn), team_size=team)
        for p in range(P):
            sl = slice(p * Bm, (p + 1) * Bm)
            state[p] = oref.update_fitness(*state[p], res[sl], match_done[sl])
    for p in range(P):
        np.testing.assert_allclose(scores[p].mean.item(), state[p][0], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(scores[p].var.item(), state[p][1], rtol=1e-4, atol=1e-7)
        assert scores[p].N.item() == state[p][2]


def test_check_overwrite_zero_variance():
    """Both variances 0 with N > 0 and different means: t = +/-inf, the
    reference's p = 1 - cdf(t) is 0 (overwrite) or 1 (keep); N = 0 gives
    NaN (never overwrite)."""
    from madrona_learn import pbt
    cases = [([1.0, 2.0], [0.0, 0.0], [5, 7]), ([2.0, 1.0], [0.0, 0.0], [5, 7]),
             ([1.0, 1.0], [0.0, 0.0], [5, 7]), ([1.0, 2.0], [0.0, 0.0], [0, 7]),
             ([1.0, 2.0], [0.5, 0.0], [3, 0]), ([-1.0, 3.0], [0.0, 1e-3], [4, 9])]
    for mean, var, N in cases:
        m, v, n = (np.asarray(a, np.float32) for a in (mean, var, N))
        with np.errstate(divide="ignore", invalid="ignore"):
            want = oref.check_overwrite(m, v, n, 1, 0)
        assert pbt.check_overwrite(None, m, v, n, 1, 0) == want, (mean, var, N)
    # the zero-variance case the fix is about: source better -> overwrite
    assert pbt.check_overwrite(None, np.float32([1, 2]), np.float32([0, 0]), np.float32([5, 7]),
                               1, 0)


def test_checkpoint_file_per_rank(tmp_path):
    """Multi-rank jobs write <update>.r<rank>.pt and each rank restores its own
    latest file; a one-rank job keeps <update>.pt."""
    from madrona_learn.train import _ckpt_file, _ckpt_name
    assert _ckpt_name(7) == "7.pt" and _ckpt_name(7, 1, 2) == "7.r1.pt"
    for name in ("3.pt", "9.pt", "3.r0.pt", "3.r1.pt", "12.r0.pt", "5.r1.pt"):
        (tmp_path / name).write_bytes(b"")
    assert _ckpt_file(str(tmp_path)).endswith("9.pt")
    assert _ckpt_file(str(tmp_path), 0, 2).endswith("12.r0.pt")
    assert _ckpt_file(str(tmp_path), 1, 2).endswith("5.r1.pt")
    with pytest.raises(FileNotFoundError):
        _ckpt_file(str(tmp_path), 2, 4)
    f = str(tmp_path / "5.r1.pt")
    assert _ckpt_file(f, 0, 2) == f


def test_cull_plan_matches_oracle():
    from madrona_learn import pbt
    rng = np.random.default_rng(1)
    for trial in range(50):
        P = 8
        mean = rng.standard_normal(P).astype(np.float32) * (0.1 if trial % 2 else 2.0)
        var = rng.random(P).astype(np.float32) + 0.1
        N = rng.integers(0 if trial % 5 == 0 else 1, 40, P).astype(np.float64)
        for k in (1, 2, 4):
            with np.errstate(divide="ignore", invalid="ignore"):
                got = pbt.cull_plan(None, mean, var, N, P, k)
            assert got == oref.cull_plan(mean, var, N, P, k)


# ---------------------------------------------------------------------------
# cross-rank copy (gloo, world 2: one policy per rank, config P's placement)
# ---------------------------------------------------------------------------
def _fake_member(pid, seed):
    from madrona_learn import pbt
    from madrona_learn.ppo import PPOHyperParams
    g = torch.Generator().manual_seed(seed)
    ps = types.SimpleNamespace(params=torch.randn(1000, generator=g), obs_est=None,
                               episode_score=pbt.MovingEpisodeScore("cpu"), synced=0)
    ps.sync_weights = lambda: setattr(ps, "synced", ps.synced + 1)
    ts = types.SimpleNamespace(
        adam_m=torch.randn(1000, generator=g), adam_v=torch.rand(1000, generator=g),
        step=torch.tensor([pid + 3], dtype=torch.int32), value_norm_est=None, policy_id=pid,
        update_prng_key=(100 + pid, 200 + pid),
        hyper_params=PPOHyperParams(lr=1e-3 * (pid + 1), gamma=0.99, gae_lambda=0.95,
                                    normalize_values=False, value_normalizer_decay=0.99,
                                    max_advantage_est_decay=0.99, entropy_coef=0.01))
    return ps, ts


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from madrona_learn import pbt
        ps, ts = _fake_member(rank, 10 + rank)
        # policy 1 is far better with many episodes: the one-sided test passes
        ps.episode_score.mean.fill_(5.0 if rank == 1 else -5.0)
        ps.episode_score.var.fill_(1.0)
        ps.episode_score.N.fill_(50)
        tsm = types.SimpleNamespace(policy_list=[ps], train_list=[ts],
                                    pbt_rng=torch.tensor([1, 2, 0], dtype=torch.int64))
        lr_pe = _pe(**EXPLORES[0])
        cfg = types.SimpleNamespace(
            lr=lr_pe, algo=types.SimpleNamespace(entropy_coef=0.01),
            pbt=types.SimpleNamespace(num_train_policies=2, num_past_policies=0,
                                      reward_hyper_params_explore={}))
        _, plan = pbt.pbt_cull_update(cfg, tsm, 1)
        q.put((rank, plan, ps.params.clone(), ts.adam_m.clone(), int(ts.step.item()),
               ts.update_prng_key, ts.hyper_params.lr, ps.synced, float(ps.episode_score.mean)))
    finally:
        dist.destroy_process_group()


def test_cull_copies_across_ranks_gloo():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    src_ps, src_ts = _fake_member(1, 11)
    plan0, params0, m0, step0, key0, lr0, synced0, mean0 = res[0]
    plan1, params1, m1, step1, key1, lr1, synced1, mean1 = res[1]
    assert plan0 == plan1 == [(0, 1, True)]
    assert torch.equal(params0, src_ps.params) and torch.equal(params1, src_ps.params)
    assert torch.equal(m0, src_ts.adam_m) and step0 == 4 and mean0 == 5.0
    assert key0 == (100, 200), "the culled policy keeps its own minibatch RNG key"
    assert synced0 == 1 and synced1 == 0
    ur, up = oref.draws(1, 2, 0, 0, 0)
    want = oref.explore_param(ur, up, src_ts.hyper_params.lr, EXPLORES[0], 0.2)
    assert np.float32(lr0) == np.float32(want) and lr1 == src_ts.hyper_params.lr


# ---------------------------------------------------------------------------
# past-policy snapshots (pbt_past_update, pbt.py:684-722)
# ---------------------------------------------------------------------------
def test_past_update_plan_matches_oracle():
    from madrona_learn import pbt
    rng = np.random.default_rng(7)
    for trial in range(60):
        P, Q = int(rng.integers(1, 6)), int(rng.integers(1, 5))
        mean = rng.standard_normal(P + Q).astype(np.float32)
        if trial % 3 == 0:
            mean[P:] = mean[P]  # ties: jnp.argmin takes the first minimum
        var = (rng.random(P + Q).astype(np.float32) + 0.1) * (0 if trial % 7 == 0 else 1)
        N = rng.integers(0 if trial % 5 == 0 else 1, 40, P + Q).astype(np.float64)
        got = pbt.past_update_plan((0x1234 + trial, 0x5678), trial, mean, var, N, P, Q)
        want = oref.past_update_plan(0x1234 + trial, 0x5678, trial, mean, var, N, P, Q)
        assert got == want
        assert 0 <= got[0] < P and P <= got[1] < P + Q
    assert oref.initial_past_sources(3, 5) == [0, 1, 2, 0, 1]


def _past_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from madrona_learn import pbt
        ps, ts = _fake_member(rank, 10 + rank)
        ps.episode_score.mean.fill_(5.0 if rank == 1 else -5.0)
        ps.episode_score.var.fill_(1.0)
        ps.episode_score.N.fill_(50)
        tsm = types.SimpleNamespace(policy_list=[ps], train_list=[ts],
                                    pbt_rng=torch.tensor([3, 4, 0], dtype=torch.int64))
        cfg = types.SimpleNamespace(pbt=types.SimpleNamespace(num_train_policies=2,
                                                              num_past_policies=3))
        pbt.init_past_policies(cfg, tsm)
        init = [p.params.clone() for p in tsm.past_list]
        # past slot fitness: slot 1 is the least fit and has data, so a train
        # policy with many good episodes overwrites it
        for j, p in enumerate(tsm.past_list):
            p.episode_score.mean.fill_([0.0, -9.0, 0.0][j])
            p.episode_score.var.fill_(1.0)
            p.episode_score.N.fill_(20)
        pbt.pbt_past_update(cfg, tsm)
        q.put((rank, init, tsm.last_past_update, [p.params.clone() for p in tsm.past_list],
               [float(p.episode_score.mean) for p in tsm.past_list], int(tsm.pbt_rng[2])))
    finally:
        dist.destroy_process_group()


def test_past_snapshots_across_ranks_gloo():
    """World 2, one train policy per rank: the past slots start as copies of
    train policy j mod P on every rank, and pbt_past_update broadcasts the
    chosen source's state into the least fit slot on both ranks."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_past_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    members = [_fake_member(r, 10 + r)[0] for r in range(2)]
    for r in range(2):
        init, plan, past, means, ctr = res[r]
        for j in range(3):
            assert torch.equal(init[j], members[j % 2].params)
        src, dst, ok = plan
        mean = np.array([-5.0, 5.0, 0.0, -9.0, 0.0], np.float32)
        want = oref.past_update_plan(3, 4, 0, mean, np.ones(5, np.float32),
                                     np.array([50, 50, 20, 20, 20.0]), 2, 3)
        assert (src, dst, ok) == want and dst == 3
        if ok:
            assert torch.equal(past[1], members[src].params)
            assert means[1] == [-5.0, 5.0][src]
        assert torch.equal(past[0], members[0].params) and torch.equal(past[2], members[0].params)
        assert ctr == 1
    assert res[0][1] == res[1][1]


def _pool_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from madrona_learn import pbt
        ps, ts = _fake_member(0, 10)  # one policy, held by both ranks (G = 2)
        ps.episode_score.mean.fill_([1.0, 4.0][rank])
        ps.episode_score.var.fill_([0.5, 2.0][rank])
        ps.episode_score.N.fill_([10, 30][rank])
        tsm = types.SimpleNamespace(policy_list=[ps], train_list=[ts])
        fit = pbt.gather_fitness(tsm, 1)
        # a past snapshot of the policy carries the pooled fitness too (so that
        # pbt_past_update compares pooled train and past statistics)
        cfg = types.SimpleNamespace(pbt=types.SimpleNamespace(num_train_policies=1,
                                                              num_past_policies=1))
        pbt.init_past_policies(cfg, tsm)
        e = tsm.past_list[0].episode_score
        q.put((rank, (fit, (float(e.mean), float(e.var), int(e.N)))))
    finally:
        dist.destroy_process_group()


def test_fitness_pooled_over_dp_holders_gloo():
    """A policy trained by 2 data-parallel ranks: its fitness pools both
    holders' episode statistics (each scores its own env shard)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_pool_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        (mean, var, N), past = res[r]
        assert past[2] == 40
        assert abs(past[0] - np.float32(mean[0])) == 0 and abs(past[1] - np.float32(var[0])) == 0
        assert N[0] == 40
        assert abs(mean[0] - (10 * 1.0 + 30 * 4.0) / 40) < 1e-12
        want_var = (10 * (0.5 + 1.0) + 30 * (2.0 + 16.0)) / 40 - mean[0] ** 2
        assert abs(var[0] - want_var) < 1e-12
