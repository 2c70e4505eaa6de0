"""BASELINE configurations at their production grid sizes against the oracle
(round-2 verdict: the L and P full updates had only been checked at toy
sizes).  bf16 throughout, MLP[256, 256]; the bf16 update is held to the
per-tensor bound of tests/bf16_bound.py (distance to the oracle's bf16 mode
within the oracle's own bf16-vs-f32 distance, per tensor).

  * L: RecurrentBackboneEncoder(MLP[256,256], LSTM(256)) over
    2048 envs with minibatches of 2048 sequences: every per-step scan launch
    of the update runs at its production grid ((2048 / 32) x (256 / 32)
    workgroups), one epoch (one 65,536-row minibatch: the oracle's BPTT
    costs ~15 s on the host).
  * L at its stated 8192 envs: oracle column windows of the whole-rollout
    launch and the whole first update (4 minibatches of 2048 sequences).
  * P at its stated size: 8 train policies x 8192 envs, the
    population rollout launch with tiles of several policies in series per
    workgroup (the parameter-restage branch), oracle windows of restaged
    tiles and one restaged policy's whole update (4 optimizer steps).
The rollout data are checked as in tests/test_gpu_train.py (obs / rewards /
dones / GAE bit-exact, values / log-probs within the bf16 tolerance)."""

import numpy as np
import pytest
import torch

from oracle import lstm_ref as lref
from oracle import native as onat
from oracle import ppo_ref as ref
from tests.bf16_bound import check_bf16_update

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]
HP = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
      "normalize_advantages": True}
D, H, T = 64, 256, 32


def _cfg(N, mb, epochs=1, pbt_policies=0, seed=5):
    import madrona_learn as ml
    pbt = None
    if pbt_policies:
        pbt = ml.PBTConfig(num_teams=1, team_size=1, num_train_policies=pbt_policies,
                           num_past_policies=0, self_play_portion=1.0, cross_play_portion=0.0,
                           past_play_portion=0.0)
    return ml.TrainConfig(
        num_worlds=N, num_agents_per_world=1, num_updates=1,
        actions={"actions": ml.DiscreteActionsConfig(BUCKETS)}, steps_per_update=T, lr=3e-4,
        algo=ml.PPOConfig(num_epochs=epochs, minibatch_size=mb, clip_coef=0.2,
                          value_loss_coef=0.5, entropy_coef={"actions": 0.01},
                          max_grad_norm=0.5),
        num_bptt_chunks=1, gamma=0.99, gae_lambda=0.95, seed=seed, metrics_buffer_size=4,
        dreamer_v3_critic=False, compute_dtype=torch.bfloat16, pbt=pbt)


def _check_store(s, ro, cols=slice(None), vsens=None):
    """vsens (two-hot critics): per-value sensitivity of mean() to the bf16
    rounding of the bin logits ([T + 1, n], bootstrap last): sum_j p_j
    |b_j - mean| ulp(l_j), the first-order change when every bin logit moves
    by one bf16 ulp.  With |b_j| up to symexp(14) = 1.2e6 one flipped ulp of
    an extreme bin's logit (the kernel and the oracle round the head's f32
    sums independently) moves mean() by thousands, so the value tolerance is
    that bound, not a fraction of the value."""
    assert np.array_equal(s.obs[:, cols].float().cpu().numpy(), ro["obs"])
    assert np.array_equal(s.rewards[:, cols].cpu().numpy(), ro["rewards"])
    assert np.array_equal(s.dones[:, cols].cpu().numpy(), ro["dones"])
    tol = 3e-2
    if vsens is None:
        np.testing.assert_allclose(s.values[:, cols].cpu().numpy(), ro["values"], rtol=tol,
                                   atol=tol)
        np.testing.assert_allclose(s.bootstrap[cols].cpu().numpy(), ro["bootstrap"], rtol=tol,
                                   atol=tol)
    else:
        got = np.concatenate([s.values[:, cols].cpu().numpy(), s.bootstrap[cols].cpu().numpy()[None]])
        want = np.concatenate([ro["values"], np.asarray(ro["bootstrap"])[None]])
        bad = np.abs(got - want) > vsens + tol * np.abs(want) + tol
        assert not bad.any(), (np.argwhere(bad)[:5], got[bad][:5], want[bad][:5], vsens[bad][:5])
    np.testing.assert_allclose(s.log_probs[:, cols].cpu().numpy(), ro["log_probs"], rtol=tol,
                               atol=tol)
    adv, _ = ref.gae_f32(s.rewards[:, cols].cpu().numpy(), s.values[:, cols].cpu().numpy(),
                         s.dones[:, cols].cpu().numpy(), s.bootstrap[cols].cpu().numpy(), 0.99,
                         0.95)
    assert np.array_equal(s.advantages[:, cols].cpu().numpy(), adv)


def test_lstm_update_production_grid(gpu):
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from tests.test_gpu_lstm import make_actor_critic
    N, mb = 2048, 2048
    env = DummyVecEnv(N, D, 6, seed=2, device=gpu)
    cfg = _cfg(N, mb)
    pol = ml.Policy(actor_critic=make_actor_critic(H, 2, torch.bfloat16),
                    obs_preprocess=ml.ObservationsCaster.create(torch.bfloat16))
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), pol, use_graph=False)
    ps, ts = mgr.state.policy_states, mgr.state.train_states
    a = ps.arch
    lay = lref.param_layout(a.obs_dim, a.hidden, a.num_layers, a.num_logits, a.critic_bins)
    p0 = ps.params.cpu().numpy().astype(np.float64)
    oenv = onat.Env(env.N, env.D, env.k0, env.k1, 0)
    oenv.reset()
    mgr.update_iter()
    torch.cuda.synchronize()
    s = mgr.rollout_mgr.store
    z = np.zeros((N, H))
    ro, _, _ = lref.rollout(p0, lay, oenv, T, T, BUCKETS, mgr.rollout.prng_key, 0, (z, z),
                            mode="bf16", gamma=cfg.gamma, actions_override=s.actions.cpu().numpy())
    _check_store(s, ro)
    store = {k: v.float().cpu().numpy() if v.dtype == torch.bfloat16 else v.cpu().numpy()
             for k, v in s.as_dict().items()}
    store["start_h"] = s.start_h.float().cpu().numpy()
    store["start_c"] = s.start_c.float().cpu().numpy()
    zeros = np.zeros_like(p0)
    upd = dict(num_epochs=1, minibatch_size=mb, bptt=T, key=ts.update_prng_key, epoch_base=0,
               lr=3e-4, max_grad_norm=0.5)
    norms = ps.init_norms.cpu().numpy().astype(np.float64)
    pb, _, _ = lref.ppo_update(p0, (zeros, zeros.copy(), 0), [store], HP, BUCKETS, lay, norms,
                               mode="bf16", **upd)
    pf, _, _ = lref.ppo_update(p0, (zeros, zeros.copy(), 0), [store], HP, BUCKETS, lay, norms,
                               mode="f32", **upd)
    got = ps.params.cpu().numpy()
    check_bf16_update("config_L_production", got, p0, pb, pf, lay)
    assert int(ts.step.item()) == 1


def _restage_tiles(grid, tpp, ntiles):
    """Tiles of the second and third rounds of the population launch whose
    workgroup's previous tile belonged to another policy (the restage branch
    of policy_rollout_pop_kernel): tile g runs on workgroup g % grid after
    tile g - grid."""
    out = []
    for k in (1, 2):
        for g in range(k * grid, min((k + 1) * grid, ntiles)):
            if (g - grid) // tpp != g // tpp:
                out.append(g)
                break
        for g in range(min((k + 1) * grid, ntiles) - 1, k * grid - 1, -1):
            if (g - grid) // tpp != g // tpp:
                out.append(g)
                break
    return sorted(set(out))


def _check_window(s, mgr, env, p0, lay, e0, cfg):
    """Replay the 32 envs [e0, e0 + 32) on the oracle env + policy."""
    c = slice(e0, e0 + 32)
    oenv = onat.Env(32, D, env.k0, env.k1, e0)
    oenv.reset()
    acts = s.actions[:, c].cpu().numpy()
    ro, _ = ref.rollout(p0, lay, oenv, T, BUCKETS, mgr.rollout.prng_key, 0, mode="bf16",
                        gamma=cfg.gamma, actions_override=acts)
    _check_store(s, ro, c)
    gum = np.stack([onat.gumbel_table(*mgr.rollout.prng_key, t, e0, 32, 26) for t in range(T)])
    noisy = ro["logits"] + gum
    off = 0
    for g, nb in enumerate(BUCKETS):
        sl = noisy[..., off:off + nb]
        srt = np.sort(sl, -1)
        clear = (srt[..., -1] - srt[..., -2]) > 1e-2
        assert np.array_equal(np.argmax(sl, -1)[clear], acts[..., g][clear]), (e0, g)
        off += nb


@pytest.mark.timeout(600)
def test_population_8x8192(gpu):
    """Config P at its stated size: 8 train policies x 8192 envs (65,536 envs)
    on one GPU, the population's rollouts as ONE launch
    (mlearn_policy_rollout_env_pop) whose 2048 env tiles outnumber the
    resident workgroups, so workgroups take tiles of several policies in
    series and restage the LayerNorm / head parameters on each move.  Env
    tiles of rounds 2 and 3 whose workgroup's previous tile belonged to
    another policy are replayed on the oracle with their own policy's
    parameters (obs / rewards / dones / GAE bit-exact, values / log-probs
    within the bf16 tolerance, sampled actions where the Gumbel margin is
    clear); then one restaged policy's whole update (4 minibatches) against
    the oracle under the per-tensor bf16 bound."""
    from madrona_learn import _native as nat
    from madrona_learn.envs import DummyVecEnv
    import madrona_learn as ml
    from tests.test_gpu_train import make_policy
    P, B, mb = 8, 8192, 2048
    N = P * B
    env = DummyVecEnv(N, D, 6, seed=3, device=gpu)
    cfg = _cfg(N, mb, pbt_policies=P, seed=9)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), make_policy(torch.bfloat16, H),
                           use_graph=False)
    pss, tss = mgr.state.policy_list, mgr.state.train_list
    rm = mgr.rollout_mgr
    assert rm.B == B and rm.P == P
    # the feature-split population kernel (the row split, the library's choice
    # here, has its own test below)
    assert nat.lib().mlearn_policy_rollout_pop_kernel(pss[0].desc, None, B, P, 0) == 2
    rm.rollout_kernel = 1
    tpp = B // 32
    grid = nat.lib().mlearn_policy_rollout_pop_workgroups(pss[0].desc, None, B, P, 0)
    assert 0 < grid < P * tpp, grid
    picks = _restage_tiles(grid, tpp, P * tpp)
    assert len(picks) >= 2, (grid, picks)
    p0s = [ps.params.cpu().numpy().astype(np.float64) for ps in pss]
    assert not np.array_equal(p0s[0], p0s[1])  # each policy its own initialisation
    mgr.update_iter()
    torch.cuda.synchronize()
    assert getattr(rm, "_pop_sig", None) is not None  # the population launch ran
    s = rm.store
    lay = ref.param_layout(D, H, 2, 26)
    for g in picks:
        p = g // tpp
        _check_window(s, mgr, env, p0s[p], lay, g * 32, cfg)
    # the whole update of the policy owning the first restaged tile
    q = picks[0] // tpp
    c = slice(q * B, (q + 1) * B)
    full = {k: (v.float() if v.dtype == torch.bfloat16 else v).cpu().numpy()
            for k, v in s.as_dict().items()}
    store = {k: (v[:, c] if v.ndim >= 2 else v[c]) for k, v in full.items()}
    adv, _ = ref.gae_f32(store["rewards"], store["values"], store["dones"],
                         s.bootstrap[c].cpu().numpy(), 0.99, 0.95)
    assert np.array_equal(store["advantages"], adv)
    z = np.zeros_like(p0s[q])
    upd = dict(num_epochs=1, minibatch_size=mb, bptt=T, key=tss[q].update_prng_key,
               epoch_base=0, lr=3e-4, max_grad_norm=0.5)
    norms = pss[q].init_norms.cpu().numpy().astype(np.float64)
    pb, _, _ = ref.ppo_update(p0s[q], (z, z.copy(), 0), [store], HP, BUCKETS, lay, norms,
                              mode="bf16", **upd)
    pf, _, _ = ref.ppo_update(p0s[q], (z, z.copy(), 0), [store], HP, BUCKETS, lay, norms,
                              mode="f32", **upd)
    check_bf16_update(f"config_P_8x8192_policy{q}", pss[q].params.cpu().numpy(), p0s[q], pb, pf,
                      lay)
    assert int(tss[q].step.item()) == B // mb
    last = mgr.metrics.last(policy=q)
    np.testing.assert_allclose(last["Rewards"].mean, store["rewards"].mean(), rtol=1e-5)


@pytest.mark.timeout(600)
def test_population_8x8192_row_split(gpu):
    """Config P on the row-split population kernel (the library's choice):
    8 policies x 512 16-env tiles dealt in rounds of 8 consecutive tiles per
    8-wave workgroup, one workgroup per CU, so every workgroup's second round
    belongs to another policy and restages its W1 / head / LayerNorm images.
    32-env windows of second-round tiles of several workgroups (and the last
    one) are replayed on the oracle with their own policy's parameters, as in
    the feature-split test above."""
    from madrona_learn import _native as nat
    from madrona_learn.envs import DummyVecEnv
    import madrona_learn as ml
    from tests.test_gpu_train import make_policy
    P, B, mb = 8, 8192, 2048
    N = P * B
    env = DummyVecEnv(N, D, 6, seed=4, device=gpu)
    cfg = _cfg(N, mb, pbt_policies=P, seed=10)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), make_policy(torch.bfloat16, H),
                           use_graph=False)
    pss = mgr.state.policy_list
    rm = mgr.rollout_mgr
    L_ = nat.lib()
    assert L_.mlearn_policy_rollout_pop_kernel(pss[0].desc, None, B, P, 0) == 2
    rm.rollout_kernel = 2
    cus = torch.cuda.get_device_properties(gpu).multi_processor_count
    tpp, TW = B // 16, cus * 8
    ntile = P * tpp
    assert ntile > TW  # rounds in series
    # second-round tiles of workgroups whose first round was another policy
    picks = []
    for wg in (0, cus // 2 - 1, cus - 1):
        t1 = TW + 8 * wg
        if t1 < ntile and t1 // tpp != (8 * wg) // tpp:
            picks.append(t1 + 2 * (wg % 4))
    picks.append(ntile - 2)
    assert len(picks) >= 3, picks
    p0s = [ps.params.cpu().numpy().astype(np.float64) for ps in pss]
    mgr.update_iter()
    torch.cuda.synchronize()
    assert getattr(rm, "_pop_sig", None) is not None  # the population launch ran
    s = rm.store
    lay = ref.param_layout(D, H, 2, 26)
    for t in picks:
        e0 = 16 * t  # a 32-env window: tiles t, t + 1 of the same workgroup round
        _check_window(s, mgr, env, p0s[e0 // B], lay, e0, cfg)


def test_lstm_8192_rollout_and_update(gpu):
    """Config L at its stated size: RecurrentBackboneEncoder(MLP[256,256],
    LSTM(256)) over 8192 envs, bf16, minibatches of 2048 sequences (one
    epoch = 4 optimizer steps).  The whole-rollout launch (carry, start
    states, done clears) is checked on oracle column windows spread over the
    env tiles; the update against the oracle's BPTT update of the same store
    under the per-tensor bf16 bound."""
    import madrona_learn as ml
    from madrona_learn import _native as nat
    from madrona_learn.envs import DummyVecEnv
    from tests.test_gpu_lstm import make_actor_critic
    N, mb = 8192, 2048
    env = DummyVecEnv(N, D, 6, seed=7, device=gpu)
    cfg = _cfg(N, mb, seed=21)
    pol = ml.Policy(actor_critic=make_actor_critic(H, 2, torch.bfloat16),
                    obs_preprocess=ml.ObservationsCaster.create(torch.bfloat16))
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), pol, use_graph=False)
    ps, ts = mgr.state.policy_states, mgr.state.train_states
    grid = nat.lib().mlearn_policy_rollout_workgroups(ps.desc, ps.lstm_desc, N, 0)
    assert grid > 0  # the whole rollout as one launch
    a = ps.arch
    lay = lref.param_layout(a.obs_dim, a.hidden, a.num_layers, a.num_logits, a.critic_bins)
    p0 = ps.params.cpu().numpy().astype(np.float64)
    mgr.update_iter()
    torch.cuda.synchronize()
    s = mgr.rollout_mgr.store
    tiles = N // 32
    z32 = np.zeros((32, H))
    for tile in sorted({0, grid - 1, min(grid, tiles - 1), tiles // 2 + 1, tiles - 1}):
        e0 = tile * 32
        c = slice(e0, e0 + 32)
        oenv = onat.Env(32, D, env.k0, env.k1, e0)
        oenv.reset()
        ro, _, _ = lref.rollout(p0, lay, oenv, T, T, BUCKETS, mgr.rollout.prng_key, 0,
                                (z32, z32), mode="bf16", gamma=cfg.gamma,
                                actions_override=s.actions[:, c].cpu().numpy())
        _check_store(s, ro, c)
    store = {k: v.float().cpu().numpy() if v.dtype == torch.bfloat16 else v.cpu().numpy()
             for k, v in s.as_dict().items()}
    store["start_h"] = s.start_h.float().cpu().numpy()
    store["start_c"] = s.start_c.float().cpu().numpy()
    assert not store["start_h"].any()  # the first rollout starts from zero carries
    zeros = np.zeros_like(p0)
    upd = dict(num_epochs=1, minibatch_size=mb, bptt=T, key=ts.update_prng_key, epoch_base=0,
               lr=3e-4, max_grad_norm=0.5)
    norms = ps.init_norms.cpu().numpy().astype(np.float64)
    pb, _, _ = lref.ppo_update(p0, (zeros, zeros.copy(), 0), [store], HP, BUCKETS, lay, norms,
                               mode="bf16", **upd)
    pf, _, _ = lref.ppo_update(p0, (zeros, zeros.copy(), 0), [store], HP, BUCKETS, lay, norms,
                               mode="f32", **upd)
    check_bf16_update("config_L_8192", ps.params.cpu().numpy(), p0, pb, pf, lay)
    assert int(ts.step.item()) == N // mb


@pytest.mark.parametrize("kernel", [1, 2])
def test_headline_rollout_tiles_in_series(gpu, kernel):
    """The headline (BASELINE metric) rollout, 65,536 envs, on both rollout
    kernels (mlearn_rollout_out.policy_kernel):
      1 feature split: 2,048 32-env tiles on fewer resident workgroups, so
        every workgroup runs several tiles in series, reusing the parameters
        it staged in LDS once;
      2 row split (the library's choice here): 4,096 16-env tiles over one
        8-wave workgroup per CU, two in series per wave, the sim's next
        observations carried in registers and written to the env once.
    32-env windows of the second tile round (and the last one) are replayed on
    the oracle env + policy: obs / rewards / dones / GAE bit-exact, values /
    log-probs within the bf16 tolerance, sampled actions equal to the oracle's
    wherever the Gumbel margin is clear, and the env's observations, state
    and rewards after the rollout bit-exact."""
    from madrona_learn import _native as nat
    from madrona_learn.envs import DummyVecEnv
    import madrona_learn as ml
    from tests.test_gpu_train import make_policy
    N, mb = 65536, 2048
    env = DummyVecEnv(N, D, 6, seed=6, device=gpu)
    cfg = _cfg(N, mb, seed=13)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), make_policy(torch.bfloat16, H),
                           use_graph=False)
    ps = mgr.state.policy_states
    rm = mgr.rollout_mgr
    rm.rollout_kernel = kernel
    L_ = nat.lib()
    assert L_.mlearn_policy_rollout_kernel(ps.desc, None, N, 0, 0) == 2  # auto: row split
    assert L_.mlearn_policy_rollout_kernel(ps.desc, None, N, 0, kernel) == kernel
    assert L_.mlearn_policy_rollout_kernel(ps.desc, None, N, 2, 2) == -1  # capped: no row split
    if kernel == 1:
        grid = L_.mlearn_policy_rollout_workgroups(ps.desc, None, N, 0)
        tiles = N // 32
        assert 0 < grid < tiles, (grid, tiles)
        assert -(-tiles // grid) >= 2
        picks = [grid + 3, tiles - 1] + ([2 * grid + 5] if 2 * grid + 5 < tiles else [])
        windows = [t * 32 for t in picks]
    else:
        waves = torch.cuda.get_device_properties(gpu).multi_processor_count * 8
        assert N // 16 >= 2 * waves
        windows = [(16 * (waves + 7)) // 32 * 32, N - 32, (16 * waves) // 32 * 32 + 32 * 40]
    _replay_windows(mgr, env, cfg, windows)


@pytest.mark.parametrize("N", [32768])
def test_row_split_rollout_rank_sizes(gpu, N):
    """The row-split rollout at a two-rank data-parallel shard (32,768 envs:
    one 8-wave workgroup per CU, one 16-env tile per wave), the library's
    choice there: oracle windows at the start, middle and end as in the
    headline test."""
    from madrona_learn import _native as nat
    from madrona_learn.envs import DummyVecEnv
    import madrona_learn as ml
    from tests.test_gpu_train import make_policy
    mb = N // 4
    env = DummyVecEnv(N, D, 6, seed=7, device=gpu)
    cfg = _cfg(N, mb, seed=17)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), make_policy(torch.bfloat16, H),
                           use_graph=False)
    ps = mgr.state.policy_states
    L_ = nat.lib()
    assert L_.mlearn_policy_rollout_kernel(ps.desc, None, N, 0, 0) == 2
    assert L_.mlearn_policy_rollout_kernel(ps.desc, None, N - 256, 0, 0) == 1
    _replay_windows(mgr, env, cfg, [0, N // 2 + 32 * 5, N - 32])


def _replay_windows(mgr, env, cfg, windows, critic_bins=1):
    ps = mgr.state.policy_states
    rm = mgr.rollout_mgr
    p0 = ps.params.cpu().numpy().astype(np.float64)
    mgr.update_iter()
    torch.cuda.synchronize()
    s = rm.store
    lay = ref.param_layout(D, H, 2, 26, critic_bins)
    for e0 in windows:
        c = slice(e0, e0 + 32)
        oenv = onat.Env(32, D, env.k0, env.k1, e0)
        oenv.reset()
        acts = s.actions[:, c].cpu().numpy()
        ro, _ = ref.rollout(p0, lay, oenv, T, BUCKETS, mgr.rollout.prng_key, 0, mode="bf16",
                            gamma=cfg.gamma, actions_override=acts)
        vsens = None
        if critic_bins > 1:  # 1-ulp sensitivity of the oracle's mean(), every step + bootstrap
            P0 = ref.unflatten(p0, lay)
            x = np.concatenate([ro["obs"], env.obs[c].cpu().numpy()[None]]).reshape(-1, D)
            _, _, cache = ref.forward(P0, ref.rnd(x, "bf16"), "bf16")
            crit = np.asarray(cache["crit"], np.float64)
            pr = np.exp(crit - crit.max(-1, keepdims=True))
            pr /= pr.sum(-1, keepdims=True)
            bins = ref.twohot_bins(critic_bins).astype(np.float64)
            mean = (pr * bins).sum(-1, keepdims=True)
            ulp = np.exp2(np.floor(np.log2(np.maximum(np.abs(crit), 1e-30))) - 7)
            vsens = (pr * np.abs(bins - mean) * ulp).sum(-1).reshape(T + 1, 32)
        _check_store(s, ro, c, vsens)
        gum = np.stack([onat.gumbel_table(*mgr.rollout.prng_key, t, e0, 32, 26)
                        for t in range(T)])
        noisy = ro["logits"] + gum
        off = 0
        for g, nb in enumerate(BUCKETS):
            sl = noisy[..., off:off + nb]
            srt = np.sort(sl, -1)
            clear = (srt[..., -1] - srt[..., -2]) > 1e-2
            assert np.array_equal(np.argmax(sl, -1)[clear], acts[..., g][clear]), (e0, g)
            off += nb
        # the env after the rollout (the row split writes it once, at the end)
        assert np.array_equal(env.obs[c].cpu().numpy(), oenv.obs), e0
        assert np.array_equal(env.state[c].cpu().numpy(), oenv.state), e0
        assert np.array_equal(env.rewards[c].cpu().numpy().reshape(-1), oenv.rew), e0
        assert np.array_equal(env.dones[c].cpu().numpy().reshape(-1).astype(np.uint8),
                              oenv.done), e0


def test_twohot_rollout_row_split(gpu):
    """The row-split rollout with the reference's default critic, a DreamerV3
    two-hot critic of 63 bins (round 6: head width 96, the head image streamed
    from L2, SymExpTwoHotDistribution.mean() by each row's four lanes), at the
    headline's 65,536 envs: oracle windows in several tile rounds (obs /
    rewards / dones / GAE bit-exact, values and log-probs within the bf16
    tolerance, sampled actions where the Gumbel margin is clear) with
    perturbed, non-trivial bin weights (the critic is zero-initialised)."""
    import dataclasses
    from madrona_learn import _native as nat
    from madrona_learn.envs import DummyVecEnv
    import madrona_learn as ml
    from tests.test_gpu_policy import perturb
    from tests.test_gpu_train import make_policy
    N, mb = 65536, 2048
    env = DummyVecEnv(N, D, 6, seed=8, device=gpu)
    cfg = dataclasses.replace(_cfg(N, mb, seed=19), dreamer_v3_critic=True)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(),
                           make_policy(torch.bfloat16, H, critic_bins=63), use_graph=False)
    ps = mgr.state.policy_states
    assert ps.arch.critic_bins == 63
    perturb(ps, 11)
    L_ = nat.lib()
    assert L_.mlearn_policy_rollout_kernel(ps.desc, None, N, 0, 0) == 2  # auto: row split
    waves = torch.cuda.get_device_properties(gpu).multi_processor_count * 8
    _replay_windows(mgr, env, cfg, [(16 * (waves + 7)) // 32 * 32, N - 32, 0], critic_bins=63)
