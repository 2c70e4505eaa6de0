"""Benchmark: env-steps/s of the full batched-PPO iteration on MI355X.

Default workload = BASELINE.json's metric: 65,536-env PPO (T=32, obs 64,
MLP[256,256] BackboneShared + discrete head [4,8,5,5,2,2] + scalar critic,
bf16 compute), PPO 2 epochs x 32 minibatches of 2048 sequences (global
minibatch), synthetic dummy vec-env (HIP kernel).  One
"step" = one full update_iter (32 rollout steps + bootstrap + GAE + 64
minibatch optimizer steps), captured in HIP graphs.  Strong scaling: the
65,536 envs and the global minibatch are split over the ranks
(torch.distributed.run, one process per GPU): each rank owns 65536/W envs
and 2048/W sequences of every minibatch, RCCL all-reduce of the advantage
statistics and of every minibatch gradient.

Other BASELINE.json configs (secondary lines, ``--config``): ``b1`` =
configs[1] (8192 envs, 4 minibatches of 2048 seqs per epoch); ``lstm`` =
configs[3] (b1 with RecurrentBackboneEncoder(MLP[256,256], LSTM(256)),
``--bptt-chunks`` C in {1, 2}); ``pbt`` = configs[4] (8 train policies x
8192 envs, self-play split, placed over the ranks: one policy per GPU at 8
GPUs, all 8 on one GPU at N = 1).

Prints ONE JSON line on rank 0.
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "madrona-learn_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np
import torch
import torch.distributed as dist

BUCKETS = [4, 8, 5, 5, 2, 2]
T, OBS, HID, LAYERS = 32, 64, 256, 2
EPOCHS, MB = 2, 2048      # global minibatch (sequences) of every config
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_PEAK_TFS = 2500.0    # dense bf16 MFMA spec
FWD_FLOP = 2 * (OBS * HID + HID * HID + HID * (sum(BUCKETS) + 1))  # 177,664 per sample
PBT_POLICIES = 8
# total envs of the job (fixed as the GPU count grows: strong scaling)
TOTAL_ENVS = {"headline": 65536, "b1": 8192, "lstm": 8192, "pbt": 8192 * PBT_POLICIES}
# the CPU baseline runs the oracle on a B1-sized shard (same work per env-step)
N_B1 = 8192


def envs_per_rank(config, world):
    total = TOTAL_ENVS[config]
    if config == "pbt" and PBT_POLICIES % world != 0 and world % PBT_POLICIES != 0:
        raise SystemExit(f"--config pbt places {PBT_POLICIES} policies: world must divide it")
    if total % world != 0:
        raise SystemExit(f"{total} envs do not split over {world} ranks")
    return total // world


def make(dev, total_envs, env_offset, n_local, dtype=torch.bfloat16, use_graph=True,
         config="headline", chunks=1, critic="scalar", fused_sim=True):
    """init_training on this rank: the config is GLOBAL (num_worlds =
    total_envs, minibatch_size = MB sequences); the sim plugin serves this
    rank's shard of n_local envs starting at env_offset."""
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from madrona_learn.models import (MLP, DenseLayerCritic, DenseLayerDiscreteActor,
                                      DreamerV3Critic)
    from madrona_learn.rnn import LSTM
    env = DummyVecEnv(n_local, OBS, len(BUCKETS), seed=0, env_offset=env_offset, device=dev)
    pbt = None
    if config == "pbt":
        pbt = ml.PBTConfig(num_teams=1, team_size=1, num_train_policies=PBT_POLICIES,
                           num_past_policies=0, self_play_portion=1.0, cross_play_portion=0.0,
                           past_play_portion=0.0)
    cfg = ml.TrainConfig(
        num_worlds=total_envs, num_agents_per_world=1, num_updates=1,
        actions={"actions": ml.DiscreteActionsConfig(BUCKETS)}, steps_per_update=T, lr=3e-4,
        algo=ml.PPOConfig(num_epochs=EPOCHS, minibatch_size=MB, clip_coef=0.2,
                          value_loss_coef=0.5, entropy_coef={"actions": 0.01},
                          max_grad_norm=0.5),
        num_bptt_chunks=chunks, gamma=0.99, gae_lambda=0.95, seed=0, metrics_buffer_size=8,
        dreamer_v3_critic=critic == "twohot", compute_dtype=dtype, pbt=pbt)
    if config == "lstm":
        encoder = ml.RecurrentBackboneEncoder(net=MLP(HID, LAYERS, dtype),
                                              rnn=LSTM(HID, 1, dtype))
    else:
        encoder = ml.BackboneEncoder(net=MLP(HID, LAYERS, dtype))
    policy = ml.Policy(
        actor_critic=ml.ActorCritic(
            backbone=ml.BackboneShared(encoder=encoder),
            actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dtype),
            critic=DenseLayerCritic(dtype) if critic == "scalar" else DreamerV3Critic(dtype)),
        obs_preprocess=ml.ObservationsCaster.create(dtype))
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        mgr = ml.init_training(dev, cfg, env.sim_fns(fused=fused_sim), policy,
                               use_graph=use_graph)
    return mgr


def time_call(fn, iters, stream):
    """Average device time of fn() over iters launches, HIP events recorded on
    `stream` (the stream fn launches on)."""
    with torch.cuda.stream(stream):
        fn()
        start = torch.cuda.Event(enable_timing=True)
        end = torch.cuda.Event(enable_timing=True)
        start.record(stream)
        for _ in range(iters):
            fn()
        end.record(stream)
    end.synchronize()
    return start.elapsed_time(end) / iters * 1e-3  # seconds


def flop_per_sample(D=OBS, H=HID, L=LAYERS, A1=sum(BUCKETS) + 1):
    """Algorithmic FLOPs per sample: trunk + heads forward, and
    the backward's dX products (d head -> d A_{L-1}, dZ_l -> dA_{l-1}); the
    weight gradients (X^T dZ) are the wgrad kernel's."""
    fwd = 2 * (D * H + (L - 1) * H * H + H * A1)
    bwd_dx = 2 * (A1 * H + (L - 1) * H * H)
    wgrad = 2 * (D * H + (L - 1) * H * H + H * A1)
    return fwd, bwd_dx, wgrad


# newest first: this round's summary of the headline kernels, then round 5's
# (which also holds the feature-split kernels the other configs run)
PMC_FILES = [os.path.join(ROOT, "profiles", f) for f in ("pmc_r06.json", "pmc_r05.json")]
PMC_SOURCE = {}


def pmc_traffic(kernel_key):
    """HBM bytes per launch of a kernel from the committed rocprofv3 PMC
    summaries (profiles/pmc_r06.json, then pmc_r05.json; tools/pmc_traffic.py):
    FETCH_SIZE doubled (gfx950 reports half the bytes of 16-B streaming reads,
    MI355X_MICROARCH.md HBM) + WRITE_SIZE, with the profiled kernel's name.
    The summary's path is kept in PMC_SOURCE[kernel_key].  (None, None) when
    no summary holds the kernel."""
    for path in PMC_FILES:
        if not os.path.exists(path):
            continue
        with open(path) as f:
            d = json.load(f)
        k = d.get("kernels", {}).get(kernel_key)
        if k is not None:
            PMC_SOURCE[kernel_key] = os.path.relpath(path, ROOT)
            return k.get("hbm_bytes_per_launch"), k.get("kernel_name")
    return None, None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def kernel_rooflines(mgr, dev, n_local, iters=20):
    """Dominant kernel (the fused PPO minibatch fwd/loss/bwd step) plus the
    rollout policy step and GAE, each timed live with HIP events on the
    stream the kernel is launched on."""
    from madrona_learn import _native as nat
    L = nat.lib()
    algo = mgr.algo
    ps = mgr.state.policy_list[0]
    stream = torch.cuda.Stream(device=dev)
    seqs = algo.perm[0, :algo.mb]

    def step():
        nat.check(L.mlearn_ppo_minibatch_fwd_bwd(ps.desc, algo.view, nat.ptr(seqs), algo.mb,
                                                 nat.ptr(algo.adv_stats[0, 0]), algo.hp,
                                                 nat.ptr(algo.ws), nat.stream_handle(stream)))

    t_step = time_call(step, iters, stream)
    M = algo.mb * algo.bptt
    A1 = ps.arch.num_logits + ps.arch.critic_bins
    fwd, bwd, _ = flop_per_sample(A1=A1)
    step_flop = (fwd + bwd) * M
    achieved = step_flop / t_step / 1e12
    # the step kernel launch_minibatch picks for this policy and minibatch
    # (mlearn_ppo_step_kernel: 2 = row-split, 1 = feature-split; csrc/ppo.hip)
    HC = 32 if A1 <= 32 else 96
    sk = int(L.mlearn_ppo_step_kernel(ps.desc, M, int(algo.hp.step_kernel)))
    if sk == 2:
        kname = "ppo_rows16_kernel<false> (row-split)"
        mangled = ("ppo_rows16_kernel",)
        pmc_key = "ppo_rows16"
    else:
        kname = f"ppo_step_kernel<bf16,{HID},{LAYERS},0,{HC},1> (feature-split)"
        mangled = ("ppo_step_kernel", f"Li{HC}ELi1E")
        pmc_key = "ppo_step"
    traffic, pmc_name = pmc_traffic(pmc_key)
    if pmc_name is None or not all(m in pmc_name for m in mangled) or "<true>" in pmc_name or "ILb1" in pmc_name:
        traffic, pmc_name = None, None  # the committed PMC pass profiled another kernel
    roof = {
        "kernel": f"{kname} (mlearn_ppo_minibatch_fwd_bwd)",
        "bound": "mfma", "achieved": achieved, "peak": BF16_PEAK_TFS, "unit": "TFLOP/s",
        "frac": achieved / BF16_PEAK_TFS, "traffic": traffic,
        "traffic_source": (f"{PMC_SOURCE.get(pmc_key)} ({pmc_name})"
                           if traffic is not None else None),
        "avg_launch_us": t_step * 1e6, "algorithmic_flop_per_launch": step_flop,
        # achieved / frac use avg_launch_us: HIP events on the stream the
        # kernel is launched on, around `iters` back-to-back launches of the
        # step-only entry (metrics off); the committed rocprofv3 stats of the
        # same kernel (profiles/) average every launch of the
        # update, metrics-on minibatches included
        "timing_source": f"hip_events: {iters} launches of mlearn_ppo_minibatch_fwd_bwd on "
                         f"its own stream",
        "units_per_launch": M, "flop_per_unit": fwd + bwd,
        "algorithmic_bytes_per_launch": 184 * M,
        # the measured traffic is dominated by the weight-gradient operands the
        # kernel writes for wgrad_kernel (X_0, A_l, dZ_l, d head rows in bf16,
        # 2,240 B/row = 147 MB at 65,536 rows)
        "traffic_note": "HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE); includes the "
                        "2240 B/row weight-gradient operand spill",
    }

    # the whole-rollout launch the update runs (mlearn_policy_rollout_env:
    # T policy steps with the fused sim step + the bootstrap critic)
    rm, rs = mgr.rollout_mgr, mgr.rollout
    extra = {}
    if rs.native_step is not None and rm.whole_rollout and ps.lstm_desc is None:
        obs0 = rm.prep_obs(rs.cur_obs)
        rout = rm._rollout_out(rs, 0, float(rm._cfg.reward_gamma))
        edesc = rm._env_desc(rs.native_step, 0)
        rstream = torch.cuda.Stream(device=dev)

        def roll():
            ps.rollout_all(obs0[:rm.B], rout, rs.prng_key, rs.counters[0:1], rm.env_offset,
                           edesc)

        t_roll = time_call(roll, 5, rstream)
        roll_flop = fwd * rm.B * (T + 1)
        rk = int(L.mlearn_policy_rollout_kernel(ps.desc, None, rm.B, rm.rollout_workgroups,
                                                int(rm.rollout_kernel)))
        if rk == 2:  # row split: one 8-wave workgroup per CU, 16-env tiles per wave
            cus = torch.cuda.get_device_properties(dev).multi_processor_count
            kname, grid, tiles = "rollout16_kernel (row-split)", min(cus, rm.B // 128), rm.B // 16
        else:
            kname = "policy_rollout_kernel (feature-split)"
            grid = int(L.mlearn_policy_rollout_workgroups(ps.desc, None, rm.B,
                                                          rm.rollout_workgroups))
            tiles = -(-rm.B // 32)
        extra["policy_rollout"] = {
            "kernel": f"{kname} (mlearn_policy_rollout_env)", "bound": "mfma",
            "envs": rm.B, "steps": T + 1, "workgroups": grid, "env_tiles": tiles,
            "avg_launch_us": t_roll * 1e6, "us_per_step": t_roll * 1e6 / (T + 1),
            "achieved": roll_flop / t_roll / 1e12, "unit": "TFLOP/s",
            "frac": roll_flop / t_roll / 1e12 / BF16_PEAK_TFS}
    # one whole minibatch gradient (step + weight gradients + reduction) and
    # one optimizer step (clip + Adam + projections + weight images)
    grad = torch.zeros_like(mgr.state.train_list[0].grads)

    def mbgrad():
        nat.check(L.mlearn_ppo_minibatch_grad(ps.desc, algo.view, nat.ptr(seqs), algo.mb,
                                              nat.ptr(algo.adv_stats[0, 0]), algo.hp,
                                              nat.ptr(grad), None, nat.ptr(algo.ws),
                                              nat.stream_handle(stream)))

    t_grad = time_call(mbgrad, iters, stream)
    ts = mgr.state.train_list[0]
    ostream = torch.cuda.Stream(device=dev)
    t_opt = time_call(lambda: ts.optimizer_step(ps), iters, ostream)
    extra["minibatch"] = {"rows": M, "step_us": t_step * 1e6,
                          "grad_us": t_grad * 1e6, "optimizer_step_us": t_opt * 1e6,
                          "optimizer_steps_per_update": algo.E * algo.num_mb}
    # the product path writes only the advantages (returns = advantages +
    # values are formed by their consumers); "materialised" = the 8 B/elem
    # form (value normaliser / compute_advantages=False paths).  frac_read
    # is capped by read / (read + write) x the achievable copy bandwidth:
    # 9/13 x 6.29/8 = 0.54 derived, 9/17 x 6.29/8 = 0.42 materialised
    gae = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
           "bytes_per_env": {"read": T * 9 + 4, "write": T * 4},
           "frac_read_ceiling": (T * 9 + 4) / (T * 13 + 4) * 6290.0 / HBM_PEAK_GBS}
    for name, n in (("operating_point", n_local), ("sweep_point", 1 << 22)):
        for mat in (False, True):
            sec, rd, wr = gae_roofline(dev, n, iters=50 if n < (1 << 20) else 20, returns=mat)
            key = name + ("_materialised_returns" if mat else "")
            gae[key] = {"N": n, "avg_launch_us": sec * 1e6,
                        "achieved_read": rd / sec / 1e9,
                        "achieved_read_write": (rd + wr) / sec / 1e9,
                        "frac_read": rd / sec / 1e9 / HBM_PEAK_GBS,
                        "frac_read_write": (rd + wr) / sec / 1e9 / HBM_PEAK_GBS}
    extra["gae"] = gae
    return roof, extra


def gae_roofline(dev, N, iters=50, returns=False):
    from madrona_learn import _native as nat
    r = torch.randn((T, N), device=dev)
    v = torch.randn((T, N), device=dev)
    d = (torch.rand((T, N), device=dev) < 0.05).to(torch.uint8)
    b = torch.randn(N, device=dev)
    adv = torch.empty_like(r)
    ret = torch.empty_like(r) if returns else None
    s = torch.cuda.Stream(device=dev)
    L = nat.lib()

    def call():
        nat.check(L.mlearn_gae_f32(nat.ptr(r), nat.ptr(v), nat.ptr(d), nat.ptr(b), nat.ptr(adv),
                                   nat.ptr(ret) if returns else None, T, N, 0.99, 0.99 * 0.95,
                                   nat.stream_handle(s)))

    sec = time_call(call, iters, s)
    read = T * N * (4 + 4 + 1) + 4 * N
    write = (8 if returns else 4) * T * N
    return sec, read, write


def cpu_baseline(iters=2):
    """Two timed runs of the oracle's CPU iteration (_cpu_baseline_run): BLAS
    on every CPU of this process's affinity mask (SURVEY §8(d)'s whole-host
    reading) and on 16 threads (the box's CPU share per GPU; on a many-socket
    host the small GEMMs of this workload lose to oversubscription across
    sockets).  `value` is the faster of the two, both runs are listed."""
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else \
        (os.cpu_count() or 1)
    runs = [_cpu_baseline_run(iters, cores)]
    if cores > 16:
        runs.append(_cpu_baseline_run(iters, 16))
    best = max(runs, key=lambda r: r["value"])
    out = dict(best)
    out["runs"] = [{"value": r["value"], "cores": r["cores"], "seconds": r["seconds"]}
                   for r in runs]
    out["threads_note"] = ("cores = BLAS pool threads during the faster timed run "
                           "(threadpoolctl); runs = every CPU of the affinity mask and 16")
    return out


def _cpu_baseline_run(iters, threads):
    """The oracle restatement (NumPy fp32 arithmetic, host BLAS threads) of
    `iters` full PPO iterations on an 8192-env shard of the workload: 8192
    envs x T=32 rollout with the synthetic env, GAE, 2 epochs over every
    sequence in minibatches of 2048 sequences (~10-30 s of CPU work on the
    GPU box's host).  The work per env-step (one policy forward in the
    rollout, two forward+backward passes in the update) is the same as in
    the 65,536-env workload, so env-steps/s compare directly."""
    from oracle import native as onat
    from oracle import ppo_ref as ref
    n_env = N_B1
    mb = MB
    lay = ref.param_layout(OBS, HID, LAYERS, sum(BUCKETS))
    rng = np.random.default_rng(0)
    p = np.zeros(lay["total"], np.float32)
    for o, shp in lay["W"]:
        p[o:o + shp[0] * shp[1]] = (rng.standard_normal(shp) / np.sqrt(shp[0])).reshape(-1)
    for o, shp in lay["s"]:
        p[o:o + shp[0]] = 1.0
    o, shp = lay["Wh"]
    p[o:o + shp[0] * shp[1]] = (rng.standard_normal(shp) * 0.01).reshape(-1)
    env = onat.Env(n_env, OBS, 1, 2)
    env.reset()
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01}
    # `threads` BLAS threads (the caller runs every host core of the affinity
    # mask), set on the BLAS pools the NumPy
    # restatement runs its products in; the thread count reported is what the
    # pools report back while the timed region runs
    from threadpoolctl import threadpool_info, threadpool_limits
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else \
        (os.cpu_count() or 1)
    limiter = threadpool_limits(limits=threads)
    used = max([p.get("num_threads", 1) for p in threadpool_info()] or [1])
    norms = np.ones(LAYERS)
    pf = p.astype(np.float64)
    opt = (np.zeros(lay["total"]), np.zeros(lay["total"]), 0)
    er = None
    t0 = time.perf_counter()
    for it in range(iters):
        ro, er = ref.rollout(pf.astype(np.float32), lay, env, T, BUCKETS, (3, 4), it * T,
                             mode="f32", ad=np.float32, env_returns=er)
        adv, ret = ref.gae_f32(ro["rewards"], ro["values"], ro["dones"], ro["bootstrap"], 0.99,
                               0.95)
        store = dict(ro)
        store["advantages"], store["returns"] = adv, ret
        pf, opt, _ = ref.ppo_update(pf, opt, [store], hp, BUCKETS, lay, norms,
                                    num_epochs=EPOCHS, minibatch_size=mb, bptt=T, key=(5, 6),
                                    epoch_base=it * EPOCHS, mode="f32", lr=3e-4,
                                    max_grad_norm=0.5, ad=np.float32)
    sec = time.perf_counter() - t0
    limiter.restore_original_limits()
    return {"value": iters * n_env * T / sec, "unit": "env-steps/s", "cores": used,
            "kind": "port", "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "cores_available": cores, "seconds": sec,
            "sample": f"{iters} full PPO iterations on a {n_env}-env shard ({n_env} envs x "
                      f"T={T}, 2 epochs x {n_env // mb} minibatches of {mb} seqs; same work per "
                      f"env-step as the 65536-env workload), NumPy fp32 oracle restatement, "
                      f"{sec:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-separate-sim-line", action="store_true",
                    help="skip the headline's second measurement with the sim step as its own "
                         "launch (separate_sim_ms_per_update)")
    ap.add_argument("--config", choices=["headline", "b1", "lstm", "pbt"], default="headline")
    ap.add_argument("--bptt-chunks", type=int, default=1)
    ap.add_argument("--separate-sim", action="store_true",
                    help="run the synthetic sim's step as its own launch between the policy "
                         "launches (as a user sim plugin runs) instead of fused into them")
    ap.add_argument("--critic", choices=["scalar", "twohot"], default="scalar",
                    help="DenseLayerCritic (SURVEY B1) or DreamerV3Critic (63-bin two-hot)")
    ap.add_argument("--emulate-world", type=int, default=1,
                    help="one process, one GPU: time rank 0's share of a W-rank headline job "
                         "(65536/W envs, minibatch slices of 2048/W seqs, every minibatch's "
                         "gradient all-reduce a real RCCL call on a one-rank communicator) and "
                         "the N=1 headline, and print the implied 1->W strong scaling")
    ap.add_argument("--per-policy-rollouts", action="store_true",
                    help="config pbt: one whole-rollout launch per policy instead of the "
                         "population launch (RolloutManager.population_launch = False)")
    ap.add_argument("--rollout-kernel", type=int, choices=[0, 1, 2], default=0,
                    help="RolloutManager.rollout_kernel: 0 the library's choice, 1 the "
                         "feature-split rollout kernels, 2 the row-split ones (A/B runs)")
    ap.add_argument("--step-kernel", type=int, choices=[0, 1, 2], default=0,
                    help="PPO.step_kernel: 0 the library's choice, 1 the feature-split "
                         "minibatch kernel, 2 the row-split one (A/B runs)")
    ap.add_argument("--wgrad-form", type=int, choices=[0, 1, 2], default=0,
                    help="PPO.wgrad_form: 0 the library's choice, 1 the register-staged "
                         "weight-gradient launch, 2 the LDS-DMA pipeline (A/B runs)")
    ap.add_argument("--optim-launch", type=int, choices=[0, 1, 2], default=0,
                    help="PolicyTrainState.optim_launch_form: 0 the library's choice, 1 the "
                         "split optimizer launches, 2 the fused one (A/B runs)")
    ap.add_argument("--no-fused-gae", action="store_true",
                    help="RolloutManager.fused_gae = False: GAE as its own launch (A/B runs)")
    args = ap.parse_args()
    from madrona_learn.train_state import PolicyTrainState
    PolicyTrainState.optim_launch_form = args.optim_launch
    from madrona_learn.ppo import PPO
    PPO.step_kernel = args.step_kernel
    PPO.wgrad_form = args.wgrad_form
    from madrona_learn.rollouts import RolloutManager
    if args.per_policy_rollouts:
        RolloutManager.population_launch = False
    RolloutManager.rollout_kernel = args.rollout_kernel
    RolloutManager.fused_gae = not args.no_fused_gae
    if args.emulate_world > 1:
        return emulate_world(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # test hooks: MLEARN_DIST_BACKEND=gloo and MLEARN_SHARE_GPU=1 run several ranks on one
    # GPU (the driver's multi-GPU runs use the defaults: RCCL, one GPU per rank)
    backend = os.environ.get("MLEARN_DIST_BACKEND", "nccl")
    if os.environ.get("MLEARN_SHARE_GPU") == "1":
        local = 0
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    total = TOTAL_ENVS[args.config]
    n_rank = envs_per_rank(args.config, world)
    mgr = make(dev, total, rank * n_rank, n_rank, use_graph=not args.no_graph,
               config=args.config, chunks=args.bptt_chunks, critic=args.critic,
               fused_sim=not args.separate_sim)
    for _ in range(args.warmup):
        mgr.update_iter()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # per-update device intervals (events between the updates, no host sync)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(args.steps):
        mgr.update_iter()
        evs[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    per_update = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_steps = total * T * args.steps
    value = total_steps / elapsed
    ms = elapsed / args.steps * 1e3

    result = None
    if rank == 0:
        npol = PBT_POLICIES if args.config == "pbt" else 1
        nmb = total // npol // MB * args.bptt_chunks
        workload = {
            "headline": f"65536-env PPO iteration (BASELINE metric; SURVEY B8 semantics): T=32, "
                        f"obs=64, MLP[256,256], heads [4,8,5,5,2,2]+critic, 2 epochs x {nmb} "
                        f"minibatches of {MB} seqs (global), envs and minibatches split over "
                        f"{world} GPU(s)",
            "b1": f"B1: PPO iteration, 8192 envs, T=32, obs=64, MLP[256,256], heads "
                  f"[4,8,5,5,2,2]+critic, 2 epochs x {nmb} minibatches of {MB} seqs",
            "lstm": f"L: B1 with RecurrentBackboneEncoder(MLP[256,256], LSTM(256)), "
                    f"{args.bptt_chunks} BPTT chunk(s), minibatches of {MB} seqs",
            "pbt": f"P: {PBT_POLICIES} train policies x 8192 envs (self-play split), placed over "
                   f"{world} GPU(s), B1 policy and PPO settings",
        }[args.config]
        result = {
            "metric": "env-steps/sec whole-node, 65536-env PPO, at 1/2/4/8 MI355X",
            "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (dummy vec-env HIP kernel, random-init orthogonal weights)",
            "config": {"workload": workload, "config": args.config,
                       "total_envs": total, "envs_per_gpu": n_rank,
                       "global_minibatch_seqs": MB, "minibatches_per_epoch": nmb,
                       "steps_per_update": T, "parallelism": f"dp{world}",
                       "critic": args.critic,
                       "hip_graph": not args.no_graph,
                       # the built-in synthetic sim's step: inside the whole-rollout
                       # launch (mlearn_policy_rollout_env) or its own launch
                       "sim_step": "separate_launch" if args.separate_sim
                       else "whole_rollout_one_launch"},
            # how the data-parallel collectives ran (a SCALE record can be checked
            # against this): "rccl_in_graph" = C ABI RCCL communicator on the
            # compute stream inside the HIP graph; "torch_distributed" = host
            # round trips between graph segments (reason on stderr); "none" = 1 GPU
            "collectives": mgr.dp.collectives, "rccl_ranks": mgr.dp.comm_ranks,
            # device time of each timed update (HIP events between the updates):
            # median / min / max over the K updates (value uses the wall clock above)
            "ms_per_update_median": per_update[len(per_update) // 2],
            "ms_per_update_min": per_update[0], "ms_per_update_max": per_update[-1],
        }
    if rank == 0 and not args.no_roofline and args.config != "lstm":
        result["roofline"], result["kernels"] = kernel_rooflines(mgr, dev, n_rank)
    if rank == 0 and world == 1 and not args.no_separate_sim_line and args.config == "headline" \
            and not args.separate_sim:
        # the same job with the synthetic sim's step as its own launch between
        # the policy launches, the path a user sim plugin takes (sim_fns 'step')
        del mgr
        torch.cuda.empty_cache()
        m2 = make(dev, total, 0, n_rank, use_graph=not args.no_graph, config=args.config,
                  chunks=args.bptt_chunks, critic=args.critic, fused_sim=False)
        result["separate_sim_ms_per_update"] = _time_updates(m2, max(args.steps // 2, 3),
                                                             args.warmup) * 1e3
        del m2
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config in ("headline", "b1"):
        result["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _time_updates(mgr, steps, warmup):
    for _ in range(warmup):
        mgr.update_iter()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        mgr.update_iter()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def emulate_world(args):
    """Strong-scaling projection on one GPU: rank 0's share of a W-rank
    headline job (madrona_learn.dist.set_emulated_world), then the N=1
    headline in the same process.  The share's per-update time bounds the
    W-GPU time from below by everything but the xGMI transfer of the
    collectives (each is issued as a one-rank RCCL all-reduce at its place
    in the graph)."""
    W = int(args.emulate_world)
    total = TOTAL_ENVS["headline"]
    if total % W or MB % W:
        raise SystemExit(f"--emulate-world {W} must divide {total} envs and {MB} seqs")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from madrona_learn import dist as mdist
    mdist.set_emulated_world(W)
    mgr = make(dev, total, 0, total // W, use_graph=not args.no_graph,
               fused_sim=not args.separate_sim)
    coll = mgr.dp.collectives
    t_w = _time_updates(mgr, args.steps, args.warmup)
    del mgr
    torch.cuda.empty_cache()
    mdist.set_emulated_world(1)
    mgr = make(dev, total, 0, total, use_graph=not args.no_graph,
               fused_sim=not args.separate_sim)
    t_1 = _time_updates(mgr, args.steps, args.warmup)
    # modeled xGMI term of the W-rank collectives the emulation runs as
    # one-rank calls: per minibatch the flat f32 gradient, per epoch the
    # advantage sums (2 doubles per minibatch).  Ring all-reduce over W
    # ranks: 2 (W - 1) steps of S / W bytes each, on one xGMI link per step
    # (beta = 153 GB/s, the per-link figure of the MI355X brief) plus a fixed
    # per-step latency alpha.  alpha is an ASSUMPTION (no measured xGMI hop
    # latency is available to this build); the line reports it.
    n_mb = EPOCHS * (total // W) // (MB // W)
    grad_bytes = 4 * int(mgr.state.policy_list[0].params.numel())
    alpha_us, beta_gbs = 2.0, 153.0

    def ring_us(nbytes):
        return 2 * (W - 1) * (alpha_us + nbytes / W / (beta_gbs * 1e3))
    ar_grad = ring_us(grad_bytes)
    ar_adv = ring_us(16 * (total // MB))  # 2 doubles per global minibatch of the epoch
    modeled_ms = n_mb * ar_grad * 1e-3 + EPOCHS * ar_adv * 1e-3
    t_w_model = t_w + modeled_ms * 1e-3
    print(json.dumps({
        "metric": "env-steps/sec whole-node, 65536-env PPO, at 1/2/4/8 MI355X (projection)",
        "emulated_world": W, "steps": args.steps, "warmup": args.warmup,
        "ms_per_update_rank_share": t_w * 1e3,
        "implied_whole_node_env_steps_per_s": total * T / t_w,
        "n1_ms_per_update": t_1 * 1e3, "n1_env_steps_per_s": total * T / t_1,
        "implied_scaling_1_to_W": t_1 / t_w,
        "modeled_allreduce": {
            "model": "ring: 2(W-1) x (alpha + S/W/beta) per all-reduce",
            "alpha_us_per_step_assumed": alpha_us, "beta_GBs_per_link": beta_gbs,
            "grad_bytes": grad_bytes, "grad_allreduces_per_update": n_mb,
            "us_per_grad_allreduce": ar_grad, "adv_allreduces_per_update": EPOCHS,
            "ms_per_update": modeled_ms},
        "ms_per_update_rank_share_with_modeled_allreduce": t_w_model * 1e3,
        "implied_scaling_1_to_W_with_modeled_allreduce": t_1 / t_w_model,
        "collectives": coll,
        "config": {"envs_per_rank": total // W, "minibatch_slice_seqs": MB // W,
                   "optimizer_steps_per_update": EPOCHS * (total // W) // (MB // W)},
        "note": "one process: the W-rank all-reduces run as one-rank RCCL calls; "
                "implied_scaling_1_to_W leaves out their xGMI transfer, the "
                "_with_modeled_allreduce fields add the ring model above"}))


if __name__ == "__main__":
    main()
