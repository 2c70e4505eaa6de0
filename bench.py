"""Benchmark: env-steps/s of the full batched-PPO iteration on MI355X.

Workload (BASELINE.json configs[1], per GPU): 8192 envs, T=32, obs 64,
MLP[256,256] BackboneShared + discrete head [4,8,5,5,2,2] + scalar critic,
bf16 compute, PPO 2 epochs x 4 minibatches of 2048 sequences, synthetic
dummy vec-env (HIP kernel).  One "step" = one full update_iter (32 rollout
steps + bootstrap + GAE + 8 minibatch optimizer steps), captured in HIP
graphs.  Multi-GPU (torch.distributed.run): each rank owns 8192 envs (weak
scaling), RCCL all-reduce of the advantage statistics and gradients.

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
N_ENVS, T, OBS, HID, LAYERS = 8192, 32, 64, 256, 2
EPOCHS, MB = 2, 2048
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_PEAK_TFS = 2500.0    # dense bf16 MFMA spec
FWD_FLOP = 2 * (OBS * HID + HID * HID + HID * (sum(BUCKETS) + 1))  # 177,664 per sample


def make(dev, dtype=torch.bfloat16, N=N_ENVS, env_offset=0, use_graph=True):
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
    env = DummyVecEnv(N, OBS, len(BUCKETS), seed=0, env_offset=env_offset, device=dev)
    cfg = ml.TrainConfig(
        num_worlds=N, num_agents_per_world=1, num_updates=1,
        actions={"actions": ml.DiscreteActionsConfig(BUCKETS)}, steps_per_update=T, lr=3e-4,
        algo=ml.PPOConfig(num_epochs=EPOCHS, minibatch_size=MB, clip_coef=0.2,
                          value_loss_coef=0.5, entropy_coef={"actions": 0.01},
                          max_grad_norm=0.5),
        num_bptt_chunks=1, gamma=0.99, gae_lambda=0.95, seed=0, metrics_buffer_size=8,
        dreamer_v3_critic=False, compute_dtype=dtype)
    policy = ml.Policy(
        actor_critic=ml.ActorCritic(
            backbone=ml.BackboneShared(encoder=ml.BackboneEncoder(net=MLP(HID, LAYERS, dtype))),
            actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(BUCKETS), dtype),
            critic=DenseLayerCritic(dtype)),
        obs_preprocess=ml.ObservationsCaster.create(dtype))
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        mgr = ml.init_training(dev, cfg, env.sim_fns(), policy, use_graph=use_graph)
    return mgr


def time_call(fn, iters, stream):
    """Average device time of fn() over iters launches, HIP events on `stream`."""
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


def gae_roofline(dev, N, iters=50):
    from madrona_learn import _native as nat
    rng = torch.Generator(device=dev)
    r = torch.randn((T, N), device=dev)
    v = torch.randn((T, N), device=dev)
    d = (torch.rand((T, N), device=dev) < 0.05).to(torch.uint8)
    b = torch.randn(N, device=dev)
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    s = torch.cuda.Stream()
    L = nat.lib()

    def call():
        nat.check(L.mlearn_gae_f32(nat.ptr(r), nat.ptr(v), nat.ptr(d), nat.ptr(b), nat.ptr(adv),
                                   nat.ptr(ret), T, N, 0.99, 0.95, nat.stream_handle(s)))

    sec = time_call(call, iters, s)
    read = T * N * (4 + 4 + 1) + 4 * N
    write = 8 * T * N
    return sec, read, write


def cpu_baseline(budget_s=25.0):
    """Oracle restatement (NumPy fp32, host BLAS threads) on a bounded sample:
    one full PPO iteration (rollout + GAE + 2 epochs x 4 minibatches) at a
    reduced env count so it stays within ~10-30 s."""
    from oracle import native as onat
    from oracle import ppo_ref as ref
    n_env = 1024
    mb = MB * n_env // N_ENVS
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
    t0 = time.perf_counter()
    ro, _ = ref.rollout(p, lay, env, T, BUCKETS, (3, 4), 0, mode="f32", ad=np.float32)
    adv, ret = ref.gae_f32(ro["rewards"], ro["values"], ro["dones"], ro["bootstrap"], 0.99, 0.95)
    store = dict(ro)
    store["advantages"], store["returns"] = adv, ret
    hp = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01}
    z = np.zeros(lay["total"])
    norms = np.ones(LAYERS)
    ref.ppo_update(p.astype(np.float64), (z, z.copy(), 0), [store], hp, BUCKETS, lay, norms,
                   num_epochs=EPOCHS, minibatch_size=mb, bptt=T, key=(5, 6), epoch_base=0,
                   mode="f32", lr=3e-4, max_grad_norm=0.5, ad=np.float32)
    sec = time.perf_counter() - t0
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": n_env * T / sec, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"1 PPO iteration at {n_env} envs x T={T} (2 epochs x 4 minibatches of "
                      f"{mb} seqs), NumPy fp32 oracle restatement, {sec:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    mgr = make(dev, env_offset=rank * N_ENVS, use_graph=not args.no_graph)
    for _ in range(args.warmup):
        mgr.update_iter()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        mgr.update_iter()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_steps = N_ENVS * world * T * args.steps
    value = total_steps / elapsed
    ms = elapsed / args.steps * 1e3

    result = None
    if rank == 0:
        result = {
            "metric": "env-steps/sec whole-node, 65536-env PPO, at 1/2/4/8 MI355X",
            "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (dummy vec-env HIP kernel, random-init orthogonal weights)",
            "config": {"workload": "B1: PPO iteration, 8192 envs/GPU, T=32, obs=64, "
                                   "MLP[256,256], heads [4,8,5,5,2,2]+critic, 2 epochs x 4 "
                                   "minibatches of 2048 seqs",
                       "envs_per_gpu": N_ENVS, "total_envs": N_ENVS * world,
                       "steps_per_update": T, "parallelism": f"dp{world}",
                       "hip_graph": not args.no_graph},
        }
    if rank == 0 and not args.no_roofline:
        # dominant-kernel roofline candidates, timed live with HIP events
        sec, rd, wr = gae_roofline(dev, N_ENVS * 1)
        big_sec, big_rd, big_wr = gae_roofline(dev, 1 << 22, iters=20)
        result["roofline"] = {
            "kernel": "gae_kernel (N=2^22 sweep point)", "bound": "hbm",
            "achieved": big_rd / big_sec / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": big_rd / big_sec / 1e9 / HBM_PEAK_GBS, "traffic": None,
            "algorithmic_read_bytes": big_rd, "algorithmic_write_bytes": big_wr,
            "avg_launch_us": big_sec * 1e6,
            "operating_point": {"N": N_ENVS, "avg_launch_us": sec * 1e6,
                                "read_GBs": rd / sec / 1e9},
        }
    if rank == 0 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
