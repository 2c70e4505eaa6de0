"""Torch-path (generic.py) update timing, eager vs HIP-graph-replayed update
(TrainingManager._update_torch: the whole update, else the PPO update only): BackboneSeparate MLP[256,256] x 2
encoders, f32, N envs, T = 32, 2 epochs x 4 minibatches, synthetic env.
usage: python tools/torch_path_bench.py [N] [updates]"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."),
                os.path.join(os.path.dirname(__file__), "..", "madrona-learn_amd")]
import torch  # noqa: E402

import madrona_learn as ml  # noqa: E402
from madrona_learn.envs import DummyVecEnv  # noqa: E402
from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
U = int(sys.argv[2]) if len(sys.argv) > 2 else 6
B = [4, 8, 5, 5, 2, 2]
dt = torch.float32
out = {}
for use_graph in (False, True):
    env = DummyVecEnv(N, 64, 6, seed=1, device="cuda:0")
    ac = ml.ActorCritic(
        backbone=ml.BackboneSeparate(actor_encoder=ml.BackboneEncoder(net=MLP(256, 2, dt)),
                                     critic_encoder=ml.BackboneEncoder(net=MLP(256, 2, dt))),
        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(B), dt), critic=DenseLayerCritic(dt))
    cfg = ml.TrainConfig(
        num_worlds=N, num_agents_per_world=1, num_updates=U,
        actions={"actions": ml.DiscreteActionsConfig(B)}, steps_per_update=32, lr=3e-4,
        algo=ml.PPOConfig(num_epochs=2, minibatch_size=N // 4, clip_coef=0.2, value_loss_coef=0.5,
                          entropy_coef={"actions": 0.01}, max_grad_norm=0.5),
        num_bptt_chunks=1, gamma=0.99, gae_lambda=0.95, seed=0, metrics_buffer_size=4,
        dreamer_v3_critic=False, compute_dtype=dt)
    mgr = ml.init_training("cuda:0", cfg, env.sim_fns(), ml.Policy(actor_critic=ac),
                           use_graph=use_graph)
    for _ in range(3):
        mgr.update_iter()
    torch.cuda.synchronize()
    ts = []
    for _ in range(U):
        t0 = time.perf_counter()
        mgr.update_iter()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    out["graph" if use_graph else "eager"] = ts[len(ts) // 2] * 1e3
    print(f"{'graph' if use_graph else 'eager'}: {ts[len(ts) // 2] * 1e3:.2f} ms per update "
          f"(median of {U}), use_graph={mgr.use_graph}", flush=True)
print(f"N={N}: eager {out['eager']:.2f} ms, graphs {out['graph']:.2f} ms per update")
