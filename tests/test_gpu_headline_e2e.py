"""The headline's own update end to end against the oracle (verdict r05 item
2): the BASELINE metric's configuration, 65,536 envs x T = 32, MLP[256, 256]
bf16, minibatches of 2,048 sequences (65,536 rows each), on exactly the
kernels bench.py times: the row-split rollout (rollout16_kernel), the
row-split step (ppo_rows16_kernel<false, 8, 2>), the weight-gradient /
reduction launches and the fused optimizer launch, all replayed from the
captured HIP graph (update 3: update 1 runs eagerly, update 2 captures).

The whole update's optimizer chain -- 32 dependent Adam steps, the first
epoch of the headline's 2 x 32 (the oracle's host time for 64 steps in both
of its modes exceeds the per-test budget; the second epoch reruns the same
kernels on another permutation) -- is compared, from the parameters and
Adam state after update 2 and the GPU's own rollout store of update 3,
against ref.ppo_update in the oracle's bf16 mode under the per-tensor bound
of tests/bf16_bound.py (the oracle's own bf16-vs-f32 distance).  A per-step
error that only compounds over the chain fails here even where the
one-minibatch checks (tests/test_gpu_fullsize.py) pass.  The store itself:
GAE bit-exact over all 65,536 columns; oracle rollout windows of update 1
are tests/test_gpu_configs.py::test_headline_rollout_tiles_in_series."""

import threading
import time

import numpy as np
import pytest
import torch

from oracle import ppo_ref as ref
from tests.bf16_bound import check_bf16_update

pytestmark = pytest.mark.gpu

BUCKETS = [4, 8, 5, 5, 2, 2]
HP = {"clip_coef": 0.2, "value_loss_coef": 0.5, "entropy_coef": 0.01,
      "normalize_advantages": True}
D, H, T, N, MB = 64, 256, 32, 65536, 2048


@pytest.mark.timeout(900)
def test_headline_update_chain_matches_oracle(gpu):
    import madrona_learn as ml
    from madrona_learn import _native as nat
    from madrona_learn.envs import DummyVecEnv
    from tests.test_gpu_configs import _cfg
    from tests.test_gpu_train import make_policy
    env = DummyVecEnv(N, D, 6, seed=31, device=gpu)
    cfg = _cfg(N, MB, epochs=1, seed=23)
    mgr = ml.init_training(gpu, cfg, env.sim_fns(), make_policy(torch.bfloat16, H),
                           use_graph=True)
    ps, ts = mgr.state.policy_states, mgr.state.train_states
    L_ = nat.lib()
    rows = MB * T
    assert L_.mlearn_ppo_step_kernel(ps.desc, rows, 0) == 2          # row-split step
    assert L_.mlearn_policy_rollout_kernel(ps.desc, None, N, 0, 0) == 2  # row-split rollout
    assert ts.optim_desc.launch_form == 0                          # the library's choice
    mgr.update_iter()   # eager
    mgr.update_iter()   # capture (runs the update once)
    torch.cuda.synchronize()
    assert mgr._segments is not None
    p0 = ps.params.cpu().numpy().astype(np.float64)
    m0 = ts.adam_m.cpu().numpy().astype(np.float64)
    v0 = ts.adam_v.cpu().numpy().astype(np.float64)
    c0 = int(ts.step.item())
    assert c0 == 2 * (N // MB)
    mgr.update_iter()   # graph replay: the update bench.py times
    torch.cuda.synchronize()
    assert int(ts.step.item()) == c0 + N // MB
    got = ps.params.cpu().numpy()
    s = mgr.rollout_mgr.store
    store = {k: v.float().cpu().numpy() if v.dtype == torch.bfloat16 else v.cpu().numpy()
             for k, v in s.as_dict().items()}
    adv, _ = ref.gae_f32(store["rewards"], store["values"], store["dones"],
                         s.bootstrap.cpu().numpy(), cfg.gamma, cfg.gae_lambda)
    assert np.array_equal(store["advantages"], adv)
    lay = ref.param_layout(D, H, 2, 26)
    norms = ps.init_norms.cpu().numpy().astype(np.float64)
    upd = dict(num_epochs=1, minibatch_size=MB, bptt=T, key=ts.update_prng_key, epoch_base=2,
               lr=3e-4, max_grad_norm=0.5, ad=np.float32)
    out = {}

    def run(mode):
        t0 = time.perf_counter()
        out[mode] = ref.ppo_update(p0, (m0.copy(), v0.copy(), c0), [store], HP, BUCKETS, lay,
                                   norms, mode=mode, **upd)[0]
        out[mode + "_s"] = time.perf_counter() - t0

    # the two oracle chains side by side (numpy releases the GIL in its kernels)
    th = [threading.Thread(target=run, args=(m,)) for m in ("bf16", "f32")]
    for t in th:
        t.start()
    for t in th:
        t.join()
    print(f"oracle chains: bf16 {out['bf16_s']:.1f} s, f32 {out['f32_s']:.1f} s")
    check_bf16_update("headline_65536_chain32", got, p0, out["bf16"], out["f32"], lay)
