"""Diagnostic: the wide step kernel (row_blocks 2 / 4) against ppo_step_kernel
(row_blocks 1) on the same minibatch, stage by stage through the step-only
ABI's workspace (X_0, A_l, dZ_l, d head rows).  Prints max |diff| per stage."""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "madrona-learn_amd")
from tests.test_gpu_policy import make_policy_state, perturb, _random_store, _device_store  # noqa
from madrona_learn import _native as nat  # noqa


def a256(x):
    return (x + 255) & ~255


def regions(M, D, H, L, HC, es):
    Mp = (M + 127) // 128 * 128
    off, out = 0, {}
    def take(name, n):
        nonlocal off
        out[name] = (off, n)
        off = a256(off + n)
    take("x0", Mp * D * es)
    for l in range(L):
        take(f"a{l}", Mp * H * es)
        take(f"dz{l}", Mp * H * es)
    take("dhead", Mp * HC * es)
    return out, Mp


def run(gpu, dtype, mode, rb, D, H, L, mb, bptt):
    ps = make_policy_state(gpu, D, H, L, dtype, seed=H)
    perturb(ps, 9, scale=0.2)
    T, N = 32, 96
    rng = np.random.default_rng(11)
    st = _random_store(rng, T, N, D, ps, mode)
    s = _device_store(gpu, st, dtype)
    seqs = rng.permutation((T // bptt) * N)[:mb].astype(np.int32)
    hp = nat.PPOHparams()
    hp.clip_coef, hp.value_loss_coef = 0.2, 0.5
    for k in range(6):
        hp.entropy_coef[k] = 0.01
    hp.normalize_advantages, hp.loss_scale = 1, 1.0
    hp.row_blocks = rb
    stats = torch.tensor([0.1, 0.9], dtype=torch.float32, device=gpu)
    M = mb * bptt
    ws = torch.zeros(int(nat.lib().mlearn_ppo_workspace_bytes(ps.desc, M)), dtype=torch.uint8,
                     device=gpu)
    sq = torch.from_numpy(seqs).to(gpu)
    nat.check(nat.lib().mlearn_ppo_minibatch_fwd_bwd(ps.desc, s.view(bptt), nat.ptr(sq), mb,
                                                     nat.ptr(stats), hp, nat.ptr(ws),
                                                     nat.stream_handle()))
    torch.cuda.synchronize()
    return ws.cpu()


def main():
    gpu = torch.device("cuda:0")
    for dtype, mode in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
        D, H, L, mb, bptt = 64, 256, 2, 40, 32
        es = 4 if dtype == torch.float32 else 2
        reg, Mp = regions(mb * bptt, D, H, L, 32, es)
        base = run(gpu, dtype, mode, 1, D, H, L, mb, bptt)
        for rb in (2, 4):
            w = run(gpu, dtype, mode, rb, D, H, L, mb, bptt)
            msg = []
            for name, (o, n) in reg.items():
                a = base[o:o + n].view(dtype).float()
                b = w[o:o + n].view(dtype).float()
                d = (a - b).abs()
                bad = int((d > 1e-3 * (a.abs() + 1e-3)).sum())
                msg.append(f"{name}: max {float(d.max()):.3g} bad {bad}/{a.numel()}")
                if bad:
                    idx = int(torch.nonzero(d > 1e-3 * (a.abs() + 1e-3))[0])
                    cols = n // es // Mp
                    msg[-1] += f" first row {idx // cols} col {idx % cols} ({float(a[idx]):.4g} vs {float(b[idx]):.4g})"
            print(mode, "rb", rb, " | ".join(msg), flush=True)
            # a0 of the wide kernel: which base rows / columns does it match?
            o, n = reg["a0"]
            a = base[o:o + n].view(dtype).float().reshape(Mp, H)
            b = w[o:o + n].view(dtype).float().reshape(Mp, H)
            for row in (0, 1, 31, 32, 33, 63, 64):
                d = (a - b[row]).abs().sum(1)
                j = int(d.argmin())
                dc = (a[row][:, None] - b[row][None, :]).abs()
                print(f"  wide row {row}: best base row {j} (dist {float(d[j]):.3g}); "
                      f"col0 best match col {int(dc[:, 0].argmin())}", flush=True)


main()
