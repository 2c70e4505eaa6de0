"""Action distributions (mirrors src/madrona_learn/dists.py:12-96).

``DiscreteActionDistributions`` wraps [N, sum(buckets)] logits (torch, on
the GPU) and dispatches to the HIP kernels.  RNG: the reference's
``prng_key`` becomes a Philox key (two uint32 words) plus a counter; see
DESIGN.md "RNG".
"""

import torch

from . import _native as nat


class PhiloxKey:
    """Counter-based key replacing jax.random keys: (k0, k1) plus a step.
    With ctr (a device tensor whose first element is a uint64 counter) the
    step is ctr[0] + step, read by the sampling kernel itself (no host read:
    a rollout that samples this way can be captured in a HIP graph)."""

    def __init__(self, k0, k1, step=0, env_offset=0, ctr=None):
        self.k0 = int(k0) & 0xFFFFFFFF
        self.k1 = int(k1) & 0xFFFFFFFF
        self.step = int(step)
        self.env_offset = int(env_offset)
        self.ctr = ctr


class DiscreteActionDistributions:
    def __init__(self, actions_num_buckets, all_logits: torch.Tensor):
        self.actions_num_buckets = list(actions_num_buckets)
        self.all_logits = all_logits
        self._layout = nat.action_layout(self.actions_num_buckets)

    def _logits_f32(self):
        # dists.py:22 upcasts each slice to f32
        lg = self.all_logits.float().contiguous()
        if lg.shape[-1] != self._layout.num_logits:
            raise ValueError("logits width does not match the action buckets")
        return lg.reshape(-1, lg.shape[-1])

    def _sample(self, key: PhiloxKey, sample):
        lg = self._logits_f32()
        N = lg.shape[0]
        K = len(self.actions_num_buckets)
        actions = torch.empty((N, K), dtype=torch.int32, device=lg.device)
        logp = torch.empty((N, K), dtype=torch.float32, device=lg.device) if sample else None
        L = nat.lib()
        nat.check(L.mlearn_discrete_sample_f32(
            nat.ptr(lg), lg.shape[1], self._layout, N, key.k0, key.k1,
            None if key.ctr is None else nat.ptr(key.ctr), key.step,
            key.env_offset, 1 if sample else 0, nat.ptr(actions), nat.ptr(logp),
            nat.stream_handle()), "discrete_sample")
        shape = self.all_logits.shape[:-1] + (K,)
        return actions.reshape(shape), (logp.reshape(shape) if logp is not None else None)

    def sample(self, prng_key: PhiloxKey):  # dists.py:26-44
        return self._sample(prng_key, True)

    def best(self):  # dists.py:46-52
        return self._sample(PhiloxKey(0, 0), False)[0]

    def action_stats(self, all_actions: torch.Tensor):  # dists.py:54-77
        if torch.is_grad_enabled() and self.all_logits.requires_grad:
            # differentiable form (the torch path's update, generic.py): the
            # same kernel forward, backward through the softmax
            from .generic import action_stats_autograd
            return action_stats_autograd(self, all_actions)
        lg = self._logits_f32()
        N = lg.shape[0]
        K = len(self.actions_num_buckets)
        acts = all_actions.to(torch.int32).reshape(N, K).contiguous()
        logp = torch.empty((N, K), dtype=torch.float32, device=lg.device)
        ent = torch.empty((N, K), dtype=torch.float32, device=lg.device)
        nat.check(nat.lib().mlearn_action_stats_f32(
            nat.ptr(lg), lg.shape[1], self._layout, N, nat.ptr(acts), nat.ptr(logp),
            nat.ptr(ent), nat.stream_handle()), "action_stats")
        shape = self.all_logits.shape[:-1] + (K,)
        return logp.reshape(shape), ent.reshape(shape)

    def probs(self):  # dists.py:79-88
        out = []
        off = 0
        lg = self.all_logits.float()
        for b in self.actions_num_buckets:
            out.append(torch.softmax(lg[..., off:off + b], dim=-1))
            off += b
        return out

    def logits(self):  # dists.py:90-96
        out = []
        off = 0
        for b in self.actions_num_buckets:
            out.append(self.all_logits[..., off:off + b].float())
            off += b
        return out


def _symexp(x):  # utils.py:39-40
    return torch.sign(x) * torch.expm1(torch.abs(x))


class SymExpTwoHotDistribution:  # dists.py:119-208 (critic of DreamerV3Critic)
    """Torch form for trees outside the fused path; the fused kernels compute
    the same mean() / two-hot cross entropy in csrc/dists.h."""

    def __init__(self, logits):
        self.logits = logits.float()

    @staticmethod
    def create(logits):
        return SymExpTwoHotDistribution(logits)

    def _compute_bins(self):
        nb = self.logits.shape[-1]
        assert nb % 2 == 1 and nb > 1
        half = _symexp(torch.linspace(-14, 0, nb // 2 + 1, dtype=torch.float32,
                                      device=self.logits.device))
        return torch.cat([half, -torch.flip(half[:-1], [0])])

    def mean(self):
        bins = self._compute_bins()
        mid = (bins.shape[-1] - 1) // 2
        p = torch.softmax(self.logits, -1)
        lo = (p[..., :mid] * bins[:mid]).flip(-1)
        hi = p[..., mid + 1:] * bins[mid + 1:]
        return (p[..., mid:mid + 1] * bins[mid:mid + 1]).sum(-1, keepdim=True) + \
            (lo + hi).sum(-1, keepdim=True)

    def two_hot_cross_entropy_loss(self, targets):
        bins = self._compute_bins()
        nb = bins.shape[-1]
        t = targets.float()
        lo = ((bins <= t).int().sum(-1) - 1).clamp(0, nb - 1)
        up = (nb - (bins > t).int().sum(-1)).clamp(0, nb - 1)
        same = (lo == up)[..., None]
        one = torch.ones_like(t)
        dl = torch.where(same, one, torch.abs(bins[lo][..., None] - t))
        du = torch.where(same, one, torch.abs(bins[up][..., None] - t))
        tot = dl + du
        two_hot = (torch.nn.functional.one_hot(lo, nb) * (dl / tot) +
                   torch.nn.functional.one_hot(up, nb) * (du / tot))
        logp = self.logits - torch.logsumexp(self.logits, -1, keepdim=True)
        return -(two_hot * logp).sum(-1, keepdim=True)

    def reshape(self, *shape):
        return SymExpTwoHotDistribution(self.logits.reshape(*shape, self.logits.shape[-1]))
