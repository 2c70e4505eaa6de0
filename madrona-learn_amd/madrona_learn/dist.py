"""Data parallelism over environments: one process per GPU.

The reference is single-device.  Here every rank runs the
reference's per-device configuration on its own environment shard
(env ids rank*N .. rank*N+N-1); the only data-path exchanges are
  * the per-minibatch advantage sums (sum x, sum x^2) so that zscore_data
    uses the statistics of the global minibatch, once per epoch, and
  * the flat fp32 gradient (89,883 floats for MLP[256,256]), summed with each
    rank's loss pre-scaled by 1/world, once per minibatch,
both via torch.distributed (backend "nccl" = RCCL over xGMI on MI355X, "gloo"
on CPU for tests).
"""

import torch
import torch.distributed as dist


def _initialized():
    return dist.is_available() and dist.is_initialized()


class DataParallel:
    """One data-parallel group: the ranks that train one policy.  ``root`` is
    the global rank of the group's first member (broadcast source)."""

    def __init__(self, group=None, root=0, solo=False):
        self.group = group
        self.root = root
        if solo or not _initialized():
            self.rank = 0
            self.world_size = 1
        else:
            self.rank = dist.get_rank(group)
            self.world_size = dist.get_world_size(group)

    def all_reduce_sum_(self, t: torch.Tensor):
        if self.world_size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def broadcast_(self, t: torch.Tensor):
        if self.world_size > 1:
            dist.broadcast(t, src=self.root, group=self.group)
        return t

    def barrier(self):
        if self.world_size > 1:
            dist.barrier(group=self.group)


def world():
    """(global rank, world size) of this process."""
    if _initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def policy_placement(num_policies):
    """Place a population of ``num_policies`` train policies on the ranks.

    * world % P == 0: policy p is trained by the G = world/P ranks
      [p*G, (p+1)*G) as one data-parallel group (gradient all-reduce inside
      the group only); each of those ranks holds that one policy.
    * P % world == 0: each rank holds P/world whole policies, each trained
      on that rank alone (no collectives): config P of SURVEY §8(d), one
      policy per GPU, is P == world.
    Returns (global ids of this rank's policies, DataParallel of their group).
    Every rank calls this in the same order (new_group is collective)."""
    rank, W = world()
    P = int(num_policies)
    if P == 1:
        return [0], DataParallel()
    if W % P == 0:
        G = W // P
        groups = [dist.new_group(list(range(p * G, (p + 1) * G))) for p in range(P)] \
            if G > 1 else [None] * P
        pid = rank // G
        if G == 1:
            return [pid], DataParallel(solo=True, root=rank)
        return [pid], DataParallel(groups[pid], root=pid * G)
    if P % W == 0:
        per = P // W
        return list(range(rank * per, (rank + 1) * per)), DataParallel(solo=True, root=rank)
    raise ValueError(f"{P} policies cannot be placed on {W} ranks (need P % world == 0 or "
                     "world % P == 0)")
