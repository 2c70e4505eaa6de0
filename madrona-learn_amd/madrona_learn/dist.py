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


class DataParallel:
    def __init__(self, group=None):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world_size = dist.get_world_size(group)
        else:
            self.rank = 0
            self.world_size = 1

    def all_reduce_sum_(self, t: torch.Tensor):
        if self.world_size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def broadcast_(self, t: torch.Tensor, src=0):
        if self.world_size > 1:
            dist.broadcast(t, src=src, group=self.group)
        return t

    def barrier(self):
        if self.world_size > 1:
            dist.barrier(group=self.group)
