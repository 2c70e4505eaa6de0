"""Data parallelism over environments: one process per GPU.

The reference is single-device.  Here every rank runs the
reference's per-device configuration on its own environment shard
(env ids rank*N .. rank*N+N-1); the only data-path exchanges are
  * the per-minibatch advantage sums (sum x, sum x^2) so that zscore_data
    uses the statistics of the global minibatch, once per epoch, and
  * the flat fp32 gradient (89,883 floats for MLP[256,256]), summed with each
    rank's loss pre-scaled by 1/world, once per minibatch,
both on the compute stream through the C ABI's RCCL communicator
(mlearn_allreduce_f32 / _f64, csrc/comm.hip) when the group runs on the
"nccl" backend (= RCCL over xGMI on MI355X), so a HIP graph captures a whole
update including its collectives; otherwise (the "gloo" backend of the CPU
tests, MLEARN_NATIVE_COLLECTIVES=0, or a failed self-check at setup) via
torch.distributed between captured graph segments.
"""

import ctypes
import os
import sys

import torch
import torch.distributed as dist


def _initialized():
    return dist.is_available() and dist.is_initialized()


_EMULATED_WORLD = 1


def set_emulated_world(w):
    """Benchmark-only (bench.py --emulate-world W, one process, one GPU): the
    next init_training runs rank 0's share of a W-rank job on this GPU, with
    a one-rank RCCL communicator standing in for the group's collectives and
    the loss scaled by 1 / W.  That trains on 1 / W of the gradient, so it is
    an explicit call (never an environment variable that could leak into a
    real run) and is refused when a process group exists.  w = 1 turns it
    off."""
    global _EMULATED_WORLD
    w = int(w)
    if w > 1 and _initialized():
        raise RuntimeError("emulated world: a torch.distributed process group is initialised; "
                           "emulation is for single-process benchmarks only")
    if w > 1:
        import sys
        print(f"madrona_learn: EMULATING rank 0 of a {w}-rank job on one GPU (benchmark "
              f"projection; the update trains on 1/{w} of the gradient)", file=sys.stderr)
    _EMULATED_WORLD = max(w, 1)


def emulated_world():
    """The world size set_emulated_world asked for (1: no emulation)."""
    return _EMULATED_WORLD if _EMULATED_WORLD > 1 and not _initialized() else 1


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

        self.comm = None  # RCCL communicator owned by libmlearn (enable_native)
        self.comm_ranks = 0  # ranks of that communicator
        # how the group's collectives run: "none" (one rank), "rccl_in_graph"
        # (C ABI communicator on the compute stream), "torch_distributed"
        self.collectives = "none" if self.world_size <= 1 else "torch_distributed"
        self.native_reason = None  # why the native path is off (None: on or not needed)

    def _fallback(self, why):
        self.native_reason = why
        if self.world_size > 1:
            print(f"[madrona_learn] rank {self.rank}: RCCL-in-graph collectives off ({why}); "
                  "using torch.distributed between graph segments", file=sys.stderr, flush=True)
        return False

    def enable_native(self, device):
        """Bootstrap this group's RCCL communicator in the C ABI: the group's
        first rank makes the unique id, torch.distributed broadcasts it
        (with that rank's success flag, so no rank calls ncclCommInitRank on
        an id that was never made), every member calls mlearn_comm_init.  A
        sum of rank ids through the new communicator must come out right on
        every rank, else the group keeps the torch.distributed path and says
        why on stderr."""
        if self.world_size <= 1:
            return False
        if os.environ.get("MLEARN_NATIVE_COLLECTIVES", "1") == "0":
            return self._fallback("MLEARN_NATIVE_COLLECTIVES=0")
        if dist.get_backend(self.group) != "nccl":
            return self._fallback(f"backend {dist.get_backend(self.group)}")
        from . import _native as nat
        L = nat.lib()
        idt = torch.zeros(129, dtype=torch.uint8, device=device)  # 128-byte id + ok flag
        if self.rank == 0:
            buf = (ctypes.c_uint8 * 128)()
            made = L.mlearn_comm_unique_id(buf) == 0
            idt[:128].copy_(torch.tensor(list(buf), dtype=torch.uint8))
            idt[128] = 1 if made else 0
        dist.broadcast(idt, src=self.root, group=self.group)
        host = idt.cpu().tolist()
        if host[128] != 1:
            return self._fallback("mlearn_comm_unique_id failed on the group's first rank")
        ids = (ctypes.c_uint8 * 128)(*host[:128])
        comm = ctypes.c_void_p()
        ok = L.mlearn_comm_init(ids, self.world_size, self.rank, ctypes.byref(comm)) == 0
        if ok:
            t = torch.full((4,), float(self.rank + 1), dtype=torch.float32, device=device)
            ok = L.mlearn_allreduce_f32(comm, nat.ptr(t), 4, nat.stream_handle()) == 0
            torch.cuda.synchronize()
            W = self.world_size
            ok = ok and bool((t == W * (W + 1) / 2).all().item())
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) != 1:
            if comm.value:
                L.mlearn_comm_destroy(comm)
            return self._fallback("communicator init or self-check failed on "
                                  + ("this rank" if not ok else "another rank"))
        self.comm = comm
        self.comm_ranks = self.world_size
        self.collectives = "rccl_in_graph"
        return True

    def all_reduce_sum_(self, t: torch.Tensor):
        if self.world_size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def native_all_reduce_sum_(self, t: torch.Tensor):
        """In-place sum over the group, enqueued on the current stream by the
        C ABI (captured into the update's HIP graph)."""
        from . import _native as nat
        L = nat.lib()
        f = L.mlearn_allreduce_f64 if t.dtype == torch.float64 else L.mlearn_allreduce_f32
        nat.check(f(self.comm, nat.ptr(t), t.numel(), nat.stream_handle()), "allreduce")
        return t

    def broadcast_(self, t: torch.Tensor):
        if self.world_size > 1:
            dist.broadcast(t, src=self.root, group=self.group)
        return t

    def barrier(self):
        if self.world_size > 1:
            dist.barrier(group=self.group)


class EmulatedDataParallel(DataParallel):
    """Rank 0 of a W-rank data-parallel group, alone on one GPU (bench.py
    --emulate-world W): the shard, minibatch slices and per-minibatch
    collectives of that rank, each collective a real RCCL all-reduce on a
    one-rank communicator (same launch, in the same graph position; the
    xGMI transfer of the W-rank ring is what it leaves out)."""

    def __init__(self, world_size):
        super().__init__(solo=True)
        self.world_size = int(world_size)
        self.collectives = "rccl_in_graph (1-rank emulation)"

    def enable_native(self, device):
        from . import _native as nat
        L = nat.lib()
        buf = (ctypes.c_uint8 * 128)()
        comm = ctypes.c_void_p()
        if L.mlearn_comm_unique_id(buf) != 0 or L.mlearn_comm_init(buf, 1, 0,
                                                                   ctypes.byref(comm)) != 0:
            raise RuntimeError("emulated world: one-rank RCCL communicator failed: "
                               + L.mlearn_last_error().decode(errors="replace"))
        self.comm = comm
        self.comm_ranks = 1
        return True

    def all_reduce_sum_(self, t):
        return t

    def broadcast_(self, t):
        return t

    def barrier(self):
        pass


def world():
    """(global rank, world size) of this process."""
    if _initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, emulated_world()


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
    if P > 1 and emulated_world() > 1:
        raise ValueError("emulated world (set_emulated_world): populations are not emulated; "
                         "run a real process group")
    if P == 1:
        ew = emulated_world()
        return [0], (EmulatedDataParallel(ew) if ew > 1 else DataParallel())
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
