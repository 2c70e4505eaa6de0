"""Population placement over ranks (madrona_learn/dist.py policy_placement)
on world_size 4 over gloo (CPU): which train policies each rank holds and
which ranks share gradients.  P == world is config P of SURVEY §8(d) (one
policy per GPU, no collectives); world % P == 0 gives each policy a
data-parallel group whose all-reduce must stay inside the group."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from madrona_learn.dist import policy_placement
        res = {}
        for P in (1, 2, 4, 8):
            ids, dp = policy_placement(P)
            t = torch.tensor([float(rank + 1)])
            dp.all_reduce_sum_(t)
            b = torch.tensor([float(rank + 100)])
            dp.broadcast_(b)
            res[P] = (ids, dp.rank, dp.world_size, dp.root, float(t), float(b))
        with pytest.raises(ValueError):
            policy_placement(3)
        # the native (RCCL-in-graph) path is off on gloo, and says why
        _, dp = policy_placement(1)
        res["native"] = (dp.enable_native(torch.device("cpu")), dp.collectives, dp.native_reason,
                         dp.comm_ranks)
        torch.save(res, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_policy_placement_world4(tmp_path):
    mp.spawn(worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=False)
           for r in range(WORLD)]
    for r in range(WORLD):
        # P = 1: plain data parallelism over all ranks
        assert res[r][1] == ([0], r, 4, 0, 10.0, 100.0)
        # P = 2: policy r//2 on the group {2p, 2p+1}; sums stay inside the group
        g = r // 2
        assert res[r][2] == ([g], r % 2, 2, 2 * g, float((2 * g + 1) + (2 * g + 2)),
                             float(2 * g + 100))
        # P = 4: one policy per rank, no exchange
        assert res[r][4] == ([r], 0, 1, r, float(r + 1), float(r + 100))
        # P = 8: two whole policies per rank
        assert res[r][8] == ([2 * r, 2 * r + 1], 0, 1, r, float(r + 1), float(r + 100))
        assert res[r]["native"] == (False, "torch_distributed", "backend gloo", 0)
