"""The C ABI's RCCL collectives (csrc/comm.hip): communicator bootstrap from
a unique id, in-place f32 / f64 sums on the compute stream, and capture into
a HIP graph (the data-parallel update runs as one graph with its
collectives).  One GPU on the test box: a one-rank communicator (the
multi-rank semantics are covered by the gloo tests of the same program,
tests/test_dp_gloo.py, tests/test_gpu_dp.py)."""

import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _comm():
    from madrona_learn import _native as nat
    L = nat.lib()
    uid = (ctypes.c_uint8 * 128)()
    nat.check(L.mlearn_comm_unique_id(uid), "unique id")
    comm = ctypes.c_void_p()
    nat.check(L.mlearn_comm_init(uid, 1, 0, ctypes.byref(comm)), "comm init")
    assert comm.value
    return L, comm


def test_allreduce_eager_and_captured(gpu):
    from madrona_learn import _native as nat
    L, comm = _comm()
    try:
        x = torch.arange(1000, dtype=torch.float32, device=gpu)
        y = torch.arange(10, dtype=torch.float64, device=gpu) * 0.5
        x0, y0 = x.clone(), y.clone()
        nat.check(L.mlearn_allreduce_f32(comm, nat.ptr(x), x.numel(), nat.stream_handle()), "f32")
        nat.check(L.mlearn_allreduce_f64(comm, nat.ptr(y), y.numel(), nat.stream_handle()), "f64")
        torch.cuda.synchronize()
        assert torch.equal(x, x0) and torch.equal(y, y0)  # sum over one rank
        # captured: a kernel, the collective, a kernel -> one graph
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                x.mul_(2.0)
                nat.check(L.mlearn_allreduce_f32(comm, nat.ptr(x), x.numel(),
                                                 nat.stream_handle(s)), "captured f32")
                x.add_(1.0)
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        want = x0
        for _ in range(3):
            want = want * 2.0 + 1.0
        assert torch.equal(x, want)
        # error path: a null communicator fails loudly
        assert L.mlearn_allreduce_f32(None, nat.ptr(x), 4, nat.stream_handle()) != 0
    finally:
        nat.check(L.mlearn_comm_destroy(comm), "destroy")
