// Data-parallel collectives issued on the compute stream (SURVEY §8(b),
// §8(e)): an RCCL communicator owned by the C ABI, so the per-minibatch
// gradient all-reduce (and the per-epoch advantage-sum all-reduce) are
// ordinary stream work that a HIP graph captures with the kernels around
// them — one graph per update instead of a host round trip per minibatch.
// The communicator is bootstrapped with a unique id the caller distributes
// (madrona_learn.dist: torch.distributed broadcast); RCCL runs over xGMI
// between the GPUs of a node.  At runtime this binds the RCCL the process
// already has loaded (soname librccl.so.1; PyTorch-ROCm's copy under torch).

#include <rccl/rccl.h>

#include <cstring>

#include "common.h"

using namespace ml;

static_assert(MLEARN_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "RCCL unique id size");

#define ML_NCCL(call, what)                                                               \
    do {                                                                                  \
        ncclResult_t r_ = (call);                                                         \
        ML_REQUIRE(r_ == ncclSuccess, "%s: %s", what, ncclGetErrorString(r_));            \
    } while (0)

extern "C" {

int mlearn_comm_unique_id(uint8_t* id_out) {
    ML_REQUIRE(id_out, "comm_unique_id: null output");
    ncclUniqueId id;
    ML_NCCL(ncclGetUniqueId(&id), "ncclGetUniqueId");
    memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return MLEARN_OK;
}

int mlearn_comm_init(const uint8_t* id, int32_t nranks, int32_t rank, mlearn_comm_t* comm_out) {
    ML_REQUIRE(id && comm_out, "comm_init: null pointer");
    ML_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "comm_init: rank %d of %d", rank,
               nranks);
    ncclUniqueId uid;
    memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t c = nullptr;
    ML_NCCL(ncclCommInitRank(&c, nranks, uid, rank), "ncclCommInitRank");
    *comm_out = (mlearn_comm_t)c;
    return MLEARN_OK;
}

int mlearn_comm_destroy(mlearn_comm_t comm) {
    if (!comm) return MLEARN_OK;
    ML_NCCL(ncclCommDestroy((ncclComm_t)comm), "ncclCommDestroy");
    return MLEARN_OK;
}

static int allreduce(mlearn_comm_t comm, void* buf, int64_t n, ncclDataType_t t,
                     mlearn_stream_t stream, const char* what) {
    ML_REQUIRE(comm, "%s: null communicator", what);
    ML_REQUIRE(n >= 0, "%s: n < 0", what);
    if (n == 0) return MLEARN_OK;
    ML_REQUIRE(buf, "%s: null buffer", what);
    ML_NCCL(ncclAllReduce(buf, buf, (size_t)n, t, ncclSum, (ncclComm_t)comm, S(stream)), what);
    return MLEARN_OK;
}

int mlearn_allreduce_f32(mlearn_comm_t comm, float* buf, int64_t n, mlearn_stream_t stream) {
    return allreduce(comm, buf, n, ncclFloat32, stream, "allreduce_f32");
}

int mlearn_allreduce_f64(mlearn_comm_t comm, double* buf, int64_t n, mlearn_stream_t stream) {
    return allreduce(comm, buf, n, ncclFloat64, stream, "allreduce_f64");
}

}  // extern "C"
