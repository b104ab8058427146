// RCCL communicator plumbing for the vertex-range partition across GPUs
// (one process per GPU, ids exchanged by the caller, e.g. torch.distributed).
#include <rccl/rccl.h>

#include <cstring>

#include "pfdr_dev.hpp"

namespace pfdr {
int report_rccl(const char *fn, ncclResult_t r);
}

int pfdr::report_rccl(const char *fn, ncclResult_t r) {
    char msg[256];
    snprintf(msg, sizeof msg, "RCCL error %d (%s)", (int)r, ncclGetErrorString(r));
    report_error(fn, msg);
    return PFDR_ERR_RCCL;
}

static_assert(PFDR_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "id size");

extern "C" int pfdr_comm_unique_id(void *id_out) {
    if (!id_out) return pfdr::report_error("pfdr_comm_unique_id", "null argument");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return pfdr::report_rccl("pfdr_comm_unique_id", r);
    memcpy(id_out, &id, sizeof id);
    return PFDR_OK;
}

extern "C" int pfdr_comm_init(void **comm_out, int nranks, int rank, const void *id_in) {
    if (!comm_out || !id_in || nranks < 1 || rank < 0 || rank >= nranks)
        return pfdr::report_error("pfdr_comm_init", "invalid arguments");
    ncclUniqueId id;
    memcpy(&id, id_in, sizeof id);
    ncclComm_t comm;
    ncclResult_t r = ncclCommInitRank(&comm, nranks, id, rank);
    if (r != ncclSuccess) return pfdr::report_rccl("pfdr_comm_init", r);
    *comm_out = comm;
    return PFDR_OK;
}

extern "C" int pfdr_comm_destroy(void *comm) {
    if (!comm) return PFDR_OK;
    ncclResult_t r = ncclCommDestroy((ncclComm_t)comm);
    if (r != ncclSuccess) return pfdr::report_rccl("pfdr_comm_destroy", r);
    return PFDR_OK;
}

// max-reduce one host double over the ranks (timing: max over ranks)
extern "C" int pfdr_comm_allreduce_max_f64(void *comm, double *value) {
    if (!comm || !value) return pfdr::report_error("pfdr_comm_allreduce_max_f64", "null argument");
    try {
        hipStream_t s = pfdr::lib_stream();
        pfdr::DevBuf<double> d(1);
        PFDR_HIP(hipMemcpyAsync(d.p, value, sizeof(double), hipMemcpyHostToDevice, s));
        ncclResult_t r = ncclAllReduce(d.p, d.p, 1, ncclDouble, ncclMax, (ncclComm_t)comm, s);
        if (r != ncclSuccess) return pfdr::report_rccl("pfdr_comm_allreduce_max_f64", r);
        PFDR_HIP(hipMemcpyAsync(value, d.p, sizeof(double), hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
    } catch (const pfdr::HipError &h) {
        return pfdr::report_error("pfdr_comm_allreduce_max_f64", h);
    }
    return PFDR_OK;
}
