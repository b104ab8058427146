// RCCL communicator plumbing for the vertex-range partition across GPUs
// (one process per GPU, ids exchanged by the caller, e.g. torch.distributed).
#include <rccl/rccl.h>

#include <cstring>
#include <map>
#include <mutex>
#include <set>

#include "pfdr_halo.hpp"

namespace pfdr {
int report_rccl(const char *fn, ncclResult_t r);

// Communicators the watchdog aborted.  The handle belongs to the caller
// (pfdr_comm_init made it), so a timed-out session cannot simply free it:
// ncclCommAbort releases the communicator, and the caller's normal clean-up
// (pfdr_comm_destroy in a finally block) must then not destroy it again.
static std::mutex g_aborted_m;
static std::set<void *> g_aborted;
// communicators split from another (Transport::split): aborted with it, so a
// failed rank's abort of its partition's communicators also releases the
// peers waiting on a speculative session's evolution chain
static std::map<void *, std::set<void *>> g_children;

static void abort_locked(void *comm) {
    if (!comm || g_aborted.count(comm)) return;
    auto it = g_children.find(comm);
    if (it != g_children.end()) {
        const std::set<void *> kids = it->second;
        for (void *k : kids) abort_locked(k);
    }
    (void)ncclCommAbort((ncclComm_t)comm);
    g_aborted.insert(comm);
}

void comm_abort(void *comm) {
    std::lock_guard<std::mutex> l(g_aborted_m);
    abort_locked(comm);
}

void comm_add_child(void *parent, void *child) {
    std::lock_guard<std::mutex> l(g_aborted_m);
    g_children[parent].insert(child);
}

void comm_forget_child(void *parent, void *child) {
    std::lock_guard<std::mutex> l(g_aborted_m);
    auto it = g_children.find(parent);
    if (it == g_children.end()) return;
    it->second.erase(child);
    if (it->second.empty()) g_children.erase(it);
}

bool comm_aborted(void *comm) {
    std::lock_guard<std::mutex> l(g_aborted_m);
    return g_aborted.count(comm) != 0;
}

// The split communicator of a parent (Transport::split), kept while the
// parent lives: the sessions a partition runs on one communicator reuse it
// instead of paying a collective ncclCommSplit (own streams and buffers)
// and its teardown per session.  One user at a time: a second live session
// on the same parent gets a split of its own (`busy`).  Released with the
// parent (comm_release_split), or dropped once the watchdog aborted it.
struct SplitEntry {
    void *child;
    bool busy;
};
static std::map<void *, SplitEntry> g_split;

void *comm_split_take(void *parent) {
    std::lock_guard<std::mutex> l(g_aborted_m);
    auto it = g_split.find(parent);
    if (it == g_split.end() || it->second.busy) return nullptr;
    if (g_aborted.count(it->second.child) || g_aborted.count(parent)) return nullptr;
    it->second.busy = true;
    return it->second.child;
}

bool comm_split_keep(void *parent, void *child) {
    std::lock_guard<std::mutex> l(g_aborted_m);
    if (g_split.count(parent)) return false;  // (one kept per parent; this one is the caller's)
    g_split[parent] = SplitEntry{child, true};
    g_children[parent].insert(child);
    return true;
}

void comm_split_return(void *parent, void *child) {
    std::lock_guard<std::mutex> l(g_aborted_m);
    auto it = g_split.find(parent);
    if (it != g_split.end() && it->second.child == child) it->second.busy = false;
}

void comm_release_split(void *parent) {
    void *child = nullptr;
    {
        std::lock_guard<std::mutex> l(g_aborted_m);
        auto it = g_split.find(parent);
        if (it == g_split.end()) return;
        child = it->second.child;
        g_split.erase(it);
        auto k = g_children.find(parent);
        if (k != g_children.end()) {
            k->second.erase(child);
            if (k->second.empty()) g_children.erase(k);
        }
        if (g_aborted.erase(child)) return;  // released by the abort
    }
    (void)ncclCommDestroy((ncclComm_t)child);
}

// a communicator just created at the address of one the watchdog aborted
// (released by ncclCommAbort, its handle never destroyed): the entry is stale
void comm_created(void *comm) {
    std::lock_guard<std::mutex> l(g_aborted_m);
    g_aborted.erase(comm);
}
}  // namespace pfdr

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
    pfdr::comm_created(comm);
    *comm_out = comm;
    return PFDR_OK;
}

extern "C" int pfdr_comm_destroy(void *comm) {
    if (!comm) return PFDR_OK;
    pfdr::comm_release_split(comm);  // (its kept split communicator first)
    {   // aborted by the watchdog: already released, forget the handle
        std::lock_guard<std::mutex> l(pfdr::g_aborted_m);
        if (pfdr::g_aborted.erase(comm)) return PFDR_OK;
    }
    ncclResult_t r = ncclCommDestroy((ncclComm_t)comm);
    if (r != ncclSuccess) return pfdr::report_rccl("pfdr_comm_destroy", r);
    return PFDR_OK;
}

// max-reduce one host double over the ranks (timing: max over ranks)
extern "C" int pfdr_comm_allreduce_max_f64(void *comm, double *value) {
    if (!comm || !value) return pfdr::report_error("pfdr_comm_allreduce_max_f64", "null argument");
    if (pfdr::comm_aborted(comm))
        return pfdr::report_error("pfdr_comm_allreduce_max_f64",
                                  "communicator aborted by the watchdog (PFDR_COMM_TIMEOUT)");
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
