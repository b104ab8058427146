// 1-D vertex-range partition of a PFDR graph across ranks (one GPU each),
// SURVEY.md §8(e):
//
//   rank r owns the global vertices [off[r], off[r+1]) and the edges it was
//   handed (normally those whose Eu it owns).  Per iteration:
//     pull  : owners send (X, P) of their boundary vertices to the ranks that
//             hold edges touching them (ghost copies), before the edge sweep;
//     push  : each rank sends the DR contributions W*Z of edge ends whose
//             vertex it does not own to that vertex's owner, after the edge
//             sweep; the owner sums them in GLOBAL edge order, exactly where
//             the single-GPU (and reference) summation puts them;
//     reduce: iterate-evolution / objective partials (2-3 scalars).
//   The preconditioner's amplitude c is a sequential sum in global vertex
//   order, carried rank to rank (chain), so every rank gets the single-GPU c.
//
// Transport = RCCL (one process per GPU, grouped ncclSend/ncclRecv over
// xGMI) or Loopback (k ranks as k host threads on one device, exchanges as
// device-to-device copies) — the latter lets the whole partitioned path be
// tested on one GPU against the unpartitioned solver.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "pfdr_graph.hpp"
#include "pfdr_monosum.hpp"

namespace pfdr {

class Transport {
  public:
    int nranks = 1, rank = 0;
    // watchdog context: what the session is doing (set by the sessions) and
    // the last collective enqueued (set by the transports); a stall longer
    // than timeout_s (PFDR_COMM_TIMEOUT, default 120 s) is reported with
    // them and fails the call instead of hanging
    const char *phase = "setup";
    long iteration = 0;
    std::string last_op = "none";
    double timeout_s = comm_timeout_s();
    static double comm_timeout_s();
    std::string describe() const;
    virtual ~Transport() = default;
    // wait for stream s (instead of hipStreamSynchronize) under the watchdog
    virtual void wait(hipStream_t s);
    virtual void on_timeout() {}
    // the transport's per-iteration operations can be captured in a hipGraph
    // (RCCL: yes, captured sends / receives / all-reduces replay on the
    // communicator; loopback: no, its exchanges rendezvous on the host)
    virtual bool capturable() const { return false; }
    // point-to-point exchange with every peer (entries for this rank and
    // zero sizes are skipped); enqueued on s
    virtual void exchange(const std::vector<const void *> &send,
                          const std::vector<size_t> &sbytes,
                          const std::vector<void *> &recv,
                          const std::vector<size_t> &rbytes, hipStream_t s) = 0;
    // in-place sum over ranks of n values of dtype (PFDR_F32 / PFDR_F64) or
    // int64 (dtype = 2), device memory
    virtual void allreduce_sum(void *dev, int n, int dtype, hipStream_t s) = 0;
    // receive `bytes` from rank-1 into dev (rank 0: nothing)
    virtual void chain_recv(void *dev, size_t bytes, hipStream_t s) = 0;
    // send `bytes` from dev to rank+1 (last rank: nothing)
    virtual void chain_send(const void *dev, size_t bytes, hipStream_t s) = 0;
    virtual void broadcast(void *dev, size_t bytes, int root, hipStream_t s) = 0;
    // host-level allgather of one int64 per rank (setup only)
    void allgather_i64(int64_t mine, std::vector<int64_t> &all, hipStream_t s);
    // variable-size all-to-all of host arrays (setup only)
    void alltoallv_host(const std::vector<std::vector<int64_t>> &send,
                        std::vector<std::vector<int64_t>> &recv, hipStream_t s);
};

std::unique_ptr<Transport> make_rccl_transport(void *comm, int nranks, int rank);
// watchdog abort of a caller-owned communicator (pfdr_comm.hip): aborted
// once, remembered so that pfdr_comm_destroy does not free it a second time
void comm_abort(void *comm);
bool comm_aborted(void *comm);
std::unique_ptr<Transport> make_loopback_transport(void *hub, int nranks, int rank);
// wake every rank waiting on the hub with an error (a rank failed)
void loopback_abort(void *hub, const char *reason);

// Partition plan of one rank plus its device-side exchange buffers.
struct Halo {
    std::unique_ptr<Transport> tr;
    int V = 0;              // owned vertices (local ids [0, V))
    int G = 0;              // ghost vertices (local ids [V, V + G)), grouped by owner
    long E = 0;             // local edges
    int64_t vtx_begin = 0;
    std::vector<int64_t> off;          // nranks + 1 global vertex offsets
    // pull: (X, P) of owned vertices to peers / into the ghost range
    std::vector<int> pull_send_cnt, pull_send_off;  // per peer, into pull_idx
    std::vector<int> ghost_cnt, ghost_off;          // per peer, into [V, V + G)
    DevBuf<int> pull_idx;                           // owned local ids to send
    // push: contributions of ghost-vertex slots to their owners
    std::vector<int> push_send_cnt, push_send_off;  // per peer, into push_addr
    std::vector<int> push_recv_cnt, push_recv_off;  // per peer, into the tail
    long R = 0;                                     // received contributions
    DevBuf<unsigned> push_addr;                     // local contribution addresses
    // CSR keys of the received slots: (owned local vertex, 2 e_global + side)
    DevBuf<unsigned long long> recv_keys;
    // scratch send buffer (bytes)
    DevBuf<char> sendbuf;

    // gather elem-sized values at idx into sendbuf, exchange, land the
    // peers' values in base + V (ghost range) — base holds Vg elements
    void pull(void *base, int elem_bytes, hipStream_t s);
    // contributions: gather wz[push_addr] (elem_bytes each) and land the
    // peers' in tail
    void push(const void *wz, void *tail, int elem_bytes, hipStream_t s);
    // the same exchange for contributions already packed in push_addr order
    // (the caller formed them, e.g. the simplex's K-wide W*Z)
    void push_packed(const void *packed, void *tail, int elem_bytes, hipStream_t s);
    // scratch buffer for push_packed of n elements
    void *push_buffer(int elem_bytes);
};

// Host-only planning (no device needed; also exported through the C ABI so
// the partition logic is testable on CPU with any transport).
struct PlanHost {
    int nranks = 1, rank = 0, V = 0;
    long E = 0;
    int64_t lo = 0, hi = 0;
    std::vector<int64_t> off;                 // nranks + 1
    std::vector<int64_t> ghosts;              // sorted global ids
    std::vector<int> ghost_cnt, ghost_off;
    std::vector<int> Eu_l, Ev_l;              // rank-local endpoint ids
    std::vector<std::vector<int64_t>> req;    // pull requests to each owner (global ids)
    std::vector<std::vector<int64_t>> items;  // push items to each owner: (g, 2 eg + side) pairs
    std::vector<std::vector<unsigned>> addr;  // my contribution address of each item
    // filled by plan_finish
    std::vector<int> pull_idx, pull_send_cnt, pull_send_off;
    std::vector<unsigned> push_addr;
    std::vector<int> push_send_cnt, push_send_off, push_recv_cnt, push_recv_off;
    std::vector<unsigned long long> recv_keys;
};
void plan_local(PlanHost &p, int nranks, int rank, const int64_t *off, long E, const int *Eu_g,
                const int *Ev_g, const int64_t *e_global, int64_t e_offset);
// inreq[q] / initems[q]: what peer q sent us (its req[rank] / items[rank])
void plan_finish(PlanHost &p, const std::vector<std::vector<int64_t>> &inreq,
                 const std::vector<std::vector<int64_t>> &initems);

// Build the plan of this rank from its local edges (global endpoint ids and
// global edge ids, host arrays), exchanging request lists with the peers.
// Writes the rank-local endpoint ids (owned [0, V), ghosts [V, V + G)).
void build_halo(Halo &h, int V, int64_t vtx_begin, long E, const int *Eu_g,
                const int *Ev_g, const int64_t *e_global, int64_t e_offset,
                std::vector<int> &Eu_l, std::vector<int> &Ev_l, hipStream_t s);

// Partitioned session setup (both solvers): the transport from p->comm, the
// plan of this rank from its global edges (host planner + exchanges), and
// the rank-local endpoint ids in Eu / Ev (device, E each; owned [0, V),
// ghosts [V, V + G)).  Global edge ids: eg (device, 32-bit) when
// p->e_global is given, else *e_offset = p->e_offset.
void partition_setup(const pfdr_problem *p, int V, long E, std::unique_ptr<Halo> &halo,
                     DevBuf<int> &Eu, DevBuf<int> &Ev, DevBuf<unsigned> &eg, long *e_offset,
                     hipStream_t s);

// Collective check (setup): the caller's labels of every rank's owned
// vertices (vtx_label, device, V per rank) form a permutation of
// [0, V_global); throws otherwise.
void check_permutation(const int *lab, int V, long Vglob, Transport &tr, hipStream_t s);

// Contribution CSR of both solvers: the 2E local slots (address e = u end,
// E + e = v end) keyed by (local vertex, 2 e_global + side) — the
// reference's summation order — then the halo's received tail (addresses
// 2E + j, keys from the plan).  eg: global edge ids or NULL (e_offset + e).
void contribution_incidence(const int *Eu, const int *Ev, long E, int V, const unsigned *eg,
                            long e_offset, const Halo *halo, Incidence &inc, hipStream_t s);

// Iterate-evolution sums of a partition with the reference's sequential
// rounding (src/PFDR_graph_quadratic_d1_l1.cpp:514-529, simplex
// src/PFDR_graph_loss_d1_simplex.cpp:653-691): nsum sums whose terms lie on
// the ranks in rank order (rank r holds its n terms of sum y at a + y *
// astride, the caller's order continuing rank to rank).  The binade scan of
// pfdr_monosum.hpp splits cleanly at the ranks: each rank summarises its
// tiles in parallel on binades predicted from the f64 totals of the ranks
// before it (one all-reduce of nranks * nsum doubles), then the exact
// running sum is carried rank to rank through the walks (chain_recv ->
// k_mono_walk -> chain_send) and the last rank broadcasts it -- every rank
// gets the single-GPU value bit for bit.  The rank-to-rank part is one
// walk per rank (~1/N of the single-GPU walk) plus N point-to-point hops.
template <typename real>
struct ChainSum {
    long n = 0;
    int nsum = 1, nranks = 1, rank = 0;
    DevBuf<char> ws;
    DevBuf<double> tot;
    DevBuf<real> seed;
    void init(long n_, int nsum_, const Transport &tr) {
        n = n_; nsum = nsum_; nranks = tr.nranks; rank = tr.rank;
        ws.alloc(mono_ws_bytes<real>(n, nsum));
        tot.alloc((size_t)nranks * nsum);
        seed.alloc(nsum);
    }
    bool ready() const { return ws.p != nullptr; }
    // out[0 .. nsum): the whole sums, on every rank (device); halt as mono_sum
    void run(Transport &tr, const real *a, long astride, real *out, const int *halt,
             hipStream_t s) {
        constexpr long TILE = MonoTile<real>::TILE;
        const long nt = (n + TILE - 1) / TILE;
        const MonoWs<real> w(ws.p, nt, nsum);
        double *tsum = w.tsum;
        int *ebase = w.ebase;
        const dim3 gt((unsigned)nt, (unsigned)nsum), g1(1, (unsigned)nsum);
        k_mono_tile_sums<real><<<gt, 256, 0, s>>>(n, a, astride, tsum, halt);
        PFDR_HIP(hipMemsetAsync(tot.p, 0, sizeof(double) * nranks * nsum, s));
        k_mono_total<<<g1, 256, 0, s>>>((int)nt, tsum, tot.p + (size_t)rank * nsum, halt);
        PFDR_HIP(hipGetLastError());
        tr.allreduce_sum(tot.p, nranks * nsum, PFDR_F64, s);
        k_mono_predict<real><<<g1, kPredThreads, 0, s>>>((int)nt, tsum, nullptr, 0, ebase, halt,
                                                         tot.p, rank);
        k_mono_summaries<real><<<gt, kMonoThreads, 0, s>>>(n, a, astride, ebase, w.summ, w.subs,
                                                           halt);
        PFDR_HIP(hipGetLastError());
        tr.chain_recv(seed.p, sizeof(real) * nsum, s);
        k_mono_walk<real><<<g1, kMonoThreads, 0, s>>>(n, a, astride, (int)nt, ebase, w.summ,
                                                      w.subs, rank > 0 ? seed.p : nullptr, 1, 0,
                                                      nullptr, out, nullptr, halt);
        PFDR_HIP(hipGetLastError());
        tr.chain_send(out, sizeof(real) * nsum, s);
        tr.broadcast(out, sizeof(real) * nsum, nranks - 1, s);
    }
};

}  // namespace pfdr
