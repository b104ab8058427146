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
#include <algorithm>
#include <memory>
#include <stdexcept>
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
    // a second transport over the same ranks whose operations may run
    // CONCURRENTLY with this one's, on another stream (a speculative
    // session's evolution sums beside the next iteration's halo exchanges).
    // RCCL: its own communicator (ncclCommSplit; collective, setup only),
    // aborted with this one by the watchdog; loopback: the same hub (its
    // exchanges are serialised by the host threads anyway)
    virtual std::unique_ptr<Transport> split(hipStream_t s) = 0;
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
void comm_created(void *comm);  // forget a stale aborted entry at this address
// a communicator split from `parent`: comm_abort(parent) aborts it first;
// forget it before destroying it
void comm_add_child(void *parent, void *child);
void comm_forget_child(void *parent, void *child);
// the split communicator kept with `parent` (pfdr_comm.hip): take it if kept
// and free (null otherwise), keep a new one (false: one is kept already, the
// caller owns this one), give it back, release it with the parent
void *comm_split_take(void *parent);
bool comm_split_keep(void *parent, void *child);
void comm_split_return(void *parent, void *child);
void comm_release_split(void *parent);
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

// item j of the route: its W terms of every sum into the send buffer (items
// grouped by destination), and back out of the receive buffer at its slot
template <typename real>
__global__ void k_route_pack(long n, int W, int nsum, const int *__restrict__ sidx,
                             const real *__restrict__ terms, long tstride,
                             real *__restrict__ buf) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * W) return;
    const long j = t / W;
    const int w = (int)(t - j * W);
    const long v = sidx[j];
    for (int y = 0; y < nsum; y++) buf[(j * nsum + y) * W + w] = terms[y * tstride + v * W + w];
}
template <typename real>
__global__ void k_route_unpack(long n, int W, int nsum, const int *__restrict__ rpos,
                               const real *__restrict__ buf, real *__restrict__ slice,
                               long sstride) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * W) return;
    const long j = t / W;
    const int w = (int)(t - j * W);
    const long p = rpos[j];
    for (int y = 0; y < nsum; y++) slice[y * sstride + p * W + w] = buf[(j * nsum + y) * W + w];
}

// Iterate-evolution sums of a RELABELLED partition (the ranks own ranges of
// internal labels, while the reference sums in the caller's order).  The
// caller's order is cut into contiguous slices, slice q = caller labels
// [Vg q / N, Vg (q + 1) / N) on rank q; every owned vertex's W terms of each
// sum travel, at positions fixed at setup, to the rank whose slice holds its
// caller label -- one variable all-to-all of ~V/N items per rank per tracked
// iteration, the vertex's own rank included when its label falls there -- and
// ChainSum then runs over the slices in rank order, which IS the caller's
// order: Dif bit-identical to one GPU, with O(V/N) bytes per rank on the
// wire instead of an all-reduce of the whole V_global term vector.
template <typename real>
struct TermRoute {
    int nsum = 1, W = 1, nranks = 1, rank = 0;
    long nsend = 0, nrecv = 0, S = 0, sstride = 0;
    std::vector<long> soff, roff;  // per peer, in items (nranks + 1)
    DevBuf<int> sidx, rpos;
    DevBuf<real> sbuf, rbuf, slice;
    ChainSum<real> chain;
    bool ready() const { return chain.ready(); }
    // lab: caller labels of the V owned vertices (host), a permutation of
    // [0, Vglob) over the ranks
    void init(const std::vector<int> &lab, long Vglob, int nsum_, int W_, Transport &tr,
              hipStream_t s) {
        nsum = nsum_; W = W_; nranks = tr.nranks; rank = tr.rank;
        const int n = nranks;
        std::vector<int64_t> coff(n + 1);
        for (int q = 0; q <= n; q++) coff[q] = Vglob * q / n;
        S = coff[rank + 1] - coff[rank];
        auto owner = [&](int64_t g) {
            return (int)(std::upper_bound(coff.begin(), coff.end(), g) - coff.begin()) - 1;
        };
        std::vector<std::vector<int64_t>> pos(n), got;
        std::vector<std::vector<int>> items(n);
        for (size_t v = 0; v < lab.size(); v++) {
            const int q = owner(lab[v]);
            items[q].push_back((int)v);
            pos[q].push_back(lab[v] - coff[q]);
        }
        tr.alltoallv_host(pos, got, s);
        soff.assign(n + 1, 0);
        roff.assign(n + 1, 0);
        std::vector<int> hs, hr;
        for (int q = 0; q < n; q++) {
            soff[q + 1] = soff[q] + (long)items[q].size();
            roff[q + 1] = roff[q] + (long)got[q].size();
            hs.insert(hs.end(), items[q].begin(), items[q].end());
            for (int64_t p : got[q]) hr.push_back((int)p);
        }
        nsend = soff[n];
        nrecv = roff[n];
        if (nrecv != S) throw std::runtime_error("vtx_label is not a permutation of [0, V_global)");
        sidx.alloc(nsend ? nsend : 1);
        rpos.alloc(nrecv ? nrecv : 1);
        if (nsend) PFDR_HIP(hipMemcpy(sidx.p, hs.data(), sizeof(int) * nsend, hipMemcpyHostToDevice));
        if (nrecv) PFDR_HIP(hipMemcpy(rpos.p, hr.data(), sizeof(int) * nrecv, hipMemcpyHostToDevice));
        sbuf.alloc((size_t)(nsend ? nsend : 1) * nsum * W);
        rbuf.alloc((size_t)(nrecv ? nrecv : 1) * nsum * W);
        sstride = (S * W + 3) / 4 * 4;
        slice.alloc((size_t)(sstride ? sstride : 4) * nsum);
        chain.init(S * W, nsum, tr);
    }
    // terms: W per owned vertex of every sum (sum y at y * tstride); out[0 ..
    // nsum) the whole sums on every rank, as ChainSum::run
    void run(Transport &tr, const real *terms, long tstride, real *out, const int *halt,
             hipStream_t s) {
        const int n = nranks;
        if (nsend) {
            k_route_pack<real><<<grid_for(nsend * W), kBlock, 0, s>>>(nsend, W, nsum, sidx.p, terms,
                                                                    tstride, sbuf.p);
            PFDR_HIP(hipGetLastError());
        }
        const size_t ib = sizeof(real) * nsum * W;  // bytes per item
        std::vector<const void *> sp(n);
        std::vector<void *> rp(n);
        std::vector<size_t> sb(n), rb(n);
        for (int q = 0; q < n; q++) {
            sp[q] = (const char *)sbuf.p + soff[q] * ib;
            sb[q] = (size_t)(soff[q + 1] - soff[q]) * ib;
            rp[q] = (char *)rbuf.p + roff[q] * ib;
            rb[q] = (size_t)(roff[q + 1] - roff[q]) * ib;
        }
        tr.exchange(sp, sb, rp, rb, s);  // (skips this rank's own part)
        if (rb[rank])
            PFDR_HIP(hipMemcpyAsync(rp[rank], sp[rank], rb[rank], hipMemcpyDeviceToDevice, s));
        if (nrecv) {
            k_route_unpack<real><<<grid_for(nrecv * W), kBlock, 0, s>>>(nrecv, W, nsum, rpos.p,
                                                                      rbuf.p, slice.p, sstride);
            PFDR_HIP(hipGetLastError());
        }
        chain.run(tr, slice.p, sstride, out, halt, s);
    }
};

}  // namespace pfdr
