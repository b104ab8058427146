// Session (host orchestration) of the MI355X quadratic PFDR solvers
// (reference src/PFDR_graph_quadratic_d1_l1.cpp:270-553,
//  src/PFDR_graph_quadratic_d1_bounds.cpp:244-530), single GPU or one rank
// of a 1-D vertex-range partition (pfdr_halo.hpp).  Kernels: see
// pfdr_quadratic_kernels.hpp.
#include <cstring>
#include <map>
#include <stdexcept>


#include "pfdr_halo.hpp"
#include "pfdr_order.hpp"
#include "pfdr_quadratic_kernels.hpp"
#include "pfdr_sort.hpp"

namespace pfdr {

template <typename real>
static void copy_in(DevBuf<real> &d, const void *src, size_t n, int mem, hipStream_t s,
                    HostPins &pins) {
    if (!src || !n) { d.release(); return; }
    d.alloc(n);
    if (mem == PFDR_MEM_DEVICE)
        PFDR_HIP(hipMemcpyAsync(d.p, src, n * sizeof(real), hipMemcpyDeviceToDevice, s));
    else
        pins.copy(d.p, src, n * sizeof(real), hipMemcpyHostToDevice);
}

template <typename real>
static int dtype_of() { return sizeof(real) == 4 ? PFDR_F32 : PFDR_F64; }


// d <- d[map] (map[i] = source index of element i)
template <typename T>
static void permute(DevBuf<T> &d, const int *map, size_t n, hipStream_t s) {
    if (!d.p || !n) return;
    DevBuf<T> t(n);
    k_gather<T><<<grid_for(n), kBlock, 0, s>>>((long)n, d.p, map, t.p);
    PFDR_HIP(hipGetLastError());
    std::swap(d.p, t.p);
    std::swap(d.n, t.n);
}

// edges sorted by their new u end (stable in the edge id): eorig[p] = the
// original id of the edge now at position p; endpoints relabelled by where
__global__ void k_edge_order_keys(long E, const int *__restrict__ Eu, const int *__restrict__ where,
                                  unsigned long long *__restrict__ keys, unsigned *__restrict__ vals) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    keys[e] = ((unsigned long long)where[Eu[e]] << 32) | (unsigned)e;
    vals[e] = (unsigned)e;
}

__global__ void k_edge_relabel(long E, const unsigned *__restrict__ eorig,
                               const int *__restrict__ Eu, const int *__restrict__ Ev,
                               const int *__restrict__ where, int *__restrict__ nEu,
                               int *__restrict__ nEv, int *__restrict__ emap) {
    const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= E) return;
    const unsigned e = eorig[p];
    nEu[p] = where[Eu[e]];
    nEv[p] = where[Ev[e]];
    emap[p] = (int)e;
}

// tile order: position p takes the edge now at perm[p]; its original id
// (through eorig when the session was relabelled first) for the incidence
// keys and the weights' permutation
__global__ void k_edge_tile_order(long E, const unsigned *__restrict__ perm,
                                  const unsigned *__restrict__ eorig, const int *__restrict__ Eu,
                                  const int *__restrict__ Ev, int *__restrict__ nEu,
                                  int *__restrict__ nEv, unsigned *__restrict__ eo,
                                  int *__restrict__ emap) {
    const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= E) return;
    const unsigned q = perm[p];
    nEu[p] = Eu[q];
    nEv[p] = Ev[q];
    const unsigned e = eorig ? eorig[q] : q;
    eo[p] = e;
    emap[p] = (int)e;
}

// the same for a partitioned rank: eo = the global edge id (incidence
// keys), emap = the rank-local position (the caller's per-edge arrays)
__global__ void k_edge_tile_order_halo(long E, const unsigned *__restrict__ perm,
                                       const unsigned *__restrict__ eg, long e_offset,
                                       const int *__restrict__ Eu, const int *__restrict__ Ev,
                                       int *__restrict__ nEu, int *__restrict__ nEv,
                                       unsigned *__restrict__ eo, int *__restrict__ emap,
                                       unsigned *__restrict__ inv) {
    const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= E) return;
    const unsigned q = perm[p];
    nEu[p] = Eu[q];
    nEv[p] = Ev[q];
    eo[p] = eg ? eg[q] : (unsigned)(e_offset + q);
    emap[p] = (int)q;
    inv[q] = (unsigned)p;
}

// the halo's push addresses (side E + e) into the tile order
__global__ void k_remap_push(long n, long E, const unsigned *__restrict__ inv,
                             unsigned *__restrict__ addr) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned a = addr[i];
    const unsigned side = a >= (unsigned)E ? 1u : 0u;
    addr[i] = side * (unsigned)E + inv[a - side * (unsigned)E];
}


template <typename real>
class QuadSession final : public SessionBase {
  public:
    explicit QuadSession(const pfdr_problem *p);
    ~QuadSession() override {
        if (hctrl_) {
            (void)hipStreamSynchronize(stream);  // no control-block copy in flight
            pinned_small_put(hctrl_);
        }
        for (Ctrl<real> *c : snap_) if (c) pinned_small_put(c);
        for (hipEvent_t e : snapev_) if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : ev_) if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : evv_) if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : evd_) if (e) (void)hipEventDestroy(e);
        if (comm_) (void)hipStreamDestroy(comm_);
        if (evs_) {
            (void)hipStreamSynchronize(evs_);
            (void)hipStreamDestroy(evs_);
        }
        drop_graphs();
    }
    int run(int iters) override;
    int run_pipelined(int target);
    void result(void *X_host, int *it, void *Obj_host, void *Dif_host) override;
    void *device_x() override;

  private:
    // problem
    int flavour_;  // 0 l1, 1 bounds
    int V_, Vg_, N_, mode_, itMax_, verbose_;
    long E_;
    real rho_, condMin_, difTol_, difRcd2_, cap_;
    int prox_, positivity_;
    real lo_, hi_;
    bool Ldiag_;
    bool rec_obj_, rec_dif_, track_;
    // XCD-aware block order (xcd_block): runs of 64 edge blocks / 16 vertex
    // blocks per XCD, so the neighbour bands a run gathers share one L2
    // (paired A/B on the headline: 0.754 -> 0.727 ms/iter; profiles/r1/r1zk)
    static constexpr int xcd_e_ = 64, xcd_v_ = 16;
    // the edge sweep stages the u ends of u-sorted edges in LDS (k_edge_sweep_us)
    // for graphs of at least 4 edges per vertex and for small (latency-bound)
    // graphs.  Measured (r2zf, paired, ms per edge sweep): headline 6 edges
    // per vertex 0.457 staged vs 0.472, shuffled headline 0.468 vs 0.500, C1
    // (130K edges) 0.008-0.010 vs 0.019; but 3 edges per vertex C2 0.450 vs
    // 0.394 and C5 6.55 vs 5.81 -- with few edges per u end the block's
    // staging barrier and search cost more than the Eu stream and the
    // (cache-served) u-end gathers they replace.
    bool us_ = true;
    DevBuf<char> mono_ws_;       // mono_sum scratch (tile summaries)
    // uniform La_d1 (k_uniform_check at setup): the iteration kernels take
    // the one value la0_ instead of streaming the array (4 B per edge)
    bool la_uniform_ = false;
    real la0_ = real(0);
    // uniform La_l1 (the headline's 0.01): the vertex sweep forms Th_l1 =
    // Ga * l1u instead of reading it (4 B per vertex)
    bool l1_uniform_ = false;
    real l1u_ = real(0);
    const real *la_it() const { return la_uniform_ ? nullptr : La_d1_.p; }
    // iterate evolution with the reference's sequential rounding
    // (PFDR_EVOLUTION_*, include/pfdr_mi355x.h): the vertex sweep stores the
    // terms (X_ - X)^2 and X^2 in the caller's vertex order, two binade-scan
    // sums (mono_sum) replace the tree of k_reduce_decide, k_decide decides
    int evo_ = PFDR_EVOLUTION_AUTO;
    bool seqdif_ = false;
    long tstride_ = 0;
    DevBuf<real> terms_;
    DevBuf<char> dws_;
    // partitioned sessions: the terms of the ranks in rank order are summed
    // rank to rank (ChainSum); a relabelled partition (lab_) first routes
    // every vertex's terms to the rank whose caller-order slice holds its
    // label (TermRoute: one all-to-all of ~V/N items per rank), then chains
    ChainSum<real> chain_;
    TermRoute<real> route_;
    // the transport of the evolution sums: a speculative partition's own
    // (Transport::split), so they run beside the next iteration's exchanges
    std::unique_ptr<Transport> evtr_;
    Transport &etr() { return evtr_ ? *evtr_ : *halo_->tr; }
    void seq_evolution(real *terms, const real *part, hipStream_t s);
    void sweeps(const Ctrl<real> *c);  // halo pull, edge sweep, halo push, vertex sweep
    // Speculative iteration (sequential evolution, no reconditioning
    // (difRcd = 0), no objective record, identity / diagonal A; one GPU or a
    // partition): the evolution sums and the decision on iteration t run on
    // a second stream (evs_) while iterations t + 1 ... t + D - 1 sweep;
    // iteration t + D waits for that decision (depth D = sd_: 2 on one GPU;
    // 4 on a partition of three or more ranks, whose rank-to-rank evolution
    // chain, run there over a split transport (evtr_) beside the halo
    // exchanges, takes several of a rank's iterations).  X cycles through D
    // buffers (iteration t reads xpb(t - 1), writes xpb(t)) and the terms
    // through D, so when the decision on t stops the loop, X_t is intact in
    // xpb(t) and the speculative iterations after it (their Z, their X in the
    // other buffers) are simply discarded: the iterate, iteration count and
    // Dif are the sequential loop's, bit for bit.
    static constexpr int kSpecMax = 4;
    bool spec_ = false;
    int sd_ = 2;
    int it0_ = 0;  // completed iterations when the captured / launched bodies start
    DevBuf<R2<real>> xpx_[kSpecMax - 1];  // X buffers 1 .. D - 1 (0 is xp_)
    R2<real> *xpb(int t) { return spec_ && t % sd_ ? xpx_[t % sd_ - 1].p : xp_.p; }
    R2<real> *xr_ = nullptr, *xw_ = nullptr;  // the sweeps' read / write (X, P)
    hipStream_t evs_ = nullptr;  // the decisions' stream (null: PFDR_SPEC_SERIAL, the session's)
    hipStream_t evs() const { return evs_ ? evs_ : stream; }
    hipEvent_t evv_[kSpecMax] = {}, evd_[kSpecMax] = {};
    // run_pipelined: the control block's snapshots after two chunks in flight
    Ctrl<real> *snap_[2] = {};
    hipEvent_t snapev_[2] = {};
    void body_spec(int i, int n);
    static constexpr long kSeqDifMin = 1L << 17;  // AUTO: sums of at least this many terms
    std::unique_ptr<Halo> halo_;  // partition plan (null on one GPU)
    // internal relabelling (pfdr_order.hpp): order_[new] = old, where_[old] = new,
    // emap_[edge position] = original edge id (setup only)
    bool reordered_ = false;
    DevBuf<int> order_, where_, emap_;
    DevBuf<unsigned> eorig_;
    DevBuf<real> amp_orig_;
    // device state
    DevBuf<int> Eu_, Ev_;
    DevBuf<real> La_d1_, La_l1_, Y_, A_, L_;
    DevBuf<R2<real>> xp_;
    DevBuf<real> diag_, Ga_, invAux_, Th_l1_, absval_, grad_, pre_, xout_;
    DevBuf<real> Z2_, wz_;
    // splitting weights as factors (k_d1_weights): a_e = cw_ La_d1[e] until the
    // first reconditioning, then A1_[e]; (Ga, invAux) pairs of every vertex
    DevBuf<real> A1_;
    DevBuf<R2<real>> gi_;
    DevBuf<real> rr_;  // per-vertex (cw la0 / Aux) / Ga of the ratio edge sweep (rat())
    int vpair_cap_ = 0;  // pair vertex sweep: entries of the largest record block (0: off)
    bool rat_on_ = false;  // rr_ formed at setup (see rat())
    real cw_ = real(0);
    DevBuf<real> R_, vpart_, opart_, Obj_, Dif_, red_, csum_;
    DevBuf<double> Rpart_;  // k_rows_partial's double partials
    DevBuf<real> Rsum_, xfull_;  // dense A on a partition: summed A X, gathered X
    // relabelled partition (pfdr_problem.vtx_label): the caller's label of
    // each owned vertex; the amplitudes are all-reduced into ampg_ at those
    // labels and summed in the caller's order on every rank
    DevBuf<int> lab_;
    DevBuf<real> ampg_;
    long v0_ = 0, Vglob_ = 0;
    DevBuf<long long> ccnt_;
    DevBuf<int> cnt_part_;
    DevBuf<Ctrl<real>> ctrl_;
    Incidence inc_;
    HostPins pins_;  // caller arrays pinned for the setup copies
    // split incidence (edges sorted by u): u-run offsets, per-vertex order
    // masks, addresses of the other entries, per-block path flag
    DevBuf<int> uptr_, blkok_;
    DevBuf<unsigned> mask_, oidx_;
    void build_split();
    // tiled contributions (tile_sum in pfdr_quadratic_kernels.hpp): large
    // single-GPU graphs keep their edges sorted by (u block, v block, edge);
    // d2_ = CSR slot of every contribution address within its vertex block,
    // ustart_ / tptr_, tstart_, tlen_ = the runs each block stages, tok_ =
    // blocks whose lists fit the LDS (the others gather through the CSR)
    bool tiled_ = false;
    DevBuf<Slots12> slots_;
    DevBuf<unsigned char> deg8_;  // CSR entries per vertex (tile_sum)
    DevBuf<unsigned short> luv_;  // both ends mod 256 (k_edge_sweep_tl)
    DevBuf<int> erec_;            // per edge block: u blocks and v runs (k_edge_sweep_tl)
    DevBuf<int> ustart_, tptr_, tstart_, tlen_, tok_, trec_;
    DevBuf<Slots12> ptab_;        // slot patterns of the record blocks' runs (k_run_hash)
    DevBuf<int> prec_;            // per record block: its runs' offsets into ptab_
    void build_tiles();
    void build_patterns(const unsigned short *d2, long n);
    void build_tile_runs();
    Ctrl<real> *hctrl_ = nullptr;  // pinned mirror
    int nbv_, nbe_, nbn_, rows_nb_, rows_cpb_;
    int it_ = 0;
    bool stopped_ = false;
    int chunk_ = 32;
    int next_print_ = 0;
    // hipGraph of a chunk of iterations (single GPU, unprofiled): a replayed
    // kernel boundary costs ~1.6 us of GPU time, a launched one ~2.8 us
    // (profiles/r2/r2d_launch_gap.log) -- the difference is a large share of
    // an iteration of a small graph.  Re-captured after a reconditioning
    // (new kernel arguments).
    bool graphs_ok_ = false;
    bool capturable_ = false;  // prepare(): graphs of any run length on request
    std::map<int, hipGraphExec_t> graphs_;
    void run_bodies(int n);
    hipGraphExec_t chunk_graph(int n);
  public:
    void prepare(int iters) override;
  private:
    void drop_graphs() {
        for (auto &kv : graphs_) (void)hipGraphExecDestroy(kv.second);
        graphs_.clear();
    }

    void setup_graph(const pfdr_problem *p);
    void amplitude(bool init);
    void precondition(bool init);
    void gemv_rows(int gate);
    void forward_dense(int gate);
    void gradient();
    void objective();
    void body(int i, int n);  // i-th of n bodies of a chunk
    void push_ctrl();
    void pull_ctrl();
    void wait_stream();
    void print_progress();
    void pull(void *base, int eb) { if (halo_) halo_->pull(base, eb, stream); }
    // halo / compute overlap (partitioned sessions): the halo exchanges run
    // on comm_ while the sweeps of interior edges [elo_, ehi_) and interior
    // vertex blocks [blo_, bhi_) (no ghost endpoint, no received
    // contribution) run on the session stream
    hipStream_t comm_ = nullptr;
    hipEvent_t ev_[4] = {};  // xp ready, pulled, boundary W*Z ready, pushed
    long elo_ = 0, ehi_ = 0;
    long Eint_ = 0;  // tiled partitioned rank: edges [0, Eint_) have no ghost end
    long zs_ = 0;    // Z layout: 0 half-edge pairs, E side-major (tiled sessions)
    // Z-direct: a tiled single-GPU session with one edge weight and no A1
    // (before any reconditioning) skips the W * Z stores of the edge sweep;
    // the vertex sweep reads Z and forms each term with its own weight
    // (a partitioned session only when every rank qualifies with the same
    // weight, zd_ranks_: the ranks then push Z, and each owner forms the
    // received terms with its own weight like the local ones)
    bool zd_ranks_ = false;
    bool zdirect() const { return tiled_ && !A1_.p && (halo_ ? zd_ranks_ : !la_it()); }
    // one edge weight and no W * Z stream (until the first reconditioning):
    // the tiled edge sweep reads the ends' formed ratios (k_ratio_vertex)
    // instead of their (Ga, invAux) pairs
    bool rat() const { return rat_on_ && zdirect() && !la_it(); }
    int blo_ = 0, bhi_ = 0;
    bool overlap_ = false;
    void plan_overlap();
    // one launch over [ebeg, eend) and, if not empty, [ebeg2, eend2)
    void edge_sweep(long ebeg, long eend, const Ctrl<real> *c, const char *name,
                    long ebeg2 = 0, long eend2 = 0, const FuseDecide<real> *fd = nullptr);
    // one launch over the blocks [bbeg, bend) and, if not empty, [bbeg2, bend2)
    void vertex_sweep(int bbeg, int bend, const Ctrl<real> *c, const char *name,
                      int bbeg2 = 0, int bend2 = 0);
    VArgs<real> vargs(int bbeg, int bend, const Ctrl<real> *c);
    // small single-GPU graphs: a chunk of iterations in one workgroup launch
    // (k_tiny_iterate; PFDR_TINY = max edges, 0 = off)
    bool tiny_ = false;
    void tiny_chunk(int n);
    const real *full_x();  // X of every vertex (A^tA mode), gathered over the ranks
    // A^tA mode on one GPU with an exactly symmetric matrix: products from the
    // block upper triangle (k_symv_tiles / k_symv_finish, half the bytes)
    bool symv_ = false;
    int snb_ = 0;
    // small dense problems on one GPU (CP's reduced problems): every dot
    // product in the reference's sequential order (k_col_seq, k_rows_seq),
    // bit-exact, when the longest chain (max(N, V) direct, V for A^tA) is
    // <= kExactChain
    bool exact_ = false;
    static constexpr long kExactChain = 8192;
    // small graphs (<= kFuseBlocks vertex blocks, dif tracked, one GPU):
    // the loop decision on iteration t taken inside the edge sweep of t + 1,
    // two launches per iteration instead of three (FuseDecide in
    // pfdr_quadratic_kernels.hpp); the decisions alternate between ctrl_
    // (even bodies of a chunk) and ctrl2_ (odd), the chunk's closing
    // decision lands in ctrl_.
    bool fuse_ = false;
    DevBuf<Ctrl<real>> ctrl2_;
    // fused sessions whose vertex blocks have at most kPadPer * kBlock CSR
    // entries: the edge sweep stores each contribution at its slot sl_[2e +
    // side] of its block's list in wzp_ (stride pad_nmax_), and the vertex
    // sweep (k_vertex_sweep_pad) stages its block's list with one dependent
    // round trip instead of three.
    bool pad_ = false;
    static constexpr int kPadBlocks = 512;
    int pad_nmax_ = 0;
    DevBuf<int> sl_;
    DevBuf<real> wzp_;
    // and, in f32 up to kEndsBlocks, the endpoint data as per-edge copies: (X, P)
    // and (Ga, 1/Aux) of both ends at xpe_ / gie_ [2e + side], scattered by
    // the vertex sweep through pidx_ (the end of each list entry), so the
    // edge sweep (k_edge_sweep_ends) streams everything: one dependent
    // round trip.
    bool ends_ = false;
    static constexpr int kEndsBlocks = 512;
    DevBuf<int> pidx_;
    DevBuf<R2<real>> xpe_, gie_;
    void refresh_ends();
    void plan_pad();
    PadOut<real> pad_out() const { return PadOut<real>{pad_ ? sl_.p : nullptr, wzp_.p}; }
    template <int EPI> void col_product(ColArgs<real> ca);
    DevBuf<real> spart_;
    void plan_symv();
    template <int EPI> void ata_product(ColArgs<real> ca);
};

// ----------------------------------------------------------------- setup --
template <typename real>
QuadSession<real>::QuadSession(const pfdr_problem *p) {
    if (p->V <= 0 || p->E < 0) throw std::runtime_error("V must be > 0 and E >= 0");
    if (!p->X || !p->Y || !p->Eu || !p->Ev || !p->La_d1)
        throw std::runtime_error("X, Y, Eu, Ev and La_d1 are required");
    PFDR_HIP(hipGetDevice(&device));
    stream = lib_stream();
    pins_.set_stream(stream);
    hipStream_t s = stream;
    flavour_ = (p->kind == PFDR_KIND_BOUNDS) ? 1 : 0;
    V_ = p->V;
    E_ = p->E;
    N_ = p->N;
    itMax_ = p->itMax;
    verbose_ = p->verbose;
    if (N_ > 0) mode_ = A_DIRECT;
    else if (N_ < 0) mode_ = A_ATA;
    else mode_ = p->A ? A_DIAG : A_IDENT;
    if (mode_ == A_DIRECT && !p->A) throw std::runtime_error("N > 0 requires A");
    if (mode_ == A_ATA && !p->A) throw std::runtime_error("N < 0 requires A = A^tA");
    rho_ = (real)p->rho;
    condMin_ = (real)p->condMin;
    difTol_ = (real)p->difTol;
    const real difRcd = (real)p->difRcd;
    difRcd2_ = difRcd * difRcd;
    rec_obj_ = p->record_obj != 0;
    rec_dif_ = p->record_dif != 0;
    track_ = (difTol_ > real(0)) || (difRcd > real(0)) || rec_dif_;
    evo_ = p->evolution;
    if (evo_ < PFDR_EVOLUTION_AUTO || evo_ > PFDR_EVOLUTION_TREE)
        throw std::runtime_error("evolution must be PFDR_EVOLUTION_AUTO, _SEQUENTIAL or _TREE");
    const bool want_seq = track_ && evo_ == PFDR_EVOLUTION_SEQUENTIAL;
    Ldiag_ = (p->Ltype == PFDR_LIPSCHITZ_DIAG) && p->L;
    us_ = E_ >= 4L * V_ || E_ < (1L << 22);
    // prox selection (ref l1 :499-512, bounds :472-490)
    positivity_ = 0;
    lo_ = hi_ = real(0);
    if (flavour_ == 0) {
        positivity_ = p->positivity != 0;
        prox_ = p->La_l1 ? PROX_L1 : (positivity_ ? PROX_POS : PROX_NONE);
    } else {
        lo_ = (real)p->min;
        hi_ = (real)p->max;
        const real inf = Lim<real>::huge;
        const bool haslo = -inf < lo_, hashi = hi_ < inf;
        prox_ = (haslo && hashi) ? PROX_BOX : haslo ? PROX_LO : hashi ? PROX_HI : PROX_NONE;
    }

    // small single-GPU graphs iterate in one 1024-lane workgroup
    // (k_tiny_iterate, four vertex blocks at a time): against the two-launch
    // loop (fused decision, per-block lists) on 4-NN grids, us/iteration
    // (profiles/r2/r2zv_exp_tiny.log): f32 1 block 4.4 vs 8.9, 4: 6.6 vs
    // 10.8, 8: 10.5 vs 10.8, 16: 19.3 vs 11.1; f64 4: 8.0 vs 10.0, 8: 13.5
    // vs 9.8 -- so up to 8 blocks in f32, 5 in f64, and 8192 edges.  The
    // split incidence is not built for them (one setup round trip less).
    if (!(p->nranks > 1 || p->comm) && !rec_obj_ && (mode_ == A_IDENT || mode_ == A_DIAG) &&
        E_ > 0 && !want_seq) {
        const char *t = getenv("PFDR_TINY");
        const long maxE = t ? atol(t) : 8192;
        const int maxB = t ? kTinyMaxBlocks : (sizeof(real) == 4 ? 8 : 5);
        tiny_ = E_ <= maxE && (V_ + kBlock - 1) / kBlock <= maxB;
        tiny = tiny_ ? 1 : 0;
    }
    // graph, partition plan, incidence CSR
    setup_graph(p);
    // dense A on a partition: this rank's columns (its vertices); A^tA columns
    // have the global length
    v0_ = halo_ ? (long)halo_->vtx_begin : 0;
    Vglob_ = halo_ ? (long)halo_->off.back() : V_;
    if (p->vtx_label) {
        if (!halo_) throw std::runtime_error("vtx_label is for partitioned sessions");
        std::vector<int64_t> h64(V_);
        PFDR_HIP(hipMemcpy(h64.data(), p->vtx_label, sizeof(int64_t) * V_,
                           p->mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToHost : hipMemcpyHostToHost));
        std::vector<int> h32(V_);
        for (int v = 0; v < V_; v++) {
            if (h64[v] < 0 || h64[v] >= Vglob_)
                throw std::runtime_error("vtx_label outside [0, V_global)");
            h32[v] = (int)h64[v];
        }
        lab_.alloc(V_);
        PFDR_HIP(hipMemcpy(lab_.p, h32.data(), sizeof(int) * V_, hipMemcpyHostToDevice));
        check_permutation(lab_.p, V_, Vglob_, *halo_->tr, s);
    }
    if (mode_ == A_ATA && -(long)N_ != Vglob_)
        throw std::runtime_error("N < 0 requires A = A^tA (columns of the owned vertices, "
                                 "length V) and N = -V (V over all ranks)");
    if ((mode_ == A_DIRECT || mode_ == A_ATA) && !halo_) {
        const long chain = mode_ == A_DIRECT ? std::max<long>(N_, V_) : (long)V_;
        exact_ = chain <= kExactChain;
        dense_exact = exact_ ? 1 : 0;
    }
    const int mem = p->mem;
    const size_t V = V_, E = E_, Vg = Vg_;
    copy_in(La_d1_, p->La_d1, E, mem, s, pins_);
    if (flavour_ == 0) copy_in(La_l1_, p->La_l1, V, mem, s, pins_);
    copy_in(Y_, p->Y, mode_ == A_DIRECT ? (size_t)N_ : V, mem, s, pins_);
    const size_t asz = mode_ == A_DIRECT ? (size_t)N_ * V : mode_ == A_ATA ? (size_t)Vglob_ * V
                     : mode_ == A_DIAG ? V : 0;
    copy_in(A_, p->A, asz, mem, s, pins_);
    if (emap_.p) {  // edge weights into the internal edge order
        permute(La_d1_, emap_.p, E, s);
        emap_.release();
    }
    if (reordered_) {  // inputs into the internal labels (identity / diagonal A only)
        permute(La_l1_, order_.p, V, s);
        permute(Y_, order_.p, V, s);
        permute(A_, order_.p, V, s);
        amp_orig_.alloc(V);
    }
    // scalar cap of the metric (ref :225-229), in `real` arithmetic like the reference
    real cap = real(1.9) * (real(2) - rho_);
    if (p->L && !Ldiag_) {
        real L0;
        PFDR_HIP(hipMemcpyAsync(&L0, p->L, sizeof(real),
                                mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToHost : hipMemcpyHostToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
        cap /= L0;
    }
    cap_ = cap;
    if (Ldiag_) copy_in(L_, p->L, V, mem, s, pins_);
    if (reordered_ && Ldiag_) permute(L_, order_.p, V, s);
    {   // iterate (X, P) pairs, owned then ghost vertices
        DevBuf<real> X0;
        copy_in(X0, p->X, V, mem, s, pins_);
        if (reordered_) permute(X0, order_.p, V, s);
        xp_.alloc(Vg + 2);  // (+2: the tiled edge sweep stages vertex pairs, k_edge_sweep_tl)
        PFDR_HIP(hipMemsetAsync(xp_.p, 0, (Vg + 2) * sizeof(R2<real>), s));
        k_xp_init<real><<<grid_for(V), kBlock, 0, s>>>(V_, X0.p, xp_.p);
        PFDR_HIP(hipGetLastError());
        pull(xp_.p, sizeof(R2<real>));
    }  // X0 goes back to the device cache (reused once the stream is idle)
    // edge state and per-vertex metric
    const size_t En = E ? E : 1;
    // (tiled partitioned ranks: Z's received tail after the 2E local entries,
    // for the Z-direct iteration)
    // (+kSlotGroup: the tiled vertex sweep reads whole groups of a run's tail, tile_sum)
    Z2_.alloc(2 * En + (halo_ ? (size_t)halo_->R : 0) + kSlotGroup);
    gi_.alloc(Vg + 2);
    PFDR_HIP(hipMemsetAsync(gi_.p, 0, (Vg + 2) * sizeof(R2<real>), s));
    diag_.alloc(V); Ga_.alloc(Vg); invAux_.alloc(Vg); absval_.alloc(V);
    if (flavour_ == 0 && p->La_l1) Th_l1_.alloc(V);
    nbv_ = grid_for(V);
    nbe_ = grid_for(E);
    nbn_ = mode_ == A_DIRECT ? grid_for(N_) : 0;
    cnt_part_.alloc(nbv_);
    vpart_.alloc(2 * (size_t)nbv_);
    red_.alloc(4);
    csum_.alloc(1);
    ccnt_.alloc(1);
    if (rec_obj_) {
        opart_.alloc(2 * (size_t)nbv_ + nbe_ + nbn_ + 1);
        Obj_.alloc((size_t)itMax_ + 1);
    }
    if (rec_dif_) Dif_.alloc(itMax_ > 0 ? itMax_ : 1);
    if (mode_ == A_DIRECT) {
        R_.alloc(N_);
        pre_.alloc(V);
        rows_nb_ = std::max(1, std::min(512, (V_ + 63) / 64));
        rows_cpb_ = (V_ + rows_nb_ - 1) / rows_nb_;
        rows_nb_ = (V_ + rows_cpb_ - 1) / rows_cpb_;
        Rpart_.alloc((size_t)rows_nb_ * N_);
    }
    if (mode_ == A_ATA) { pre_.alloc(V); xout_.alloc(V); xfull_.alloc(Vglob_); plan_symv(); }
    if (mode_ == A_DIRECT && halo_) Rsum_.alloc(N_);

    // control block
    ctrl_.alloc(1);
    static_assert(sizeof(Ctrl<real>) <= kPinnedSmall, "control block");
    hctrl_ = static_cast<Ctrl<real> *>(pinned_small_get());
    std::memset(hctrl_, 0, sizeof(Ctrl<real>));
    const real difTol2 = difTol_ * difTol_;
    hctrl_->obj_it = -1;
    hctrl_->itMax = itMax_;
    hctrl_->dif = difTol2 > difRcd2_ ? difTol2 : difRcd2_;  // ref :342
    hctrl_->difTol = difTol2;
    hctrl_->difRcd = difRcd2_;
    hctrl_->eps = (real(0) < difTol_ && difTol_ < Lim<real>::eps) ? difTol_ : Lim<real>::eps;
    push_ctrl();

    // diagonal of A^t A
    if (mode_ == A_DIRECT) {
        ColArgs<real> ca{};
        ca.A = A_.p; ca.ncols = V_; ca.len = N_; ca.out = diag_.p;
        col_product<EPI_SELF>(ca);
    } else {
        k_diag<real><<<grid_for(V), kBlock, 0, s>>>(V_, mode_, A_.p, Vglob_, v0_, diag_.p);
    }
    PFDR_HIP(hipGetLastError());
    // uniform La_d1 / La_l1? (read back with c below)
    DevBuf<int> ubad(2);
    PFDR_HIP(hipMemsetAsync(ubad.p, 0, 2 * sizeof(int), s));
    if (E_) k_uniform_check<real><<<grid_for(E), kBlock, 0, s>>>(E_, La_d1_.p, ubad.p);
    if (La_l1_.p) k_uniform_check<real><<<grid_for(V), kBlock, 0, s>>>(V_, La_l1_.p, ubad.p + 1);
    // Z = X at both ends, first preconditioning, first forward step
    zs_ = tiled_ ? E_ : 0;
    if (E_) k_z_init<real><<<grid_for(E), kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, xp_.p, Z2_.p, zs_);
    precondition(true);
    if (mode_ == A_IDENT || mode_ == A_DIAG) {
        grad_.alloc(V);
        k_grad_vertex<real><<<grid_for(V), kBlock, 0, s>>>(V_, mode_, A_.p, Y_.p, xp_.p, grad_.p);
        k_forward_grad<real><<<grid_for(V), kBlock, 0, s>>>(V_, Ga_.p, grad_.p, xp_.p);
        PFDR_HIP(hipGetLastError());
        grad_.release();
    } else {
        forward_dense(GATE_NONE);
    }
    if (rec_obj_) objective();  // Obj[0]
    PFDR_HIP(hipStreamSynchronize(s));
    // c of the first conditioning: a_e = cw_ La_d1[e] in the edge sweeps
    PFDR_HIP(hipMemcpy(&cw_, &ctrl_.p->c, sizeof(real), hipMemcpyDeviceToHost));
    if (E_) {
        int bad = 1;
        PFDR_HIP(hipMemcpy(&bad, ubad.p, sizeof(int), hipMemcpyDeviceToHost));
        PFDR_HIP(hipMemcpy(&la0_, La_d1_.p, sizeof(real), hipMemcpyDeviceToHost));
        la_uniform_ = bad == 0;
        la_uniform = la_uniform_ ? 1 : 0;
    }
    if (La_l1_.p) {
        int bad = 1;
        PFDR_HIP(hipMemcpy(&bad, ubad.p + 1, sizeof(int), hipMemcpyDeviceToHost));
        PFDR_HIP(hipMemcpy(&l1u_, La_l1_.p, sizeof(real), hipMemcpyDeviceToHost));
        l1_uniform_ = bad == 0;
    }
    if (halo_) {  // Z-direct on every rank or on none (see zdirect)
        Transport &tr = *halo_->tr;
        DevBuf<real> l0(1);
        DevBuf<int64_t> nbad(1);
        PFDR_HIP(hipMemcpyAsync(l0.p, &la0_, sizeof(real), hipMemcpyHostToDevice, s));
        tr.broadcast(l0.p, sizeof(real), 0, s);
        real la0r0 = real(0);
        PFDR_HIP(hipMemcpyAsync(&la0r0, l0.p, sizeof(real), hipMemcpyDeviceToHost, s));
        tr.wait(s);
        const int64_t mine = (tiled_ && la_uniform_ && la0_ == la0r0) ? 0 : 1;
        PFDR_HIP(hipMemcpyAsync(nbad.p, &mine, sizeof(int64_t), hipMemcpyHostToDevice, s));
        tr.allreduce_sum(nbad.p, 1, 2, s);
        int64_t all = 1;
        PFDR_HIP(hipMemcpyAsync(&all, nbad.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        tr.wait(s);
        zd_ranks_ = all == 0;
    }
    pins_.release();
    stopped_ = (itMax_ <= 0);
    interior_edges = E_;

    device_bytes = 0;
    auto acc = [&](size_t b) { device_bytes += (int64_t)b; };
    acc(Eu_.n * 4 + Ev_.n * 4);
    for (DevBuf<real> *b : {&La_d1_, &La_l1_, &Y_, &A_, &L_, &diag_, &Ga_, &invAux_, &Th_l1_, &absval_,
                            &pre_, &Z2_, &A1_, &wz_, &R_,
                            &vpart_, &opart_, &Obj_, &Dif_, &xout_, &Rsum_, &xfull_, &spart_})
        acc(b->n * sizeof(real));
    acc(Rpart_.n * sizeof(double));
    acc((xp_.n + gi_.n) * sizeof(R2<real>) + inc_.ptr.n * 4 + inc_.idx.n * 4);
    acc((uptr_.n + mask_.n + oidx_.n + blkok_.n) * 4);
    acc(slots_.n * sizeof(Slots12) + luv_.n * 2 + deg8_.n +
        (ustart_.n + tptr_.n + tstart_.n + tlen_.n + tok_.n + trec_.n + erec_.n) * 4);
    if (halo_) {
        plan_overlap();
        // RCCL partitions replay captured chunks too (pull, sweeps, push and
        // the all-reduces of a chunk of iterations in one hipGraph launch:
        // the host's ~30 API calls per iteration otherwise approach a rank's
        // GPU time at N = 8); the loopback transport rendezvous on the host
        capturable_ = halo_->tr->capturable() && !rec_obj_;
        graphs_ok_ = itMax_ >= 2 * chunk_ && capturable_;
    } else if (!tiny_) {
        capturable_ = true;
        graphs_ok_ = itMax_ >= 2 * chunk_;
        // (an edgeless graph has no edge sweep to carry the decision)
        fuse_ = track_ && !rec_obj_ && (mode_ == A_IDENT || mode_ == A_DIAG) &&
                nbv_ <= kFuseBlocks && E_ > 0 && !want_seq;
        if (fuse_) ctrl2_.alloc(1);
        fused = fuse_ ? 1 : 0;
        if (fuse_) plan_pad();
    }
    // sequential evolution statistic: the plain multi-launch loop on one GPU;
    // a partition sums in the caller's order across the ranks (seq_evolution)
    seqdif_ = track_ && !tiny_ && !fuse_ &&
              (want_seq || (evo_ == PFDR_EVOLUTION_AUTO && Vglob_ >= kSeqDifMin));
    if (seqdif_) {
        const long nt = V_;  // terms per sum, in this rank's vertex order
        tstride_ = (nt + 3) / 4 * 4;  // 16-byte aligned second array
        terms_.alloc(2 * (size_t)tstride_);
        if (!halo_) {
            dws_.alloc(mono_ws_bytes<real>(nt, 2));
        } else if (lab_.p) {  // routed to caller-order slices, then chained
            std::vector<int> hl(V_);
            PFDR_HIP(hipMemcpy(hl.data(), lab_.p, sizeof(int) * V_, hipMemcpyDeviceToHost));
            route_.init(hl, Vglob_, 2, 1, *halo_->tr, s);
        } else {
            chain_.init(V_, 2, *halo_->tr);
        }
        seqdif = 1;
        const int smode = spec_mode(p);
        spec_ = difRcd2_ == real(0) && !rec_obj_ && (mode_ == A_IDENT || mode_ == A_DIAG) &&
                smode != PFDR_SPEC_OFF;
        const bool serial = smode == PFDR_SPEC_SERIAL;
        if (spec_ && halo_ && !serial) {
            evtr_ = halo_->tr->split(s);  // (a collective: every rank decides alike)
            // the halo exchanges stay on the session stream: a third stream
            // for them (overlap_) shared a hardware queue with the evolution
            // stream, so the next pull waited behind the whole evolution chain
            // (1-rank RCCL headline_conv 0.686 ms/iter against 0.557 on one GPU)
            overlap_ = false;
        }
        if (spec_) {
            sd_ = halo_ && halo_->tr->nranks >= 3 ? 4 : 2;
            DevBuf<real> t2((size_t)sd_ * 2 * tstride_);  // terms of D iterations
            std::swap(terms_.p, t2.p);
            std::swap(terms_.n, t2.n);
            DevBuf<real> p2((size_t)sd_ * 2 * nbv_);  // and their block sums
            std::swap(vpart_.p, p2.p);
            std::swap(vpart_.n, p2.n);
            for (int k = 0; k + 1 < sd_; k++) {
                xpx_[k].alloc(Vg_ + 2);  // (+2 as xp_)
                PFDR_HIP(hipMemcpyAsync(xpx_[k].p, xp_.p, sizeof(R2<real>) * (Vg_ + 2),
                                        hipMemcpyDeviceToDevice, s));
            }
            if (!serial) PFDR_HIP(hipStreamCreateWithFlags(&evs_, hipStreamNonBlocking));
            for (int k = 0; k < sd_; k++) {
                PFDR_HIP(hipEventCreateWithFlags(&evv_[k], hipEventDisableTiming));
                PFDR_HIP(hipEventCreateWithFlags(&evd_[k], hipEventDisableTiming));
            }
            speculative = serial ? 2 : 1;
        }
    }
    {
        // the ratio edge sweep where it pays: not beside an overlapped
        // evolution chain, whose kernels the faster sweep (eight waves per
        // SIMD against the pair sweep's seven) leaves no room to run in --
        // converged headline 0.570 ms/iter against 0.524 (f6d).
        // PFDR_EDGE_RATIO=0 / 1: never / wherever it applies.
        const char *e = getenv("PFDR_EDGE_RATIO");
        rat_on_ = e && *e ? e[0] != '0' : speculative != 1;
    }
    if (rat()) {  // cw_ and la0_ are known from here (owned and ghost ends)
        rr_.alloc(Vg_ + 2);  // (+2: the tiled edge sweep stages vertex pairs)
        PFDR_HIP(hipMemsetAsync(rr_.p, 0, (Vg_ + 2) * sizeof(real), s));
        k_ratio_vertex<real><<<grid_for(Vg_), kBlock, 0, s>>>(Vg_, cw_, la0_, Ga_.p, invAux_.p,
                                                              rr_.p);
        PFDR_HIP(hipGetLastError());
        device_bytes += (int64_t)(rr_.n * sizeof(real));
        edge_ratio = 1;
    }
    xr_ = xw_ = xp_.p;
    // a speculative session launches directly on its two streams: the
    // decision's kernels must run BESIDE the next sweeps, and a replayed
    // graph ran its branches one after the other (headline_conv 0.852
    // ms/iter with the graph, r4h)
    if (spec_) graphs_ok_ = capturable_ = false;
    if (!seqdif_ || !reordered_) order_.release();  // inputs are in the internal labels now
    acc(where_.n * 4 + amp_orig_.n * sizeof(real) + order_.n * 4 + terms_.n * sizeof(real) + dws_.n);
    acc(route_.slice.n * sizeof(real) + route_.chain.ws.n + chain_.ws.n + ampg_.n * sizeof(real) +
        (xpx_[0].n + xpx_[1].n + xpx_[2].n) * sizeof(R2<real>));
    acc(sl_.n * 4 + wzp_.n * sizeof(real) + pidx_.n * 4 + (xpe_.n + gie_.n) * sizeof(R2<real>));
    // the chunk graph is part of the setup (instantiation costs ~0.1-1 ms,
    // which a small solve timed to tolerance would otherwise pay in its loop)
    if (graphs_ok_) {
        try {
            (void)chunk_graph(chunk_);
        } catch (const std::exception &) {
            if (!halo_) throw;
            graphs_ok_ = capturable_ = false;  // this transport would not capture: launch directly
            (void)hipGetLastError();
        }
    }
    graphs = graphs_ok_ ? 1 : 0;
}

template <typename real>
void QuadSession<real>::plan_pad() {
    // up to kPadBlocks vertex blocks: at 1024 blocks (512^2 grid, f32) the
    // scattered contribution stores cost more than the round trips they save
    // (profiles/r2/r2zp_exp_pad.log, r2zq_exp_pad.log)
    if (halo_ || !E_ || nbv_ > kPadBlocks) return;
    hipStream_t s = stream;
    PinnedSmall pin(s);
    int *hm = static_cast<int *>(pin.p);
    DevBuf<int> dm(1);
    PFDR_HIP(hipMemsetAsync(dm.p, 0, sizeof(int), s));
    k_pad_nmax<<<grid_for(nbv_), kBlock, 0, s>>>(V_, nbv_, inc_.ptr.p, dm.p);
    PFDR_HIP(hipGetLastError());
    PFDR_HIP(hipMemcpyAsync(hm, dm.p, sizeof(int), hipMemcpyDeviceToHost, s));
    PFDR_HIP(hipStreamSynchronize(s));
    const int nmax = std::max(kBlock, (*hm + kBlock - 1) / kBlock * kBlock);
    if (nmax > kPadPer * kBlock) return;
    sl_.alloc(2 * (size_t)E_);
    wzp_.alloc((size_t)nbv_ * nmax);
    PFDR_HIP(hipMemsetAsync(wzp_.p, 0, wzp_.n * sizeof(real), s));
    // f32 up to kEndsBlocks (f32 us/iter 11.2 -> 9.6 at 9 blocks, 11.5 ->
    // 10.5 at 256, 12.7 -> 12.2 at 507; f64 slower: 10.4 -> 11.0 at 9 blocks,
    // 12.5 -> 26 at 256; profiles/r2/r2zz_exp_ends.log, r2zz2)
    ends_ = sizeof(real) == 4 && nbv_ <= kEndsBlocks;
    if (ends_) {
        pidx_.alloc((size_t)nbv_ * nmax);
        PFDR_HIP(hipMemsetAsync(pidx_.p, 0, pidx_.n * sizeof(int), s));
        xpe_.alloc(2 * (size_t)E_);
        gie_.alloc(2 * (size_t)E_);
    }
    k_pad_slots<<<nbv_, kBlock, 0, s>>>(V_, E_, inc_.ptr.p, inc_.idx.p, nmax, sl_.p,
                                        ends_ ? pidx_.p : nullptr);
    PFDR_HIP(hipGetLastError());
    pad_nmax_ = nmax;
    pad_ = true;
    padded = 1;
    refresh_ends();
}

template <typename real>
void QuadSession<real>::refresh_ends() {
    if (!ends_) return;
    k_pad_ends<real><<<grid_for(E_), kBlock, 0, stream>>>(E_, Eu_.p, Ev_.p, xp_.p, gi_.p, xpe_.p,
                                                          gie_.p);
    PFDR_HIP(hipGetLastError());
}

// endpoints (local ids), partition plan, incidence CSR keyed by global edge id
template <typename real>
void QuadSession<real>::setup_graph(const pfdr_problem *p) {
    hipStream_t s = stream;
    const size_t E = E_;
    const auto kind = p->mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    Eu_.alloc(E ? E : 1);
    Ev_.alloc(E ? E : 1);
    DevBuf<unsigned> eg;
    const unsigned *eg_ptr = nullptr;  // original edge ids of a relabelled graph
    long e_offset = 0;
    if (p->nranks > 1 || p->comm) {
        partition_setup(p, V_, E_, halo_, Eu_, Ev_, eg, &e_offset, s);
        Vg_ = V_ + halo_->G;
        ghosts = halo_->G;
    } else {
        Vg_ = V_;
        if (E && kind == hipMemcpyHostToDevice) {
            pins_.copy(Eu_.p, p->Eu, E * 4, kind);
            pins_.copy(Ev_.p, p->Ev, E * 4, kind);
        } else if (E) {
            PFDR_HIP(hipMemcpyAsync(Eu_.p, p->Eu, E * 4, kind, s));
            PFDR_HIP(hipMemcpyAsync(Ev_.p, p->Ev, E * 4, kind, s));
        }
    }
    check_endpoints(Eu_.p, Ev_.p, E_, Vg_, s);
    if (!halo_ && E_ && (mode_ == A_IDENT || mode_ == A_DIAG) && p->reorder != PFDR_REORDER_OFF &&
        (p->reorder == PFDR_REORDER_ON || labels_scattered(Eu_.p, Ev_.p, E_, V_, s)) &&
        bfs_order(Eu_.p, Ev_.p, E_, V_, order_, where_, s)) {
        // relabel the vertices and sort the edges by their new u end; the
        // incidence keys keep the original edge ids (summation order)
        reordered_ = true;
        reordered = 1;
        DevBuf<unsigned long long> k(E), ks(E);
        DevBuf<unsigned> v(E);
        eorig_.alloc(E);
        k_edge_order_keys<<<grid_for(E), kBlock, 0, s>>>(E_, Eu_.p, where_.p, k.p, v.p);
        PFDR_HIP(hipGetLastError());
        radix_sort_pairs_stable<unsigned long long>(k.p, ks.p, v.p, eorig_.p, (long)E, 64, s);
        DevBuf<int> nu(E), nv(E);
        emap_.alloc(E);
        k_edge_relabel<<<grid_for(E), kBlock, 0, s>>>(E_, eorig_.p, Eu_.p, Ev_.p, where_.p, nu.p,
                                                      nv.p, emap_.p);
        PFDR_HIP(hipGetLastError());
        PFDR_HIP(hipStreamSynchronize(s));
        std::swap(Eu_.p, nu.p);
        std::swap(Ev_.p, nv.p);
        eg_ptr = eorig_.p;
    }
    // tile order of large graphs (see tile_sum): edges sorted by (u block,
    // v block), stable in the current order; the incidence keys keep the
    // original edge ids (summation order).  A partitioned rank puts the
    // edges with a ghost end after the others (the interior ones overlap
    // the halo pull) and renumbers its push addresses.
    tiled_ = !tiny_ && E_ > 0 && (long)V_ > (long)kFuseBlocks * kBlock;
    if (tiled_) {
        const int nb = grid_for(Vg_);
        int vbits = 1;
        while (vbits < 31 && (1L << vbits) < (long)nb) vbits++;
        DevBuf<unsigned long long> k(E), ks(E), nint(1);
        DevBuf<unsigned> v(E), perm(E);
        k_tile_keys<<<grid_for(E), kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, vbits, k.p, v.p, V_,
                                                   halo_ != nullptr);
        PFDR_HIP(hipGetLastError());
        radix_sort_pairs_stable<unsigned long long>(k.p, ks.p, v.p, perm.p, (long)E,
                                                    2 * vbits + (halo_ ? 1 : 0), s);
        if (halo_) k_count_below<<<1, 1, 0, s>>>(E_, ks.p, 1ull << (2 * vbits), nint.p);
        DevBuf<int> nu(E), nv(E);
        DevBuf<unsigned> eo(E);
        emap_.alloc(E);
        if (halo_) {
            DevBuf<unsigned> inv(E);
            k_edge_tile_order_halo<<<grid_for(E), kBlock, 0, s>>>(
                E_, perm.p, eg.p, e_offset, Eu_.p, Ev_.p, nu.p, nv.p, eo.p, emap_.p, inv.p);
            const long np = halo_->push_send_off.back();
            if (np) k_remap_push<<<grid_for(np), kBlock, 0, s>>>(np, E_, inv.p, halo_->push_addr.p);
            PFDR_HIP(hipGetLastError());
            unsigned long long ni = 0;
            PFDR_HIP(hipMemcpyAsync(&ni, nint.p, sizeof(ni), hipMemcpyDeviceToHost, s));
            PFDR_HIP(hipStreamSynchronize(s));
            Eint_ = (long)ni;
            e_offset = 0;
        } else {
            k_edge_tile_order<<<grid_for(E), kBlock, 0, s>>>(E_, perm.p, eorig_.p, Eu_.p, Ev_.p,
                                                             nu.p, nv.p, eo.p, emap_.p);
            PFDR_HIP(hipGetLastError());
            PFDR_HIP(hipStreamSynchronize(s));
            Eint_ = E_;
        }
        std::swap(Eu_.p, nu.p);
        std::swap(Ev_.p, nv.p);
        std::swap(eorig_.p, eo.p);
        std::swap(eorig_.n, eo.n);
        eg_ptr = eorig_.p;
    }
    // contributions: local side-major [u ends | v ends] then the received tail
    const long R = halo_ ? halo_->R : 0;
    wz_.alloc(2 * E_ + R + kSlotGroup);  // (+kSlotGroup: tile_sum's whole groups)
    contribution_incidence(Eu_.p, Ev_.p, E_, V_, eg_ptr ? eg_ptr : eg.p, e_offset, halo_.get(),
                           inc_, s);
    eorig_.release();
    if (tiled_) build_tiles();
    else if (!tiny_) build_split();
}

// the runs of every vertex block of a tile-ordered graph and the slots of
// its contributions (see tile_sum)
template <typename real>
void QuadSession<real>::build_tiles() {
    hipStream_t s = stream;
    const long R = halo_ ? halo_->R : 0;
    {
        const long n = 2 * E_ + R, ng = n / kSlotGroup + 1;  // (+1: tile_sum's whole groups)
        DevBuf<unsigned short> d2(n);
        k_tile_slots<<<grid_for(V_), kBlock, 0, s>>>(V_, inc_.ptr.p, inc_.idx.p, d2.p);
        slots_.alloc(ng);
        k_pack_slots<<<grid_for(ng), kBlock, 0, s>>>(ng, n, d2.p, slots_.p);
        PFDR_HIP(hipGetLastError());
        build_tile_runs();
        build_patterns(d2.p, n);
    }  // (d2's block is reused only once the stream is idle, dev_free)
}

// the record and run tables of the tiled blocks (see tile_sum)
template <typename real>
void QuadSession<real>::build_tile_runs() {
    hipStream_t s = stream;
    const int nb = grid_for(V_);
    const long R = halo_ ? halo_->R : 0;
    luv_.alloc((size_t)E_);
    k_tile_luv<<<grid_for(E_), kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, luv_.p);
    {
        constexpr int EB = kBlock * Vec<real>::kPer16B;  // edges per k_edge_sweep_tl block
        const int neb = (int)((E_ + EB - 1) / EB);
        erec_.alloc((size_t)neb * kErec);
        k_tile_erec<<<(neb + kBlock / kWave - 1) / (kBlock / kWave), kBlock, 0, s>>>(
            E_, EB, 0, neb, Eu_.p, Ev_.p, erec_.p);
        PFDR_HIP(hipGetLastError());
    }
    ustart_.alloc((size_t)nb + 1);
    // u runs: the interior edges (sorted by u block); a partitioned rank's
    // boundary edges [Eint_, E) add their owned u ends as runs, its received
    // contributions theirs (k_tile_runs_count)
    k_tile_ustart<<<grid_for(Eint_ + 1), kBlock, 0, s>>>(Eint_, nb, Eu_.p, ustart_.p);
    DevBuf<int> cnt(nb), fill(nb);
    PFDR_HIP(hipMemsetAsync(cnt.p, 0, sizeof(int) * nb, s));
    PFDR_HIP(hipMemsetAsync(fill.p, 0, sizeof(int) * nb, s));
    struct Src { long n; const int *a; const unsigned long long *keys; long rs; };
    const Src src[3] = {{E_, Ev_.p, nullptr, 0},
                        {E_ - Eint_, Eu_.p + Eint_, nullptr, Eint_ - E_},
                        {R, nullptr, halo_ ? halo_->recv_keys.p : nullptr, E_}};
    for (const Src &q : src)
        if (q.n > 0) k_tile_runs_count<<<grid_for(q.n), kBlock, 0, s>>>(q.n, q.a, q.keys, V_, cnt.p);
    PFDR_HIP(hipGetLastError());
    std::vector<int> h(nb), tp((size_t)nb + 1, 0);
    PFDR_HIP(hipMemcpyAsync(h.data(), cnt.p, sizeof(int) * nb, hipMemcpyDeviceToHost, s));
    PFDR_HIP(hipStreamSynchronize(s));
    for (int b = 0; b < nb; b++) tp[b + 1] = tp[b] + h[b];
    const int nruns = tp[nb];
    tptr_.alloc((size_t)nb + 1);
    PFDR_HIP(hipMemcpyAsync(tptr_.p, tp.data(), sizeof(int) * (nb + 1), hipMemcpyHostToDevice, s));
    tstart_.alloc(nruns ? nruns : 1);
    tlen_.alloc(nruns ? nruns : 1);
    for (const Src &q : src)
        if (q.n > 0)
            k_tile_runs_fill<<<grid_for(q.n), kBlock, 0, s>>>(q.n, q.a, q.keys, V_, q.rs, tptr_.p,
                                                              fill.p, tstart_.p, tlen_.p);
    tok_.alloc(nb);
    k_tile_ok<<<grid_for(nb), kBlock, 0, s>>>(V_, nb, inc_.ptr.p, tptr_.p, kTileCap, tok_.p);
    trec_.alloc((size_t)nb * kTileRec);
    k_tile_rec<<<grid_for(nb), kBlock, 0, s>>>(nb, ustart_.p, tptr_.p, tstart_.p, tlen_.p, tok_.p,
                                               trec_.p);
    deg8_.alloc(V_);
    k_tile_deg<<<grid_for(V_), kBlock, 0, s>>>(V_, inc_.ptr.p, deg8_.p);
    PFDR_HIP(hipGetLastError());
    PFDR_HIP(hipMemcpyAsync(h.data(), tok_.p, sizeof(int) * nb, hipMemcpyDeviceToHost, s));
    PFDR_HIP(hipStreamSynchronize(s));
    long n = 0, nr = 0;
    for (int x : h) {
        n += x != 0;
        nr += x == 2;
    }
    tiled_blocks = n;
    record_blocks = nr;
    // the pair vertex sweep (k_vertex_sweep_pair): f32 sessions whose every
    // block is a record block, when two blocks' lists still leave LDS for
    // seven workgroups per CU (the kernel's seven waves per SIMD): C5 (6
    // entries per vertex) vertex sweep 3.15-3.22 -> 2.83-2.85 ms, C2 -2 %;
    // the headline's 12 per vertex would halve the resident workgroups
    // (0.174 -> 0.226 ms, f6j), so it keeps the one-block sweep.
    // PFDR_VPAIR=0: the one-block sweep throughout
    const char *e = getenv("PFDR_VPAIR");
    if (sizeof(real) == 4 && nr == nb && !(e && e[0] == '0')) {
        DevBuf<int> ent(nb);
        k_rec_entries<<<grid_for(nb), kBlock, 0, s>>>(V_, nb, inc_.ptr.p, tok_.p, ent.p);
        PFDR_HIP(hipGetLastError());
        PFDR_HIP(hipMemcpyAsync(h.data(), ent.p, sizeof(int) * nb, hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
        const int cap = std::max(1, *std::max_element(h.begin(), h.end()));
        const size_t per_wg = 2 * (size_t)cap * sizeof(real) + 2048;  // (+ the static arrays)
        if (per_wg * 7 <= 160 * 1024) vpair_cap_ = cap;
        vertex_pair = vpair_cap_;
    }
}

// Slot patterns (k_run_hash): when the record blocks' runs repeat a few
// slot sequences (regular grids), the distinct ones go to a small table
// (ptab_) and each block's runs point into it (prec_), so the vertex sweep
// streams no per-entry slots; runs that hash alike are verified equal
// entry by entry (k_run_verify) before the table is used.  Off when the
// patterns do not repeat (the jittered headline) or PFDR_TILE_PATTERNS=0.
template <typename real>
void QuadSession<real>::build_patterns(const unsigned short *d2, long n) {
    const char *e = getenv("PFDR_TILE_PATTERNS");
    if ((e && e[0] == '0') || !record_blocks) return;
    hipStream_t s = stream;
    const int nb = grid_for(V_);
    const long nr = (long)nb * kPrec;
    std::vector<unsigned long long> hh(nr);
    std::vector<int> rec((size_t)nb * kTileRec);
    {
        DevBuf<unsigned long long> h(nr);
        k_run_hash<<<grid_for(nr), kBlock, 0, s>>>(nb, E_, tok_.p, trec_.p, d2, h.p);
        PFDR_HIP(hipGetLastError());
        PFDR_HIP(hipMemcpyAsync(hh.data(), h.p, sizeof(unsigned long long) * nr,
                                hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipMemcpyAsync(rec.data(), trec_.p, sizeof(int) * rec.size(),
                                hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
    }
    constexpr size_t kMaxPatterns = 65536;
    std::unordered_map<unsigned long long, int> pat;
    std::vector<long long> pA;
    std::vector<int> pLen, pOff, prec(nr, 0);
    std::vector<long long> repA(nr, -1);
    long groups = 0;
    for (long id = 0; id < nr; id++) {
        if (hh[id] == ~0ull) continue;
        auto it = pat.find(hh[id]);
        int pi;
        if (it == pat.end()) {
            const int b = (int)(id / kPrec), q = (int)(id % kPrec);
            const int *r = &rec[(size_t)b * kTileRec];
            const long long A = q == 0 ? r[0] : E_ + r[1 + 2 * q];
            const int len = q == 0 ? r[1] : r[2 + 2 * q];
            pi = (int)pA.size();
            pat.emplace(hh[id], pi);
            pA.push_back(A);
            pLen.push_back(len);
            pOff.push_back((int)groups);
            groups += ((A & 7) + len + 7) / 8;
            if (pat.size() > kMaxPatterns || groups * kSlotGroup > n / 4) return;  // no repeats
        } else {
            pi = it->second;
        }
        prec[id] = pOff[pi];
        repA[id] = pA[pi];
    }
    if (!groups) return;
    {   // same hash, same slots: checked entry by entry on the device
        DevBuf<long long> dr(nr);
        DevBuf<int> bad(1);
        PFDR_HIP(hipMemcpyAsync(dr.p, repA.data(), sizeof(long long) * nr, hipMemcpyHostToDevice, s));
        PFDR_HIP(hipMemsetAsync(bad.p, 0, sizeof(int), s));
        k_run_verify<<<grid_for(nr), kBlock, 0, s>>>(nb, E_, tok_.p, trec_.p, d2, dr.p, bad.p);
        PFDR_HIP(hipGetLastError());
        int hb = 1;
        PFDR_HIP(hipMemcpyAsync(&hb, bad.p, sizeof(int), hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
        if (hb) return;
    }
    // the table: each pattern's groups packed from its representative's
    // slots (12 bits each, as k_pack_slots; entries outside the run are 0)
    std::vector<Slots12> tab((size_t)groups);
    std::vector<unsigned short> sl;
    for (size_t pi = 0; pi < pA.size(); pi++) {
        const long long A = pA[pi], g0 = A / kSlotGroup;
        const int len = pLen[pi];
        const long gn = ((A & 7) + len + 7) / 8;
        if (!gn) continue;
        sl.assign((size_t)gn * kSlotGroup, 0);
        PFDR_HIP(hipMemcpy(sl.data() + (A - g0 * kSlotGroup), d2 + A, sizeof(unsigned short) * len,
                           hipMemcpyDeviceToHost));
        for (long g = 0; g < gn; g++) {
            unsigned long long lo = 0, hi = 0;
            for (int q = 0; q < kSlotGroup; q++) {
                const unsigned long long x = sl[(size_t)g * kSlotGroup + q] & 0xfffu;
                const int bit = 12 * q;
                if (bit + 12 <= 64) lo |= x << bit;
                else if (bit >= 64) hi |= x << (bit - 64);
                else { lo |= x << bit; hi |= x >> (64 - bit); }
            }
            Slots12 &t = tab[(size_t)pOff[pi] + g];
            t.w[0] = (unsigned)lo;
            t.w[1] = (unsigned)(lo >> 32);
            t.w[2] = (unsigned)hi;
        }
    }
    ptab_.alloc((size_t)groups);
    prec_.alloc((size_t)nr);
    PFDR_HIP(hipMemcpyAsync(ptab_.p, tab.data(), sizeof(Slots12) * groups, hipMemcpyHostToDevice, s));
    PFDR_HIP(hipMemcpyAsync(prec_.p, prec.data(), sizeof(int) * nr, hipMemcpyHostToDevice, s));
    PFDR_HIP(hipStreamSynchronize(s));
    slot_patterns = (int64_t)pA.size();
}

// Split incidence for the vertex sweep (split_sum): when the edges are
// sorted by their u end (natural emission order, relabelled sessions), each
// vertex's u-end contributions are a contiguous run of wz and need no
// address.  Blocks that do not qualify keep the CSR gather.
template <typename real>
void QuadSession<real>::build_split() {
    if (!E_) return;
    hipStream_t s = stream;
    DevBuf<unsigned long long> bad(1);
    PFDR_HIP(hipMemsetAsync(bad.p, 0, sizeof(unsigned long long), s));
    k_u_order_check<<<grid_for(E_), kBlock, 0, s>>>(E_, V_, Eu_.p, bad.p);
    PFDR_HIP(hipGetLastError());
    unsigned long long nbad = 0;
    PFDR_HIP(hipMemcpyAsync(&nbad, bad.p, sizeof(nbad), hipMemcpyDeviceToHost, s));
    PFDR_HIP(hipStreamSynchronize(s));
    if (nbad) return;
    const int nb = grid_for(V_);
    const long ototal = inc_.n - E_;  // every local edge's u end is an owned row
    if (ototal < 0) return;
    uptr_.alloc((size_t)V_ + 1);
    k_uptr<<<grid_for(E_ + 1), kBlock, 0, s>>>(E_, V_, Eu_.p, uptr_.p);
    PFDR_HIP(hipGetLastError());
    ustaged = us_ ? 1 : 0;
    mask_.alloc(V_);
    oidx_.alloc(ototal ? ototal : 1);
    blkok_.alloc(nb);
    k_split_build<<<nb, kBlock, 0, s>>>(V_, E_, inc_.ptr.p, inc_.idx.p, uptr_.p, ototal, mask_.p,
                                        oidx_.p, blkok_.p, GatherCap<real>::v / 2);
    PFDR_HIP(hipGetLastError());
    std::vector<int> h(nb);
    PFDR_HIP(hipMemcpyAsync(h.data(), blkok_.p, nb * sizeof(int), hipMemcpyDeviceToHost, s));
    PFDR_HIP(hipStreamSynchronize(s));
    long n = 0;
    for (int x : h) n += x;
    split_blocks = n;
    if (!n) { mask_.release(); oidx_.release(); blkok_.release(); }  // uptr_ serves the edge sweep
    ustaged = us_ ? 1 : 0;
}

template <typename real>
void QuadSession<real>::push_ctrl() {
    PFDR_HIP(hipMemcpyAsync(ctrl_.p, hctrl_, sizeof(Ctrl<real>), hipMemcpyHostToDevice, stream));
}
template <typename real>
void QuadSession<real>::pull_ctrl() {
    PFDR_HIP(hipMemcpyAsync(hctrl_, ctrl_.p, sizeof(Ctrl<real>), hipMemcpyDeviceToHost, stream));
    wait_stream();
}

// host wait for the session stream; partitioned sessions wait under the
// transport's watchdog (a stalled halo exchange fails the call with the
// rank, peers, bytes and iteration instead of hanging)
template <typename real>
void QuadSession<real>::wait_stream() {
    if (!halo_) { PFDR_HIP(hipStreamSynchronize(stream)); return; }
    halo_->tr->phase = "iterations";
    halo_->tr->iteration = it_;
    halo_->tr->wait(stream);
}

// R = Y - A X (direct mode), gated
template <typename real>
void QuadSession<real>::gemv_rows(int gate) {
    hipStream_t s = stream;
    ProfScope ps(prof, "gemv_rows", s);
    if (exact_) {
        k_rows_seq<real><<<grid_for(N_), kBlock, 0, s>>>(N_, V_, A_.p, xp_.p, Y_.p, R_.p,
                                                        gate ? ctrl_.p : nullptr, gate);
        PFDR_HIP(hipGetLastError());
        return;
    }
    k_rows_partial<real><<<rows_nb_, kBlock, 0, s>>>(N_, V_, A_.p, xp_.p, rows_cpb_, Rpart_.p,
                                                    gate ? ctrl_.p : nullptr, gate);
    const Ctrl<real> *c = gate ? ctrl_.p : nullptr;
    if (!halo_) {
        k_rows_finish<real><<<grid_for(N_), kBlock, 0, s>>>(N_, rows_nb_, Rpart_.p, Y_.p, R_.p,
                                                           c, gate);
    } else {  // partial A X of this rank's columns, summed over the ranks
        k_rows_finish<real><<<grid_for(N_), kBlock, 0, s>>>(N_, rows_nb_, Rpart_.p, nullptr,
                                                           Rsum_.p, c, gate);
        halo_->tr->allreduce_sum(Rsum_.p, N_, dtype_of<real>(), s);
        k_rows_residual<real><<<grid_for(N_), kBlock, 0, s>>>(N_, Y_.p, Rsum_.p, R_.p, c, gate);
    }
    PFDR_HIP(hipGetLastError());
}

// forward step of the dense modes: P = 2X - Ga (A^t A X - A^t Y)
template <typename real>
void QuadSession<real>::forward_dense(int gate) {
    hipStream_t s = stream;
    ColArgs<real> ca{};
    ca.A = A_.p; ca.ncols = V_; ca.xp = xp_.p; ca.Ga = Ga_.p; ca.Y = Y_.p;
    ca.ctrl = gate ? ctrl_.p : nullptr;
    ca.gate = gate;
    if (mode_ == A_DIRECT) {
        // the residual is also what the objective needs
        gemv_rows(gate == GATE_NONE ? GATE_NONE : (rec_obj_ ? GATE_ACTIVE_OR_OBJ : GATE_ACTIVE));
        ca.len = N_; ca.w = R_.p;
        ProfScope ps(prof, "gemv_cols", s);
        col_product<EPI_FWD_DIRECT>(ca);
    } else {
        ca.w = full_x();
        ProfScope ps(prof, "symv", s);
        ata_product<EPI_FWD_ATA>(ca);
    }
    PFDR_HIP(hipGetLastError());
}

template <typename real>
const real *QuadSession<real>::full_x() {
    hipStream_t s = stream;
    k_x_extract<real><<<grid_for(V_), kBlock, 0, s>>>(V_, xp_.p, xfull_.p + v0_);
    PFDR_HIP(hipGetLastError());
    if (halo_) {  // all-gather of the owned blocks
        Transport &tr = *halo_->tr;
        const int n = tr.nranks;
        std::vector<const void *> sp(n, xfull_.p + v0_);
        std::vector<size_t> sb(n, (size_t)V_ * sizeof(real));
        std::vector<void *> rp(n);
        std::vector<size_t> rb(n);
        for (int q = 0; q < n; q++) {
            rp[q] = xfull_.p + halo_->off[q];
            rb[q] = (size_t)(halo_->off[q + 1] - halo_->off[q]) * sizeof(real);
        }
        tr.exchange(sp, sb, rp, rb, s);
    }
    return xfull_.p;
}

// (A^tA) w of the owned columns with epilogue EPI: block upper triangle when
// symv_ (one GPU, exactly symmetric matrix), else one wave per column
template <typename real>
template <int EPI>
void QuadSession<real>::ata_product(ColArgs<real> ca) {
    hipStream_t s = stream;
    ca.A = A_.p; ca.ncols = V_; ca.len = (int)Vglob_;
    if (exact_) {
        col_product<EPI>(ca);
    } else if (symv_) {
        const long nt = (long)snb_ * (snb_ + 1) / 2;
        k_symv_tiles<real><<<nt, kBlock, 0, s>>>(V_, A_.p, ca.w, spart_.p, ca.ctrl, ca.gate);
        k_symv_finish<real, EPI><<<(V_ + 63) / 64, kBlock, 0, s>>>(snb_, spart_.p, ca);
    } else {
        k_col_dot<real, EPI><<<grid_for((long)V_ * 64), kBlock, 0, s>>>(ca);
    }
    PFDR_HIP(hipGetLastError());
}

// column dots with epilogue EPI: sequential order (exact_) or one wave per column
template <typename real>
template <int EPI>
void QuadSession<real>::col_product(ColArgs<real> ca) {
    hipStream_t s = stream;
    if (exact_)
        k_col_seq<real, EPI><<<grid_for(ca.ncols), kBlock, 0, s>>>(ca);
    else
        k_col_dot<real, EPI><<<grid_for((long)ca.ncols * 64), kBlock, 0, s>>>(ca);
    PFDR_HIP(hipGetLastError());
}

// symmetric products for V >= 4 T: one GPU, V a multiple of the 16-byte
// vector, A 16-byte aligned, and the caller's matrix exactly symmetric
// (k_sym_check, one pass at setup; a matrix that is not keeps the column
// dots, which read it as given)
template <typename real>
void QuadSession<real>::plan_symv() {
    using S = SymT<real>;
    if (halo_ || exact_ || V_ < 4 * S::T) return;
    if (V_ % S::VW || ((uintptr_t)A_.p % 16)) return;
    hipStream_t s = stream;
    DevBuf<int> flag(1);
    PFDR_HIP(hipMemsetAsync(flag.p, 0, sizeof(int), s));
    const long n64 = (V_ + 63) / 64;
    k_sym_check<real><<<n64 * (n64 + 1) / 2, kBlock, 0, s>>>(V_, A_.p, flag.p);
    PFDR_HIP(hipGetLastError());
    int f = 1;
    PFDR_HIP(hipMemcpyAsync(&f, flag.p, sizeof(int), hipMemcpyDeviceToHost, s));
    PFDR_HIP(hipStreamSynchronize(s));
    if (f) return;
    symv_ = true;
    snb_ = (V_ + S::T - 1) / S::T;
    spart_.alloc((size_t)snb_ * V_);
    symv = 1;
}

// gradient of the smooth part at the current X into grad_ (reconditioning)
template <typename real>
void QuadSession<real>::gradient() {
    hipStream_t s = stream;
    grad_.alloc(Vg_);
    if (mode_ == A_IDENT || mode_ == A_DIAG) {
        k_grad_vertex<real><<<grid_for(V_), kBlock, 0, s>>>(V_, mode_, A_.p, Y_.p, xp_.p, grad_.p);
    } else {
        ColArgs<real> ca{};
        ca.A = A_.p; ca.ncols = V_; ca.out = grad_.p; ca.Y = Y_.p;
        if (mode_ == A_DIRECT) {
            gemv_rows(GATE_NONE);
            ca.len = N_; ca.w = R_.p;
            col_product<EPI_GRAD_DIRECT>(ca);
        } else {
            ca.w = full_x();
            ata_product<EPI_GRAD_ATA>(ca);
        }
    }
    PFDR_HIP(hipGetLastError());
}

// amplitude scale c of the preconditioner (ref :124-154): the sum of |a| is
// sequential in global vertex order across the ranks (chain)
template <typename real>
void QuadSession<real>::amplitude(bool init) {
    hipStream_t s = stream;
    if (init && mode_ == A_DIRECT) {
        ColArgs<real> ca{};
        ca.A = A_.p; ca.ncols = V_; ca.len = N_; ca.w = Y_.p; ca.out = pre_.p; ca.div = diag_.p;
        col_product<EPI_DIV>(ca);
    }
    k_amp<real><<<nbv_, kBlock, 0, s>>>(V_, init ? (mode_ == A_DIRECT ? 1 : 0) : 2, Y_.p, diag_.p,
                                        pre_.p, xp_.p, absval_.p, cnt_part_.p);
    PFDR_HIP(hipGetLastError());
    if (halo_ && lab_.p) {
        // relabelled partition: every rank holds the amplitudes of all
        // vertices at the caller's labels (one writer per position, so the
        // all-reduce adds zeros only) and sums them in that order
        Transport &tr = *halo_->tr;
        if (ampg_.n < (size_t)Vglob_) ampg_.alloc(Vglob_);
        PFDR_HIP(hipMemsetAsync(ampg_.p, 0, sizeof(real) * Vglob_, s));
        k_scatter<real><<<nbv_, kBlock, 0, s>>>(V_, absval_.p, lab_.p, ampg_.p);
        PFDR_HIP(hipGetLastError());
        tr.allreduce_sum(ampg_.p, (int)Vglob_, dtype_of<real>(), s);
        if (mono_ws_.n < mono_ws_bytes<real>(Vglob_)) mono_ws_.alloc(mono_ws_bytes<real>(Vglob_));
        mono_sum<real>(Vglob_, ampg_.p, nullptr, nbv_, cnt_part_.p, csum_.p, ccnt_.p, mono_ws_.p,
                       s);
        tr.allreduce_sum(ccnt_.p, 1, 2, s);
        k_set_c<real><<<1, 64, 0, s>>>(csum_.p, ccnt_.p, init ? 1 : 0, ctrl_.p);
        PFDR_HIP(hipGetLastError());
        return;
    }
    const bool seeded = halo_ && halo_->tr->rank > 0;
    if (halo_) halo_->tr->chain_recv(red_.p + 3, sizeof(real), s);
    const real *amp = absval_.p;
    if (reordered_) {  // the reference's sequential sum runs in the caller's labels
        k_gather<real><<<nbv_, kBlock, 0, s>>>(V_, absval_.p, where_.p, amp_orig_.p);
        amp = amp_orig_.p;
    }
    if (mono_ws_.n < mono_ws_bytes<real>(V_)) mono_ws_.alloc(mono_ws_bytes<real>(V_));
    mono_sum<real>(V_, amp, seeded ? red_.p + 3 : nullptr, nbv_, cnt_part_.p, csum_.p, ccnt_.p,
                   mono_ws_.p, s);
    PFDR_HIP(hipGetLastError());
    if (halo_) {
        Transport &tr = *halo_->tr;
        tr.chain_send(csum_.p, sizeof(real), s);
        tr.broadcast(csum_.p, sizeof(real), tr.nranks - 1, s);
        tr.allreduce_sum(ccnt_.p, 1, 2, s);
    }
    k_set_c<real><<<1, 64, 0, s>>>(csum_.p, ccnt_.p, init ? 1 : 0, ctrl_.p);
    PFDR_HIP(hipGetLastError());
}

// ref :57-268 (l1) / bounds :58-242
template <typename real>
void QuadSession<real>::precondition(bool init) {
    hipStream_t s = stream;
    const size_t V = V_;
    ProfScope ps(prof, init ? "precondition" : "recondition", s);
    amplitude(init);
    if (!init) {
        gradient();
        pull(xp_.p, sizeof(R2<real>));  // X at the ghosts
        pull(grad_.p, sizeof(real));
    }
    const bool first_recond = !init && !A1_.p;
    if (first_recond) A1_.alloc(E_ ? E_ : 1);  // a_e leave cw La_d1 for good
    if (E_) {
        k_d1_weights<real><<<nbe_, kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, La_d1_.p, ctrl_.p, init ? 1 : 0,
                                                   condMin_, xp_.p, first_recond ? nullptr : A1_.p,
                                                   cw_, invAux_.p, A1_.p, wz_.p, Ga_.p, grad_.p,
                                                   Z2_.p, zs_);
        PFDR_HIP(hipGetLastError());
    }
    if (halo_) halo_->push(wz_.p, wz_.p + 2 * E_, sizeof(real), s);
    k_precond_vertex<real><<<nbv_, kBlock, 0, s>>>(V_, inc_.ptr.p, inc_.idx.p, wz_.p, diag_.p,
                                                   La_l1_.p, xp_.p, ctrl_.p, init ? 1 : 0, condMin_,
                                                   cap_, Ldiag_ ? L_.p : nullptr, Ga_.p,
                                                   invAux_.p, Th_l1_.p);
    PFDR_HIP(hipGetLastError());
    pull(Ga_.p, sizeof(real));
    pull(invAux_.p, sizeof(real));
    if (E_ && !init) {
        k_recond_edge<real><<<nbe_, kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, A1_.p, invAux_.p, Ga_.p,
                                                    xp_.p, grad_.p, Z2_.p, zs_);
    }
    k_gi_pack<real><<<grid_for(Vg_), kBlock, 0, s>>>(Vg_, Ga_.p, invAux_.p, gi_.p);
    PFDR_HIP(hipGetLastError());
    if (!init && !rat() && rr_.p) {  // (A1 from the first reconditioning on)
        rr_.release();
        edge_ratio = 0;
    }
    if (!init) {
        // forward step with the new metric from the gradient taken before
        // reconditioning (ref :448-464)
        k_forward_grad<real><<<grid_for(V), kBlock, 0, s>>>(V_, Ga_.p, grad_.p, xp_.p);
        PFDR_HIP(hipGetLastError());
        grad_.release();
    }
}

// objective at the current iterate (ref :387-422), written at Obj[it]
template <typename real>
void QuadSession<real>::objective() {
    hipStream_t s = stream;
    const Ctrl<real> *c = ctrl_.p;
    const real *papp = nullptr;
    pull(xp_.p, sizeof(R2<real>));  // TV of boundary edges needs the ghosts' X
    if (mode_ == A_ATA) {
        ColArgs<real> ca{};
        ca.out = pre_.p;
        ca.ctrl = c; ca.gate = GATE_OBJ;
        ca.w = full_x();
        ata_product<EPI_STORE>(ca);
        papp = pre_.p;
    }
    k_obj_vertex<real><<<nbv_, kBlock, 0, s>>>(V_, mode_, xp_.p, A_.p, papp, Y_.p,
                                               flavour_ == 0 ? La_l1_.p : nullptr, opart_.p, nbv_, c);
    if (E_) k_obj_edge<real><<<nbe_, kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, xp_.p, La_d1_.p, opart_.p + 2 * nbv_, c);
    // the residual is replicated on every rank: its norm counts once (rank 0)
    const int nbn = (halo_ && halo_->tr->rank != 0) ? 0 : nbn_;
    if (mode_ == A_DIRECT && nbn)
        k_obj_rsq<real><<<nbn, kBlock, 0, s>>>(N_, R_.p, opart_.p + 2 * nbv_ + nbe_, c);
    k_obj_reduce<real><<<1, kBlock, 0, s>>>(opart_.p, nbv_, E_ ? nbe_ : 0, nbn, mode_ == A_DIRECT,
                                            c, red_.p);
    if (halo_) halo_->tr->allreduce_sum(red_.p, 3, dtype_of<real>(), s);
    k_obj_write<real><<<1, 64, 0, s>>>(red_.p, mode_ == A_DIRECT,
                                       flavour_ == 0 && La_l1_.p != nullptr, ctrl_.p, Obj_.p);
    PFDR_HIP(hipGetLastError());
}

template <typename real>
void QuadSession<real>::edge_sweep(long ebeg, long eend, const Ctrl<real> *c, const char *name,
                                   long ebeg2, long eend2, const FuseDecide<real> *fd) {
    constexpr int EPT = Vec<real>::kPer16B;
    if (eend <= ebeg) { ebeg = ebeg2; eend = eend2; ebeg2 = eend2 = 0; }
    if (eend <= ebeg) return;
    hipStream_t s = stream;
    ProfScope ps(prof, name, s);
    ERange rg{ebeg, eend, ebeg2, eend2, grid_for(eend - ebeg, EPT)};
    const int nb = rg.nb0 + (eend2 > ebeg2 ? grid_for(eend2 - ebeg2, EPT) : 0);
    const int xm = xcd_fit(nb, xcd_e_), g = xcd_grid(nb, xm);
    const FuseDecide<real> f = fd ? *fd : FuseDecide<real>{};
    if (ends_ && fuse_) {  // the whole edge range (fused sessions sweep [0, E) in one launch)
        k_edge_sweep_ends<real><<<g, kBlock, 0, s>>>(E_, xpe_.p, gie_.p, Z2_.p, A1_.p, cw_,
                                                     la_it(), la0_, rho_, c, nb, xm, f, pad_out());
        return;
    }
    constexpr long EB = kBlock * EPT;  // edges per tiled edge-sweep block
    if (tiled_ && !fuse_ && rg.nb0 == nb && ebeg % EB == 0 && (eend % EB == 0 || eend == E_)) {
        // edge blocks [ebeg / EB, ...) of the tile order (a partitioned rank
        // sweeps its interior blocks and the rest in two launches)
        auto k = rr_.p ? k_edge_sweep_tl<real, true, true>
                 : (!la_it() && !A1_.p) ? k_edge_sweep_tl<real, true>
                                        : k_edge_sweep_tl<real, false>;
        k<<<g, kBlock, 0, s>>>(E_, V_, Eu_.p, luv_.p, erec_.p, Ev_.p, xr_, Z2_.p, A1_.p, cw_,
                               gi_.p, la_it(), la0_, zdirect() ? nullptr : wz_.p, rho_, c,
                               (int)(ebeg / EB), nb, xm, rr_.p);
        return;
    }
    if (tiled_) throw std::logic_error("tiled edge sweep: range not on edge blocks");
    if (us_ && uptr_.p) {
        auto k = fuse_ ? k_edge_sweep_us<real, true> : k_edge_sweep_us<real, false>;
        k<<<g, kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, uptr_.p, xr_, Z2_.p, A1_.p, cw_, gi_.p,
                               la_it(), la0_, wz_.p, rho_, c, nb, xm, rg, f, pad_out());
    } else {
        auto k = fuse_ ? k_edge_sweep<real, true> : k_edge_sweep<real, false>;
        k<<<g, kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, xr_, Z2_.p, A1_.p, cw_, gi_.p, la_it(), la0_,
                               wz_.p, rho_, c, nb, xm, rg, f, pad_out());
    }
}

template <typename real>
void QuadSession<real>::tiny_chunk(int n) {
    const bool gated = track_ || rec_obj_;
    TinyArgs<real> t{};
    t.E = E_; t.Eu = Eu_.p; t.Ev = Ev_.p; t.Z2 = Z2_.p; t.A1 = A1_.p; t.La_d1 = la_it();
    t.la0 = la0_; t.cw = cw_; t.rho = rho_; t.gi = gi_.p; t.wz = wz_.p;
    t.va = vargs(0, nbv_, nullptr);
    t.red = red_.p; t.ctrl = gated ? ctrl_.p : nullptr; t.Dif = rec_dif_ ? Dif_.p : nullptr;
    t.track = track_ ? 1 : 0; t.iters = n;
    ProfScope ps(prof, "tiny_iterate", stream);
    k_tiny_iterate<real><<<1, kTiny, 0, stream>>>(t);
    PFDR_HIP(hipGetLastError());
}

template <typename real>
VArgs<real> QuadSession<real>::vargs(int bbeg, int bend, const Ctrl<real> *c) {
    VArgs<real> a{};
    a.V = V_; a.ptr = inc_.ptr.p; a.idx = inc_.idx.p; a.xp = xr_; a.wz = wz_.p;
    a.xpo = xw_ == xr_ ? nullptr : xw_;
    a.uptr = uptr_.p; a.mask = mask_.p; a.oidx = oidx_.p; a.blkok = blkok_.p;
    a.Y = Y_.p; a.A = A_.p; a.Ga = Ga_.p; a.Th_l1 = Th_l1_.p;
    a.prox = prox_; a.positivity = positivity_; a.lo = lo_; a.hi = hi_;
    a.fwd = mode_ == A_IDENT ? 1 : (mode_ == A_DIAG ? 2 : 0);
    a.track = track_ ? 1 : 0; a.part = vpart_.p; a.ctrl = c;
    a.late = fuse_ ? 1 : 0;
    a.E = E_;
    if (tiled_) {
        a.slots = slots_.p; a.trec = trec_.p; a.ptab = ptab_.p; a.prec = prec_.p; a.deg8 = deg8_.p; a.ustart = ustart_.p; a.tptr = tptr_.p; a.tstart = tstart_.p;
        a.tlen = tlen_.p; a.tok = tok_.p;
        a.zs = Z2_.p; a.invAux = invAux_.p; a.a0 = cw_ * la0_;
        a.gi = gi_.p;  // (Ga, 1/Aux) in one load
    }
    a.l1uni = l1_uniform_ ? 1 : 0;
    a.l1u = l1u_;
    a.terms = seqdif_ ? terms_.p : nullptr;
    a.tmap = seqdif_ && reordered_ ? order_.p : nullptr;
    a.tstride = tstride_;
    a.bbeg = bbeg; a.nb = bend - bbeg; a.xcd = xcd_fit(a.nb, xcd_v_);
    a.bsplit = a.nb; a.bjump = 0;
    return a;
}

template <typename real>
void QuadSession<real>::vertex_sweep(int bbeg, int bend, const Ctrl<real> *c, const char *name,
                                     int bbeg2, int bend2) {
    if (bend <= bbeg) { bbeg = bbeg2; bend = bend2; bbeg2 = bend2 = 0; }
    if (bend <= bbeg) return;
    hipStream_t s = stream;
    VArgs<real> a = vargs(bbeg, bend, c);
    if (bend2 > bbeg2) {  // second range: logical blocks past the first jump to it
        a.bsplit = bend - bbeg;
        a.bjump = bbeg2 - bend;
        a.nb += bend2 - bbeg2;
        a.xcd = xcd_fit(a.nb, xcd_v_);
    }
    ProfScope ps(prof, name, s);
    if (pad_ && bend2 <= bbeg2) {
        k_vertex_sweep_pad<real><<<xcd_grid(a.nb, a.xcd), kBlock, 0, s>>>(
            a, wzp_.p, pad_nmax_, ends_ ? pidx_.p : nullptr, ends_ ? xpe_.p : nullptr);
        return;
    }
    if (vpair_cap_ && bend2 <= bbeg2 && a.nb >= 2) {  // pairs of record blocks, one range
        const int np = a.nb / 2;
        const size_t lb = 2 * (size_t)vpair_cap_ * sizeof(real);
        if (a.nb & 1) {  // the odd last block first, on its own
            VArgs<real> a1 = a;
            a1.bbeg = a.bbeg + a.nb - 1;
            a1.nb = 1;
            a1.bsplit = 1;
            a1.xcd = 0;
            if (zdirect()) k_vertex_sweep<real, 8, true><<<1, kBlock, 0, s>>>(a1);
            else k_vertex_sweep<real, 8><<<1, kBlock, 0, s>>>(a1);
        }
        a.xcd = xcd_fit(np, xcd_v_);
        const int g = xcd_grid(np, a.xcd);
        if (zdirect()) k_vertex_sweep_pair<real, true><<<g, kBlock, lb, s>>>(a, vpair_cap_);
        else k_vertex_sweep_pair<real><<<g, kBlock, lb, s>>>(a, vpair_cap_);
        return;
    }
    if (zdirect())
        k_vertex_sweep<real, 8, true><<<xcd_grid(a.nb, a.xcd), kBlock, 0, s>>>(a);
    else
        k_vertex_sweep<real, 8><<<xcd_grid(a.nb, a.xcd), kBlock, 0, s>>>(a);
}

// the sweeps of one iteration: (partitions) the ghosts' (X, P) pulled into
// the buffer the edge sweep reads (xr_), the edge sweep, the ghost ends'
// contributions pushed to their owners, the vertex sweep (into xw_)
template <typename real>
void QuadSession<real>::sweeps(const Ctrl<real> *c) {
    hipStream_t s = stream;
    if (overlap_) {
        // pull ghosts (comm) || interior edges; boundary edges; push (comm)
        // || interior vertices; boundary vertices
        PFDR_HIP(hipEventRecord(ev_[0], s));
        PFDR_HIP(hipStreamWaitEvent(comm_, ev_[0], 0));
        {
            ProfScope ps(prof, "halo_pull", comm_);
            halo_->pull(xr_, sizeof(R2<real>), comm_);
        }
        PFDR_HIP(hipEventRecord(ev_[1], comm_));
        edge_sweep(elo_, ehi_, c, "edge_sweep");
        PFDR_HIP(hipStreamWaitEvent(s, ev_[1], 0));
        edge_sweep(0, elo_, c, "edge_sweep_b", ehi_, E_);  // both boundary ranges, one launch
        PFDR_HIP(hipEventRecord(ev_[2], s));
        PFDR_HIP(hipStreamWaitEvent(comm_, ev_[2], 0));
        {
            ProfScope ps(prof, "halo_push", comm_);
            real *src = zdirect() ? Z2_.p : wz_.p;  // Z-direct ranks push Z
            halo_->push(src, src + 2 * E_, sizeof(real), comm_);
        }
        PFDR_HIP(hipEventRecord(ev_[3], comm_));
        vertex_sweep(blo_, bhi_, c, "vertex_sweep");
        PFDR_HIP(hipStreamWaitEvent(s, ev_[3], 0));
        vertex_sweep(0, blo_, c, "vertex_sweep_b", bhi_, nbv_);
    } else {
        if (halo_) {
            ProfScope ps(prof, "halo_pull", s);
            halo_->pull(xr_, sizeof(R2<real>), s);
        }
        edge_sweep(0, E_, c, "edge_sweep");
        if (halo_) {
            ProfScope ps(prof, "halo_push", s);
            real *src = zdirect() ? Z2_.p : wz_.p;  // Z-direct ranks push Z
            halo_->push(src, src + 2 * E_, sizeof(real), s);
        }
        vertex_sweep(0, nbv_, c, "vertex_sweep");
    }
}

// iteration t = it0_ + 1 + i of a speculative session (see spec_)
template <typename real>
void QuadSession<real>::body_spec(int i, int n) {
    hipStream_t s = stream;
    const int t = it0_ + 1 + i;
    const Ctrl<real> *c = ctrl_.p;
    const int b = t % sd_;
    if (i >= sd_) PFDR_HIP(hipStreamWaitEvent(s, evd_[b], 0));  // the decision on t - D
    xr_ = xpb(t - 1);
    xw_ = xpb(t);
    real *terms = terms_.p + (long)b * 2 * tstride_, *part = vpart_.p + (long)b * 2 * nbv_;
    real *const keep = terms_.p, *const keepp = vpart_.p;
    terms_.p = terms;  // vargs() hands the sweep this iteration's terms
    vpart_.p = part;
    sweeps(c);
    terms_.p = keep;
    vpart_.p = keepp;
    xr_ = xw_ = xp_.p;
    PFDR_HIP(hipEventRecord(evv_[b], s));
    const hipStream_t es = evs();
    PFDR_HIP(hipStreamWaitEvent(es, evv_[b], 0));
    seq_evolution(terms, part, es);  // overlaps the sweeps of t + 1 (not when serial)
    k_decide<real><<<1, 64, 0, es>>>(ctrl_.p, red_.p, rec_dif_ ? Dif_.p : nullptr, 1);
    PFDR_HIP(hipGetLastError());
    PFDR_HIP(hipEventRecord(evd_[b], es));
    if (i == n - 1) PFDR_HIP(hipStreamWaitEvent(s, evd_[b], 0));  // join: the chunk's last
}

template <typename real>
void QuadSession<real>::body(int i, int n) {
    hipStream_t s = stream;
    if (spec_) { body_spec(i, n); return; }
    const bool gated = track_ || rec_obj_;
    const Ctrl<real> *c = gated ? ctrl_.p : nullptr;
    if (fuse_) {
        // E(i) decides iteration i - 1 (from cb[(i-1)&1] into cb[i&1]), V(i)
        // reads cb[i&1]; the last body closes the chunk with k_reduce_decide's
        // arithmetic, its decision into ctrl_
        Ctrl<real> *cb[2] = {ctrl_.p, ctrl2_.p};
        FuseDecide<real> fd{};
        if (i > 0) {
            fd.src = cb[(i - 1) & 1]; fd.dst = cb[i & 1]; fd.part = vpart_.p;
            fd.red = red_.p; fd.Dif = rec_dif_ ? Dif_.p : nullptr; fd.nparts = nbv_;
        }
        edge_sweep(0, E_, cb[0], "edge_sweep", 0, 0, &fd);
        vertex_sweep(0, nbv_, cb[i & 1], "vertex_sweep");
        if (i == n - 1) {
            FuseDecide<real> fl{cb[i & 1], cb[0], vpart_.p, red_.p, rec_dif_ ? Dif_.p : nullptr,
                                nbv_};
            k_decide_fused<real><<<1, kBlock, 0, s>>>(fl);
        }
        PFDR_HIP(hipGetLastError());
        return;
    }
    sweeps(c);
    if (seqdif_) {
        // the reference's two sequential sums (ref :518-526), then its decision
        ProfScope ps(prof, "seq_evolution", s);
        seq_evolution(terms_.p, vpart_.p, s);
        k_decide<real><<<1, 64, 0, s>>>(ctrl_.p, red_.p, rec_dif_ ? Dif_.p : nullptr, 1);
    } else if (gated && !halo_) {
        k_reduce_decide<real><<<1, kBlock, 0, s>>>(nbv_, vpart_.p, red_.p, ctrl_.p,
                                                   rec_dif_ ? Dif_.p : nullptr, track_ ? 1 : 0);
    } else if (gated) {  // the partial sums are all-reduced before the decision
        if (track_) {
            k_reduce_pairs<real><<<1, kBlock, 0, s>>>(nbv_, vpart_.p, red_.p, 1);
            halo_->tr->allreduce_sum(red_.p, 2, dtype_of<real>(), s);
        }
        k_decide<real><<<1, 64, 0, s>>>(ctrl_.p, red_.p, rec_dif_ ? Dif_.p : nullptr, track_ ? 1 : 0);
    }
    PFDR_HIP(hipGetLastError());
    if (mode_ == A_DIRECT || mode_ == A_ATA) forward_dense(gated ? GATE_ACTIVE : GATE_NONE);
    if (rec_obj_) objective();
}

// red_[0..2) = the sums of (X_ - X)^2 and X^2 over every vertex in the
// caller's order, rounded as the reference's one-thread loop.  part: the
// vertex sweep's per-block sums of the same terms (their binades predicted
// from them when the terms lie in vertex order)
template <typename real>
void QuadSession<real>::seq_evolution(real *terms, const real *part, hipStream_t s) {
    const int *halt = &ctrl_.p->halt;
    if (!halo_) {
        mono_sum<real>(V_, terms, nullptr, 0, nullptr, red_.p, nullptr, dws_.p, s, 2, tstride_,
                       halt, reordered_ ? nullptr : part, nbv_);
    } else if (!lab_.p) {
        chain_.run(etr(), terms, tstride_, red_.p, halt, s);
    } else {
        route_.run(etr(), terms, tstride_, red_.p, halt, s);
    }
}

// interior edge range and vertex-block range of a partitioned session (the
// longest runs without ghost endpoints / received contributions); edges
// outside [elo_, ehi_) and blocks outside [blo_, bhi_) wait for the halo
template <typename real>
void QuadSession<real>::plan_overlap() {
    hipStream_t s = stream;
    constexpr int EPT = Vec<real>::kPer16B;
    // edges: a ghost endpoint (u is always owned; v may be a ghost)
    std::vector<int> hv(E_);
    if (E_) PFDR_HIP(hipMemcpy(hv.data(), Ev_.p, E_ * 4, hipMemcpyDeviceToHost));
    long best0 = 0, best1 = 0;
    for (long e = 0; e < E_;) {
        if (hv[e] >= V_) { e++; continue; }
        long f = e;
        while (f < E_ && hv[f] < V_) f++;
        if (f - e > best1 - best0) { best0 = e; best1 = f; }
        e = f;
    }
    // both cuts on the lane width: every launch starts vector-aligned
    elo_ = ((best0 + EPT - 1) / EPT) * EPT;
    ehi_ = std::max(elo_, (best1 / EPT) * EPT);
    if (tiled_) {  // tile order: the interior edges come first, cut on whole edge blocks
        constexpr long EB = kBlock * EPT;
        elo_ = 0;
        ehi_ = (Eint_ / EB) * EB;
    }
    // vertex blocks: any CSR entry from the received tail
    std::vector<int> ptr(V_ + 1);
    std::vector<unsigned> idx(inc_.n);
    PFDR_HIP(hipMemcpy(ptr.data(), inc_.ptr.p, (V_ + 1) * 4, hipMemcpyDeviceToHost));
    if (inc_.n) PFDR_HIP(hipMemcpy(idx.data(), inc_.idx.p, inc_.n * 4, hipMemcpyDeviceToHost));
    int b0 = 0, b1 = 0;
    for (int b = 0; b < nbv_;) {
        auto tailblk = [&](int q) {
            const int v0 = q * kBlock, v1 = std::min(V_, v0 + kBlock);
            for (int j = ptr[v0]; j < ptr[v1]; j++)
                if (idx[j] >= (unsigned)(2 * E_)) return true;
            return false;
        };
        if (tailblk(b)) { b++; continue; }
        int f = b;
        while (f < nbv_ && !tailblk(f)) f++;
        if (f - b > b1 - b0) { b0 = b; b1 = f; }
        b = f;
    }
    blo_ = b0;
    bhi_ = b1;
    PFDR_HIP(hipStreamCreateWithFlags(&comm_, hipStreamNonBlocking));
    for (hipEvent_t &e : ev_) PFDR_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    overlap_ = true;
    interior_edges = ehi_ - elo_;
    (void)s;
}

// the captured graph of n bodies (a whole chunk, or a run's tail after
// prepare()), instantiated once -- at the end of the setup for chunk_, and
// again after a reconditioning dropped them
template <typename real>
hipGraphExec_t QuadSession<real>::chunk_graph(int n) {
    const int key = kSpecMax * n + (spec_ ? it0_ % sd_ : 0);  // speculative: X buffers by t mod D
    auto it = graphs_.find(key);
    if (it != graphs_.end()) return it->second;
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    PFDR_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    try {
        for (int i = 0; i < n; i++) body(i, n);
    } catch (...) {
        (void)hipStreamEndCapture(stream, &g);
        if (g) (void)hipGraphDestroy(g);
        throw;
    }
    PFDR_HIP(hipStreamEndCapture(stream, &g));
    const hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    PFDR_HIP(e);
    // uploaded now, so that its first replay (a timed run's, after
    // prepare()) pays no upload: the driver's 20-step line 0.522 -> 0.517 ms
    PFDR_HIP(hipGraphUpload(ge, stream));
    graphs_.emplace(key, ge);
    return ge;
}

// whole chunks replay the captured graph; a partial chunk (the tail of a
// run) replays one only if prepare() built it, else it is launched directly
// rather than captured for one use
template <typename real>
void QuadSession<real>::run_bodies(int n) {
    it0_ = it_;
    const int key = kSpecMax * n + (spec_ ? it0_ % sd_ : 0);
    if (!prof.on && capturable_ && graphs_.count(key)) {
        PFDR_HIP(hipGraphLaunch(graphs_[key], stream));
        return;
    }
    if (!graphs_ok_ || prof.on || n != chunk_) {
        for (int i = 0; i < n; i++) body(i, n);
        return;
    }
    PFDR_HIP(hipGraphLaunch(chunk_graph(chunk_), stream));
}

// the graphs a run of `iters` iterations will replay (chunks of chunk_ and
// the tail), built now so that the run itself launches no capture
template <typename real>
void QuadSession<real>::prepare(int iters) {
    if (!capturable_ || iters <= 0) return;
    it0_ = it_;  // (the run starts here: its parity)
    if (iters >= chunk_) (void)chunk_graph(chunk_);
    if (iters % chunk_) (void)chunk_graph(iters % chunk_);
    PFDR_HIP(hipStreamSynchronize(stream));
}

template <typename real>
void QuadSession<real>::print_progress() {
    if (halo_ && halo_->tr->rank != 0) return;
    printf("iteration %d (max. %d)\n", it_, itMax_);
    if (track_) {
        printf("iterate evolution %g (recond. %g; tol. %g)\n", (double)hctrl_->dif,
               (double)hctrl_->difRcd, (double)hctrl_->difTol);
    }
    fflush(stdout);
}

template <typename real>
int QuadSession<real>::run(int iters) {
    const bool gated = track_ || rec_obj_;
    const int target = (int)std::min<long>((long)it_ + std::max(iters, 0), (long)itMax_);
    if (gated && !halo_ && !spec_) return run_pipelined(target);
    // every rank runs the same number of bodies: the decisions come from
    // all-reduced values, so the control blocks agree
    while (!stopped_ && it_ < target) {
        const int n = std::min(target - it_, chunk_);
        if (tiny_) tiny_chunk(n);
        else run_bodies(n);
        if (gated) {
            pull_ctrl();
            it_ = hctrl_->it;
            if (hctrl_->stop) {
                stopped_ = true;
            } else if (hctrl_->recond) {
                if (verbose_) { print_progress(); printf("Reconditioning... "); fflush(stdout); }
                precondition(false);
                refresh_ends();  // (X, P) and (Ga, 1/Aux) rewritten
                drop_graphs();  // A1_ now holds the splitting weights' factors
                difRcd2_ *= real(0.01);  // ref :458
                hctrl_->difRcd = difRcd2_;
                hctrl_->recond = 0;
                hctrl_->halt = 0;
                push_ctrl();
                if (verbose_) { printf("done.\n"); fflush(stdout); }
            }
        } else {
            it_ += n;
            if (it_ >= itMax_) stopped_ = true;
        }
        if (verbose_ && (it_ >= next_print_ || stopped_)) {
            if (!gated) hctrl_->it = it_;
            print_progress();
            next_print_ = it_ + verbose_;
        }
    }
    wait_stream();
    if (prof.on) prof.resolve();
    return it_;
}

// Gated single-GPU runs: chunk k + 1 is launched before the host reads the
// control block chunk k left (a device-to-host snapshot ordered between the
// two chunks), so the host's round trip -- ≈35-45 us per chunk, a tenth of
// a 32-iteration chunk of C1 -- overlaps the GPU's work instead of idling
// it.  A chunk launched after a stop or a reconditioning request runs with
// the halt flag set: every kernel of it returns at once and changes nothing,
// so the iterates, the iteration count and Dif are those of the one-chunk-
// at-a-time loop.
template <typename real>
int QuadSession<real>::run_pipelined(int target) {
    for (int k = 0; k < 2; k++) {
        if (!snap_[k]) snap_[k] = static_cast<Ctrl<real> *>(pinned_small_get());
        if (!snapev_[k]) PFDR_HIP(hipEventCreateWithFlags(&snapev_[k], hipEventDisableTiming));
    }
    int k = 0, nq = 0;  // slot of the oldest unread snapshot, chunks in flight
    int ahead = it_;    // iterations launched so far, if none stops
    while (!stopped_) {
        while (nq < 2 && ahead < target) {
            const int n = std::min(target - ahead, chunk_);
            if (tiny_) tiny_chunk(n);
            else run_bodies(n);
            const int slot = (k + nq) & 1;
            PFDR_HIP(hipMemcpyAsync(snap_[slot], ctrl_.p, sizeof(Ctrl<real>),
                                    hipMemcpyDeviceToHost, stream));
            PFDR_HIP(hipEventRecord(snapev_[slot], stream));
            ahead += n;
            nq++;
        }
        if (nq == 0) break;
        PFDR_HIP(hipEventSynchronize(snapev_[k]));
        *hctrl_ = *snap_[k];
        k ^= 1;
        nq--;
        it_ = hctrl_->it;
        if (hctrl_->stop) {
            stopped_ = true;
        } else if (hctrl_->recond) {
            wait_stream();  // the chunk queued behind it ran halted
            nq = 0;
            ahead = it_;
            if (verbose_) { print_progress(); printf("Reconditioning... "); fflush(stdout); }
            precondition(false);
            refresh_ends();
            drop_graphs();
            difRcd2_ *= real(0.01);  // ref :458
            hctrl_->difRcd = difRcd2_;
            hctrl_->recond = 0;
            hctrl_->halt = 0;
            push_ctrl();
            if (verbose_) { printf("done.\n"); fflush(stdout); }
        }
        if (verbose_ && (it_ >= next_print_ || stopped_)) {
            print_progress();
            next_print_ = it_ + verbose_;
        }
        if (!stopped_ && nq == 0 && ahead >= target) break;
    }
    wait_stream();
    if (prof.on) prof.resolve();
    return it_;
}

template <typename real>
void *QuadSession<real>::device_x() {
    if (xout_.n < (size_t)V_) xout_.alloc(V_);
    if (reordered_)
        k_x_extract_perm<real><<<grid_for(V_), kBlock, 0, stream>>>(V_, xpb(it_), where_.p,
                                                                    xout_.p);
    else
        k_x_extract<real><<<grid_for(V_), kBlock, 0, stream>>>(V_, xpb(it_), xout_.p);
    PFDR_HIP(hipGetLastError());
    PFDR_HIP(hipStreamSynchronize(stream));
    return xout_.p;
}

template <typename real>
void QuadSession<real>::result(void *X_host, int *it, void *Obj_host, void *Dif_host) {
    hipStream_t s = stream;
    HostPins hp(s);
    if (X_host) {
        void *dx = device_x();
        hp.copy(X_host, dx, sizeof(real) * V_, hipMemcpyDeviceToHost);
    }
    if (it) *it = it_;
    if (Obj_host && rec_obj_)
        hp.copy(Obj_host, Obj_.p, sizeof(real) * (it_ + 1), hipMemcpyDeviceToHost);
    if (Dif_host && rec_dif_ && it_ > 0)
        hp.copy(Dif_host, Dif_.p, sizeof(real) * it_, hipMemcpyDeviceToHost);
    hp.release();
    PFDR_HIP(hipStreamSynchronize(s));
}

SessionBase *create_quadratic_session(const pfdr_problem *p) {
    if (p->dtype == PFDR_F32) return new QuadSession<float>(p);
    if (p->dtype == PFDR_F64) return new QuadSession<double>(p);
    throw std::runtime_error("dtype must be PFDR_F32 or PFDR_F64");
}

// ------------------------------------------------ drop-in entry points --
template <typename real>
static int quadratic_host(const char *fn, int kind, int V, int E, int N, real *X,
                          const real *Y, const real *A, const int *Eu,
                          const int *Ev, const real *La_d1, const real *La_l1,
                          int positivity, real mn, real mx, int Ltype,
                          const real *L, real rho, real condMin, real difRcd,
                          real difTol, int itMax, int *it, real *Obj,
                          real *Dif, int verbose) {
    pfdr_problem p{};
    p.kind = kind;
    p.dtype = dtype_of<real>();
    p.mem = PFDR_MEM_HOST;
    p.V = V; p.E = E; p.N = N;
    p.X = X; p.Y = Y; p.A = A; p.Eu = Eu; p.Ev = Ev;
    p.La_d1 = La_d1; p.La_l1 = La_l1; p.positivity = positivity;
    p.min = mn; p.max = mx; p.Ltype = Ltype; p.L = L;
    p.rho = rho; p.condMin = condMin; p.difRcd = difRcd; p.difTol = difTol;
    p.itMax = itMax; p.verbose = verbose;
    p.record_obj = Obj != nullptr;
    p.record_dif = Dif != nullptr;
    try {
        CallTrace tr(fn);
        if (verbose) { printf("Initializing constants and variables... "); fflush(stdout); }
        const std::vector<int> devs = multidev_devices(&p);
        if (!devs.empty()) {  // partitioned across the configured devices
            if (verbose) { printf("done (%d devices).\n", (int)devs.size()); fflush(stdout); }
            int its = 0;
            multidev_solve(&p, devs, &its, Obj, Dif);
            if (it) *it = its;
            tr.finish(V, E, N, 1, its);
            return PFDR_OK;
        }
        std::unique_ptr<QuadSession<real>> s(new QuadSession<real>(&p));
        if (verbose) { printf("done.\nPreconditioned forward-Douglas-Rachford algorithm\n"); fflush(stdout); }
        tr.setup_done();
        s->run(itMax);
        tr.run_done();
        int its = 0;
        s->result(X, &its, Obj, Dif);
        if (it) *it = its;
        s.reset();
        tr.finish(V, E, N, 1, its);
    } catch (const HipError &h) {
        return report_error(fn, h);
    } catch (const std::exception &ex) {
        return report_error(fn, ex.what());
    }
    return PFDR_OK;
}

}  // namespace pfdr

using pfdr::quadratic_host;

extern "C" int pfdr_quadratic_d1_l1_f32(int V, int E, int N, float *X,
    const float *Y, const float *A, const int *Eu, const int *Ev,
    const float *La_d1, const float *La_l1, int positivity, int Ltype,
    const float *L, float rho, float condMin, float difRcd, float difTol,
    int itMax, int *it, float *Obj, float *Dif, int verbose) {
    return quadratic_host<float>("pfdr_quadratic_d1_l1_f32", PFDR_KIND_L1, V, E, N, X, Y, A, Eu,
                                 Ev, La_d1, La_l1, positivity, 0.f, 0.f, Ltype, L, rho, condMin,
                                 difRcd, difTol, itMax, it, Obj, Dif, verbose);
}
extern "C" int pfdr_quadratic_d1_l1_f64(int V, int E, int N, double *X,
    const double *Y, const double *A, const int *Eu, const int *Ev,
    const double *La_d1, const double *La_l1, int positivity, int Ltype,
    const double *L, double rho, double condMin, double difRcd,
    double difTol, int itMax, int *it, double *Obj, double *Dif,
    int verbose) {
    return quadratic_host<double>("pfdr_quadratic_d1_l1_f64", PFDR_KIND_L1, V, E, N, X, Y, A, Eu,
                                  Ev, La_d1, La_l1, positivity, 0.0, 0.0, Ltype, L, rho, condMin,
                                  difRcd, difTol, itMax, it, Obj, Dif, verbose);
}
extern "C" int pfdr_quadratic_d1_bounds_f32(int V, int E, int N, float *X,
    const float *Y, const float *A, const int *Eu, const int *Ev,
    const float *La_d1, float min, float max, int Ltype, const float *L,
    float rho, float condMin, float difRcd, float difTol, int itMax,
    int *it, float *Obj, float *Dif, int verbose) {
    return quadratic_host<float>("pfdr_quadratic_d1_bounds_f32", PFDR_KIND_BOUNDS, V, E, N, X, Y,
                                 A, Eu, Ev, La_d1, nullptr, 0, min, max, Ltype, L, rho, condMin,
                                 difRcd, difTol, itMax, it, Obj, Dif, verbose);
}
extern "C" int pfdr_quadratic_d1_bounds_f64(int V, int E, int N, double *X,
    const double *Y, const double *A, const int *Eu, const int *Ev,
    const double *La_d1, double min, double max, int Ltype, const double *L,
    double rho, double condMin, double difRcd, double difTol, int itMax,
    int *it, double *Obj, double *Dif, int verbose) {
    return quadratic_host<double>("pfdr_quadratic_d1_bounds_f64", PFDR_KIND_BOUNDS, V, E, N, X, Y,
                                  A, Eu, Ev, La_d1, nullptr, 0, min, max, Ltype, L, rho, condMin,
                                  difRcd, difTol, itMax, it, Obj, Dif, verbose);
}

// Test hook (pfdr_mi355x.h, "debug"): the edge-block records of
// k_edge_sweep_tl for host arrays; only blocks [blk_begin, blk_begin +
// blk_count) are built, every other record keeps the caller's contents.
extern "C" int pfdr_debug_tile_erec(int64_t E, int dtype, const int *Eu, const int *Ev,
                                    int blk_begin, int blk_count, int *rec, int64_t rec_ints) {
    using namespace pfdr;
    const char *fn = "pfdr_debug_tile_erec";
    try {
        if (E <= 0 || !Eu || !Ev || !rec || (dtype != PFDR_F32 && dtype != PFDR_F64))
            return report_error(fn, "invalid argument");
        const int EB = kBlock * (dtype == PFDR_F32 ? Vec<float>::kPer16B : Vec<double>::kPer16B);
        const long neb = (E + EB - 1) / EB;
        if (rec_ints != neb * kErec || blk_begin < 0 || blk_count < 0 || blk_begin + blk_count > neb)
            return report_error(fn, "record array or block range does not match E");
        hipStream_t s = lib_stream();
        DevBuf<int> dEu(E), dEv(E), dr(rec_ints);
        PFDR_HIP(hipMemcpyAsync(dEu.p, Eu, E * 4, hipMemcpyHostToDevice, s));
        PFDR_HIP(hipMemcpyAsync(dEv.p, Ev, E * 4, hipMemcpyHostToDevice, s));
        PFDR_HIP(hipMemcpyAsync(dr.p, rec, rec_ints * 4, hipMemcpyHostToDevice, s));
        if (blk_count) {
            const int wpb = kBlock / kWave;
            k_tile_erec<<<(blk_count + wpb - 1) / wpb, kBlock, 0, s>>>(E, EB, blk_begin,
                                                                     blk_begin + blk_count, dEu.p,
                                                                     dEv.p, dr.p);
            PFDR_HIP(hipGetLastError());
        }
        PFDR_HIP(hipMemcpyAsync(rec, dr.p, rec_ints * 4, hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
    } catch (const HipError &h) {
        return report_error(fn, h);
    } catch (const std::exception &ex) {
        return report_error(fn, ex.what());
    }
    return PFDR_OK;
}

// the record layout the hook writes: ints per record, v runs per record,
// nub of an unstaged (u-block drop) block
extern "C" int pfdr_debug_erec_layout(int *ints, int *runs, int *nostage) {
    if (ints) *ints = pfdr::kErec;
    if (runs) *runs = pfdr::kEbRuns;
    if (nostage) *nostage = pfdr::kErecNoStage;
    return PFDR_OK;
}
