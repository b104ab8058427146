// MI355X PFDR solver for
//     F(x) = 1/2 ||y - A x||^2 + sum_e la_e |x_u - x_v| + sum_v la_v |x_v|
//            (+ x >= 0)                              [flavour l1]
//     F(x) = 1/2 ||y - A x||^2 + sum_e la_e |x_u - x_v| + i_[min,max](x)
//                                                    [flavour bounds]
// by preconditioned forward-Douglas-Rachford splitting, the algorithm of
// reference src/PFDR_graph_quadratic_d1_l1.cpp:270-553 and
// src/PFDR_graph_quadratic_d1_bounds.cpp:244-530, re-designed for gfx950:
//
//   per iteration (identity / diagonal A):
//     k_edge_sweep   : TV prox of every edge + relaxed Z update + the two
//                      DR contributions W*Z (one fused, fully coalesced
//                      sweep over the edge arrays; (X, P) of both endpoints
//                      gathered as one 8/16-byte pair)          ref :466-489
//     k_vertex_sweep : ordered segmented DR average over the incidence CSR
//                      (replaces the serial scatter :491-497), l1 / box
//                      prox, iterate-evolution partials, and the NEXT
//                      forward step P = 2X - Ga (A X - Y)      ref :491-529,
//                                                                  :355-464
//     k_finalize     : (only when dif is tracked / Obj recorded) evolution,
//                      stop / recondition flags in device memory
//   dense A adds a column-dot GEMV pair (N > 0) or one symmetric GEMV
//   (N < 0) producing the forward step; they are HBM bound (M = 1), so they
//   stream A with 16-byte loads instead of using MFMA.
//
// Arithmetic is written operation-for-operation as the reference and the
// library is built with -ffp-contract=off, so the per-edge and per-vertex
// updates round identically to it; the per-vertex sums run in the
// reference's order (incidence CSR sorted by (e, side)).  Reductions (dif,
// Obj, dense dot products) use fixed-shape trees.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <type_traits>

#include "pfdr_graph.hpp"
#include "pfdr_monosum.hpp"
#include "pfdr_session.hpp"

namespace pfdr {

enum AMode : int { A_IDENT = 0, A_DIAG = 1, A_DIRECT = 2, A_ATA = 3 };
enum Prox : int { PROX_NONE = 0, PROX_L1 = 1, PROX_POS = 2, PROX_BOX = 3,
                  PROX_LO = 4, PROX_HI = 5 };
// launch gates evaluated from the device control block
enum Gate : int { GATE_NONE = 0, GATE_ACTIVE = 1, GATE_OBJ = 2,
                  GATE_ACTIVE_OR_OBJ = 3 };

template <typename real> using R2 = typename Vec<real>::v2;

template <typename T, int N>
__device__ __forceinline__ Pk<T, N> ldv(const T *p) {
    return *reinterpret_cast<const Pk<T, N> *>(p);
}
template <typename T, int N>
__device__ __forceinline__ void stv(T *p, const Pk<T, N> &x) {
    *reinterpret_cast<Pk<T, N> *>(p) = x;
}

template <typename real>
__device__ __forceinline__ bool gated(const Ctrl<real> *c, int gate) {
    if (!c || gate == GATE_NONE) return false;
    const bool halt = c->halt != 0;
    const bool objdone = c->obj_it >= c->it;
    if (gate == GATE_ACTIVE) return halt;
    if (gate == GATE_OBJ) return objdone;
    return halt && objdone;
}

// Ordered sum over the incidence CSR of the block's vertices.  The entries
// of the block's contiguous vertex range (idx = address of each
// contribution) are gathered cooperatively — all lanes busy whatever the
// degrees, coalesced index reads, GB index loads then GB value gathers in
// flight per lane — into LDS chunks; then each lane adds its own vertex's
// entries in CSR order, i.e. in the reference's order (e, side).
// ZD: the list holds the edge variables Z and each term is w * z, w the
// vertex's own splitting weight (the contribution the edge sweep did not
// form, see k_edge_sweep_tl), computed as the edge sweep would
template <typename real, int CAP, int GB = 16, bool ZD = false>
__device__ __forceinline__ real gather_sum(int V, int v0,
                                           const int *__restrict__ ptr,
                                           const unsigned *__restrict__ idx,
                                           const real *__restrict__ wz,
                                           real *lds, real wv = real(1)) {
    static_assert(CAP % (kBlock * GB) == 0, "chunk must be a whole batch");
    const int tid = threadIdx.x;
    const int v = v0 + tid;
    const int vend = min(v0 + kBlock, V);
    const long seg0 = ptr[v0], seg1 = ptr[vend];
    const long my0 = (v < V) ? (long)ptr[v] : seg1;
    const long my1 = (v < V) ? (long)ptr[v + 1] : seg1;
    real s = real(0);
    for (long c0 = seg0; c0 < seg1; c0 += CAP) {
        const int n = (int)min((long)CAP, seg1 - c0);
        for (int b = 0; b < n; b += kBlock * GB) {
            unsigned id[GB];
#pragma unroll
            for (int u = 0; u < GB; u++) {
                const int j = b + u * kBlock + tid;
                id[u] = (j < n) ? idx[c0 + j] : 0u;
            }
            real w[GB];
#pragma unroll
            for (int u = 0; u < GB; u++) {
                const int j = b + u * kBlock + tid;
                w[u] = (j < n) ? wz[id[u]] : real(0);
            }
#pragma unroll
            for (int u = 0; u < GB; u++) {
                const int j = b + u * kBlock + tid;
                if (j < n) lds[j] = w[u];
            }
        }
        __syncthreads();
        const long a = max(my0, c0), e = min(my1, c0 + (long)n);
        for (long j = a; j < e; j++) s += ZD ? wv * lds[j - c0] : lds[j - c0];
        __syncthreads();
    }
    return s;
}

template <typename real> struct GatherCap;
template <> struct GatherCap<float> { static constexpr int v = 4096; };
template <> struct GatherCap<double> { static constexpr int v = 4096; };

// exclusive prefix sum over the block's lanes (lane order), all lanes call
__device__ __forceinline__ int block_excl_scan(int x, int *lds /* kBlock / kWave */) {
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    int inc = x;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int y = __shfl_up(inc, o, kWave);
        if (lane >= o) inc += y;
    }
    if (lane == kWave - 1) lds[w] = inc;
    __syncthreads();
    int base = 0;
    for (int i = 0; i < w; i++) base += lds[i];
    return base + inc - x;
}

// Split incidence of a graph whose edges are sorted by their u end (see
// k_split_build): the u-end contributions of vertex v are the contiguous
// run wz[uptr[v] .. uptr[v+1]) (side-major wz, u ends first), so only the
// OTHER entries (v ends and received contributions) need an address,
// oidx[ptr[v] - uptr[v] ...], and one 32-bit code per vertex says, entry by
// entry in the reference's order, which list the next term comes from
// (bit i set: the vertex's next own u-run entry), with a terminator bit at
// position deg.  The lanes' offsets into the two lists are a block scan of
// the codes' counts, so a lane reads 4 bytes of metadata, not 12.
// The block's u-runs are staged with coalesced loads (no index, no
// pointer chase), the others gathered; both lists meet in LDS and each
// lane adds its vertex's terms in the reference's (e, side) order.
// Valid for a block whose runs fit the LDS halves (checked at setup).
template <typename real, int GB>
__device__ __forceinline__ real split_sum(int V, int v0, int v, const int *__restrict__ ptr,
                                          const int *__restrict__ uptr,
                                          const unsigned *__restrict__ code,
                                          const unsigned *__restrict__ oidx,
                                          const real *__restrict__ wz, real *lds, int *scan) {
    constexpr int CU = GatherCap<real>::v / 2;
    const int tid = threadIdx.x;
    const int vend = min(v0 + kBlock, V);
    // per-lane code first: its latency hides under the staging
    unsigned m = (v < V) ? code[v] : 0u;
    const int ua = uptr[v0], ub = uptr[vend];
    const int oa = ptr[v0] - ua, ob = ptr[vend] - ub;
    const int nu = ub - ua, no = ob - oa;
    const int nmax = max(nu, no);
    for (int b = 0; b < nmax; b += kBlock * GB) {
        unsigned id[GB];
        real wu[GB], wo[GB];
#pragma unroll
        for (int u = 0; u < GB; u++) {
            const int j = b + u * kBlock + tid;
            id[u] = (j < no) ? oidx[oa + j] : 0u;
            wu[u] = (j < nu) ? wz[ua + j] : real(0);
        }
#pragma unroll
        for (int u = 0; u < GB; u++) {
            const int j = b + u * kBlock + tid;
            wo[u] = (j < no) ? wz[id[u]] : real(0);
        }
#pragma unroll
        for (int u = 0; u < GB; u++) {
            const int j = b + u * kBlock + tid;
            if (j < nu) lds[j] = wu[u];
            if (j < no) lds[CU + j] = wo[u];
        }
    }
    // lane offsets into the staged lists: counts (u | others << 16) scanned
    const int deg = m ? 31 - __clz(m) : 0;
    const int cu = m ? __popc(m) - 1 : 0;
    const int off = block_excl_scan(cu | ((deg - cu) << 16), scan);  // syncs the block
    real s = real(0);
    if (v < V) {
        int pu = off & 0xffff, po = CU + (off >> 16);
        for (int i = 0; i < deg; i++) {
            const bool own = m & 1u;
            s += lds[own ? pu : po];
            pu += own;
            po += !own;
            m >>= 1;
        }
    }
    return s;
}

// ---------------------------------------------- tiled DR contributions --
// Large single-GPU graphs store their edges in TILE order: sorted by
// (u block, v block, edge), 256-vertex blocks (the vertex sweep's).  The
// edge sweep then writes both contributions W*Z at the edge's position
// (wz[p] u end, wz[E + p] v end) as plain streams, and every vertex block
// finds ALL of its contributions in a few contiguous runs: the u ends of
// its own block's edges (wz[ustart[b] .. ustart[b+1]), one run) and the
// v ends of the (u block, b) tiles (runs of wz[E + p] listed in tptr /
// tstart / tlen).  Each run is read once, coalesced, by exactly one
// workgroup; every entry carries its slot in the block's CSR-ordered list
// (d2, 16 bits, the CSR position of (edge, side) minus the block's first),
// so staging puts each contribution where the reference's (e, side) order
// wants it, and each lane then adds its vertex's slots in order -- the sums
// of gather_sum / split_sum bit for bit, without a single gathered load.
constexpr int kTileCap = 4096;  // staged entries per vertex block (LDS: GatherCap)

// Each vertex's slots [my0, my0 + deg) in the block's list come from its
// degree (deg8: one byte per vertex, < 256 in every tiled block -- k_tile_ok)
// by a block scan, instead of two CSR pointers (1 B per vertex, not 4).
// The slots are 12-bit (a tiled block lists at most kTileCap = 4096
// contributions), packed eight to a 12-byte group (Slots12), and the runs
// are staged a group at a time: one 12-byte slot load beside the group's
// contributions (two 16-byte loads f32, four f64), from the aligned group
// at or below each run's start, elements outside the run dropped.  The
// contribution arrays carry one spare group at their end for the last
// run's tail.
constexpr int kTileRuns = 128;  // v-end runs per vertex block
constexpr int kSlotGroup = 8;   // contributions per packed slot group
struct alignas(4) Slots12 { unsigned w[3]; };  // 8 x 12 bits, little-endian
__device__ __forceinline__ int slot12(const Slots12 &g, int i) {
    const unsigned long long lo = g.w[0] | ((unsigned long long)g.w[1] << 32);  // bits 0..63
    const unsigned long long hi = g.w[1] | ((unsigned long long)g.w[2] << 32);  // bits 32..95
    return i < 5 ? (int)((lo >> (12 * i)) & 0xfff) : (int)((hi >> (12 * i - 32)) & 0xfff);
}

template <typename real, int GB, bool ZD = false>
__device__ __forceinline__ real tile_sum(int V, long E, int blk, int v,
                                         const unsigned char *__restrict__ deg8,
                                         const Slots12 *__restrict__ slots,
                                         const int *__restrict__ ustart,
                                         const int *__restrict__ tptr,
                                         const int *__restrict__ tstart,
                                         const int *__restrict__ tlen,
                                         const real *__restrict__ wz, real *lds, int *runs,
                                         real wv = real(1)) {
    constexpr int VE = Vec<real>::kPer16B, G = kSlotGroup, ZV = G / VE;
    constexpr int GG = GB / G > 0 ? GB / G : 1;  // groups in flight per lane
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    const int dg = v < V ? deg8[v] : 0;
    const int us = ustart[blk], nu = ustart[blk + 1] - us;
    const int t0 = tptr[blk], nt = tptr[blk + 1] - t0;
    // run table (wave 0): starts, lengths, inclusive prefix of the runs'
    // group counts; the degrees' wave totals after it (read after the
    // barriers below)
    int *rs = runs, *rl = runs + kTileRuns, *rp = runs + 2 * kTileRuns;
    int *wt = runs + 3 * kTileRuns;
    int dinc = dg;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int y = __shfl_up(dinc, o, kWave);
        if (lane >= o) dinc += y;
    }
    if (lane == kWave - 1) wt[w] = dinc;
    if (tid < kWave) {
        int acc = 0;
        for (int c = 0; c < nt; c += kWave) {
            const int i = c + tid;
            int ng = 0;
            if (i < nt) {
                const int st = tstart[t0 + i], len = tlen[t0 + i];
                rs[i] = st;
                rl[i] = len;
                const long A = E + st;
                ng = len > 0 ? (int)((A + len - 1) / G - A / G + 1) : 0;
            }
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const int y = __shfl_up(ng, o, kWave);
                if (tid >= o) ng += y;
            }
            if (i < nt) rp[i] = acc + ng;
            acc += __shfl(ng, kWave - 1, kWave);
        }
    }
    // u ends: one contiguous run [us, us + nu), GG groups in flight per lane
    {
        const long fu = us / G;
        const int ngu = nu > 0 ? (int)((us + nu - 1) / G - fu + 1) : 0;
        for (int b = 0; b < ngu; b += kBlock * GG) {
            Slots12 d[GG];
            Pk<real, VE> x[GG][ZV];
#pragma unroll
            for (int u = 0; u < GG; u++) {
                const long g = fu + min(b + u * kBlock + tid, ngu - 1);
                d[u] = slots[g];
#pragma unroll
                for (int z = 0; z < ZV; z++) x[u][z] = ldv<real, VE>(wz + g * G + z * VE);
            }
#pragma unroll
            for (int u = 0; u < GG; u++) {
                const int k = b + u * kBlock + tid;
                if (k < ngu) {
                    const long base = (fu + k) * G;
#pragma unroll
                    for (int q = 0; q < G; q++)
                        if (base + q >= us && base + q < (long)us + nu)
                            lds[slot12(d[u], q)] = x[u][q / VE].v[q % VE];
                }
            }
        }
    }
    __syncthreads();  // run table
    const int ngv = nt ? rp[nt - 1] : 0;
    // run of the lane's group k and its bounds in the group list
    int lo = 0, end = nt ? rp[0] : 0, beg = 0;
    for (int b = 0; b < ngv; b += kBlock * GG) {
        Slots12 d[GG];
        Pk<real, VE> x[GG][ZV];
        long base[GG], A[GG];
        int L[GG];
#pragma unroll
        for (int u = 0; u < GG; u++) {
            // the lane's groups grow by 256: its run only advances, no search
            const int k = min(b + u * kBlock + tid, ngv - 1);
            while (end <= k) {
                beg = end;
                end = rp[++lo];
            }
            A[u] = E + rs[lo];
            L[u] = rl[lo];
            base[u] = (A[u] / G + (k - beg)) * G;
        }
#pragma unroll
        for (int u = 0; u < GG; u++) {
            d[u] = slots[base[u] / G];
#pragma unroll
            for (int z = 0; z < ZV; z++) x[u][z] = ldv<real, VE>(wz + base[u] + z * VE);
        }
#pragma unroll
        for (int u = 0; u < GG; u++)
            if (b + u * kBlock + tid < ngv) {
#pragma unroll
                for (int q = 0; q < G; q++)
                    if (base[u] + q >= A[u] && base[u] + q < A[u] + L[u])
                        lds[slot12(d[u], q)] = x[u][q / VE].v[q % VE];
            }
    }
    __syncthreads();
    int my0 = dinc - dg;
    for (int q = 0; q < w; q++) my0 += wt[q];
    const int my1 = my0 + dg;
    // the vertex's slots in order; four reads in flight ahead of the adds
    real s = real(0);
    int j = my0;
    for (; j + 4 <= my1; j += 4) {
        const real a0 = lds[j], a1 = lds[j + 1], a2 = lds[j + 2], a3 = lds[j + 3];
        s += ZD ? wv * a0 : a0;
        s += ZD ? wv * a1 : a1;
        s += ZD ? wv * a2 : a2;
        s += ZD ? wv * a3 : a3;
    }
    for (; j < my1; j++) s += ZD ? wv * lds[j] : lds[j];
    return s;
}

// tile_sum from a per-block record (blocks with at most kRecRuns v-end runs,
// tok = 2): [u start, u count, runs, (start, length) x runs] in 32 ints, so
// the block's metadata is ONE load round (the run table otherwise costs two
// dependent ones, tptr then tstart / tlen, and a barrier), every wave holds
// the runs in its lanes, and the u-end and v-end groups are loaded in the
// same round -- two groups in flight per lane -- before one barrier.
constexpr int kRecRuns = 14, kTileRec = 32;
constexpr int kPrec = 16;  // runs per block in prec: the u run, then up to 15 v runs

template <typename real, bool ZD = false>
__device__ __forceinline__ real tile_sum_rec(int V, long E, int blk, int v,
                                             const unsigned char *__restrict__ deg8,
                                             const Slots12 *__restrict__ slots,
                                             const int *__restrict__ trec,
                                             const real *__restrict__ wz, real *lds, int *wt,
                                             real wv = real(1),
                                             const Slots12 *__restrict__ ptab = nullptr,
                                             const int *__restrict__ prec = nullptr,
                                             bool pre = false, int pre_rv = 0, int pre_pr = 0,
                                             int pre_dg = 0) {
    constexpr int VE = Vec<real>::kPer16B, G = kSlotGroup, ZV = G / VE;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    // (pre: the record, pattern offsets and degree came with the caller's
    // first load round, see vertex_block)
    const int dg = pre ? pre_dg : v < V ? deg8[v] : 0;
    const int rv = pre ? pre_rv : lane < kTileRec ? trec[(long)blk * kTileRec + lane] : 0;
    // pattern offsets of the runs (prec, with the record; null: per-entry slots)
    const int pr = pre ? pre_pr : prec && lane < kPrec ? prec[(long)blk * kPrec + lane] : 0;
    int dinc = dg;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int y = __shfl_up(dinc, o, kWave);
        if (lane >= o) dinc += y;
    }
    if (lane == kWave - 1) wt[w] = dinc;
    const int us = __builtin_amdgcn_readlane(rv, 0), nu = __builtin_amdgcn_readlane(rv, 1);
    const int nt = __builtin_amdgcn_readlane(rv, 2);
    // run r in lane r: start, length, groups, inclusive prefix of the groups
    const int st = __shfl(rv, min(3 + 2 * lane, kWave - 1), kWave);
    const int ln = __shfl(rv, min(4 + 2 * lane, kWave - 1), kWave);
    int P = 0;
    if (lane < nt && ln > 0) {
        const long A = E + st;
        P = (int)((A + ln - 1) / G - A / G + 1);
    }
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int y = __shfl_up(P, o, kWave);
        if (lane >= o) P += y;
    }
    const int ngv = __builtin_amdgcn_readlane(P, kWave - 1);
    const long fu = us / G;
    const int ngu = nu > 0 ? (int)((us + nu - 1) / G - fu + 1) : 0;
    const int tot = ngu + ngv;
    for (int b = 0; b < tot; b += 2 * kBlock) {
        Slots12 d[2];
        Pk<real, VE> x[2][ZV];
        long gb[2], lo[2], hi[2];
        int pg[2];  // the group's entry in the pattern table
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int k = min(b + u * kBlock + tid, tot - 1);
            // the run of a v-end group (every lane takes part in the
            // shuffles: a lane's run table entries must be read while it is
            // active)
            const int kv = k - ngu;
            int r = 0;
            for (int q = 0; q < nt; q++) r += __builtin_amdgcn_readlane(P, q) <= kv;
            r = min(r, kWave - 1);
            const int sr = __shfl(st, r, kWave), lr = __shfl(ln, r, kWave);
            const int pb = __shfl(P, max(r - 1, 0), kWave);
            const int pv = __shfl(pr, min(r + 1, kWave - 1), kWave);
            if (k < ngu) {
                gb[u] = fu + k;
                lo[u] = us;
                hi[u] = (long)us + nu;
                pg[u] = __builtin_amdgcn_readlane(pr, 0) + k;
            } else {
                const long A = E + sr;
                const int gi = kv - (r > 0 ? pb : 0);
                gb[u] = A / G + gi;
                lo[u] = A;
                hi[u] = A + lr;
                pg[u] = pv + gi;
            }
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
            d[u] = prec ? ptab[pg[u]] : slots[gb[u]];
#pragma unroll
            for (int z = 0; z < ZV; z++) x[u][z] = ldv<real, VE>(wz + gb[u] * G + z * VE);
        }
#pragma unroll
        for (int u = 0; u < 2; u++)
            if (b + u * kBlock + tid < tot) {
#pragma unroll
                for (int q = 0; q < G; q++) {
                    const long p = gb[u] * G + q;
                    if (p >= lo[u] && p < hi[u]) lds[slot12(d[u], q)] = x[u][q / VE].v[q % VE];
                }
            }
    }
    __syncthreads();
    int my0 = dinc - dg;
    for (int q = 0; q < w; q++) my0 += wt[q];
    const int my1 = my0 + dg;
    real s = real(0);
    int j = my0;
    for (; j + 4 <= my1; j += 4) {
        const real a0 = lds[j], a1 = lds[j + 1], a2 = lds[j + 2], a3 = lds[j + 3];
        s += ZD ? wv * a0 : a0;
        s += ZD ? wv * a1 : a1;
        s += ZD ? wv * a2 : a2;
        s += ZD ? wv * a3 : a3;
    }
    for (; j < my1; j++) s += ZD ? wv * lds[j] : lds[j];
    return s;
}

// tile_sum_rec for two consecutive record blocks b0, b0 + 1 in one
// workgroup (the pair vertex sweep): both records in one register (lanes
// 0..31 block b0's, 32..63 block b0 + 1's; kTileRec = 32 ints each, so one
// load), both blocks' runs in one register (lane 32 h + r: block b0 + h's run
// r), both blocks' groups in one list (b0's first), each scattered into its
// block's LDS list (lds + h cap) -- every lane keeps two vertices' gathers
// in flight where the one-block sweep keeps one, at the same eight waves per
// SIMD.  Each vertex's sum runs over its block's list in CSR order, as in
// tile_sum_rec: the same sums bit for bit.
template <typename real, bool ZD = false>
__device__ __forceinline__ void tile_sum_rec2(int V, long E, int b0, int v0, int v1,
                                              const unsigned char *__restrict__ deg8,
                                              const Slots12 *__restrict__ slots,
                                              const int *__restrict__ trec,
                                              const real *__restrict__ wz, real *lds, int cap,
                                              int *wt, real wv0, real wv1,
                                              const Slots12 *__restrict__ ptab,
                                              const int *__restrict__ prec, real &x0, real &x1) {
    static_assert(kTileRec == 32 && kWave == 64 && kPrec == 16, "two records per wave register");
    constexpr int VE = Vec<real>::kPer16B, G = kSlotGroup, ZV = G / VE, NW = kBlock / kWave;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    const int dg0 = v0 < V ? deg8[v0] : 0, dg1 = v1 < V ? deg8[v1] : 0;
    const int rv = trec[(long)b0 * kTileRec + lane];
    // pattern offsets: lane 16 h + q holds block b0 + h's entry q
    const int pr = prec ? prec[(long)b0 * kPrec + (lane & 31)] : 0;
    int i0 = dg0, i1 = dg1;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int y0 = __shfl_up(i0, o, kWave), y1 = __shfl_up(i1, o, kWave);
        if (lane >= o) {
            i0 += y0;
            i1 += y1;
        }
    }
    if (lane == kWave - 1) {
        wt[w] = i0;
        wt[NW + w] = i1;
    }
    const int us0 = __builtin_amdgcn_readlane(rv, 0), nu0 = __builtin_amdgcn_readlane(rv, 1);
    const int nt0 = __builtin_amdgcn_readlane(rv, 2);
    const int us1 = __builtin_amdgcn_readlane(rv, 32), nu1 = __builtin_amdgcn_readlane(rv, 33);
    const int nt1 = __builtin_amdgcn_readlane(rv, 34);
    const int hf = lane >> 5, rl = lane & 31;
    const int st = __shfl(rv, 32 * hf + min(3 + 2 * rl, 31), kWave);
    const int ln = __shfl(rv, 32 * hf + min(4 + 2 * rl, 31), kWave);
    int P = 0;
    if (rl < (hf ? nt1 : nt0) && ln > 0) {
        const long A = E + st;
        P = (int)((A + ln - 1) / G - A / G + 1);
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {  // inclusive prefix within each half
        const int y = __shfl_up(P, o, kWave);
        if (rl >= o) P += y;
    }
    const int ngv0 = __builtin_amdgcn_readlane(P, 31), ngv1 = __builtin_amdgcn_readlane(P, 63);
    const long fu0 = us0 / G, fu1 = us1 / G;
    const int ngu0 = nu0 > 0 ? (int)((us0 + nu0 - 1) / G - fu0 + 1) : 0;
    const int ngu1 = nu1 > 0 ? (int)((us1 + nu1 - 1) / G - fu1 + 1) : 0;
    const int tot0 = ngu0 + ngv0, tot = tot0 + ngu1 + ngv1;
    const int pu0 = __builtin_amdgcn_readlane(pr, 0), pu1 = __builtin_amdgcn_readlane(pr, 16);
    for (int b = 0; b < tot; b += 2 * kBlock) {
        Slots12 d[2];
        Pk<real, VE> x[2][ZV];
        long gb[2];
        // the run's bounds relative to the group (clamped to [-1, G + 1]) and
        // the block, packed: (lo + 1) | (hi + 1) << 4 | h << 8
        int pg[2], mt[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int k = min(b + u * kBlock + tid, tot - 1);
            const int h = k >= tot0;
            const int kk = k - (h ? tot0 : 0);
            const int ngu = h ? ngu1 : ngu0;
            const int kv = kk - ngu;
            // the group's run in its block (both halves' tables walked by
            // every lane: the loop bounds stay uniform)
            int ra = 0, rb = 0;
            for (int q = 0; q < nt0; q++) ra += __builtin_amdgcn_readlane(P, q) <= kv;
            for (int q = 0; q < nt1; q++) rb += __builtin_amdgcn_readlane(P, 32 + q) <= kv;
            const int r = min(h ? rb : ra, 31), base = 32 * h;
            const int sr = __shfl(st, base + r, kWave), lr = __shfl(ln, base + r, kWave);
            const int pb = __shfl(P, base + max(r - 1, 0), kWave);
            const int pv = __shfl(pr, 16 * h + min(r + 1, 15), kWave);
            long L, H;
            if (kk < ngu) {
                gb[u] = (h ? fu1 : fu0) + kk;
                L = h ? us1 : us0;
                H = L + (h ? nu1 : nu0);
                pg[u] = (h ? pu1 : pu0) + kk;
            } else {
                const long A = E + sr;
                const int gi = kv - (r > 0 ? pb : 0);
                gb[u] = A / G + gi;
                L = A;
                H = A + lr;
                pg[u] = pv + gi;
            }
            const int lo = (int)max(L - gb[u] * G, -1L), hi = (int)min(H - gb[u] * G, (long)G + 1);
            mt[u] = (lo + 1) | (hi + 1) << 4 | h << 8;
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
            d[u] = prec ? ptab[pg[u]] : slots[gb[u]];
#pragma unroll
            for (int z = 0; z < ZV; z++) x[u][z] = ldv<real, VE>(wz + gb[u] * G + z * VE);
        }
#pragma unroll
        for (int u = 0; u < 2; u++)
            if (b + u * kBlock + tid < tot) {
                real *l = lds + ((mt[u] >> 8) ? cap : 0);
                const int lo = (mt[u] & 15) - 1, hi = ((mt[u] >> 4) & 15) - 1;
#pragma unroll
                for (int q = 0; q < G; q++)
                    if (q >= lo && q < hi) l[slot12(d[u], q)] = x[u][q / VE].v[q % VE];
            }
    }
    __syncthreads();
    int my0 = i0 - dg0, my1 = i1 - dg1;
    for (int q = 0; q < w; q++) {
        my0 += wt[q];
        my1 += wt[NW + q];
    }
    real s0 = real(0), s1 = real(0);
    for (int j = 0; j < dg0; j++) s0 += ZD ? wv0 * lds[my0 + j] : lds[my0 + j];
    for (int j = 0; j < dg1; j++) s1 += ZD ? wv1 * lds[cap + my1 + j] : lds[cap + my1 + j];
    x0 = s0;
    x1 = s1;
}

// tile-order keys: (u block, v block) in the high bits, edge position the
// value; a partitioned rank (split) puts the edges with a ghost end after
// all the others (bit 2 vbits)
static __global__ void k_tile_keys(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                                   int vbits, unsigned long long *__restrict__ keys,
                                   unsigned *__restrict__ vals, int V = 0, bool split = false) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int u = Eu[e], v = Ev[e];
    const unsigned long long g = split && (u >= V || v >= V) ? 1ull << (2 * vbits) : 0ull;
    keys[e] = g | ((unsigned long long)(u / kBlock) << vbits) | (unsigned)(v / kBlock);
    vals[e] = (unsigned)e;
}

// *out = the number of sorted keys below `bound` (one lane, binary search)
static __global__ void k_count_below(long n, const unsigned long long *__restrict__ keys,
                                     unsigned long long bound, unsigned long long *out) {
    long lo = 0, hi = n;
    while (lo < hi) {
        const long mid = (lo + hi) >> 1;
        if (keys[mid] < bound) lo = mid + 1;
        else hi = mid;
    }
    *out = (unsigned long long)lo;
}

// d2[address] = CSR slot of the (edge, side) at that address, relative to the
// first slot of its vertex block; one lane per vertex
static __global__ void k_tile_slots(int V, const int *__restrict__ ptr,
                                    const unsigned *__restrict__ idx,
                                    unsigned short *__restrict__ d2) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const int base = ptr[v - v % kBlock];
    for (int j = ptr[v]; j < ptr[v + 1]; j++) d2[idx[j]] = (unsigned short)(j - base);
}

// the slots of addresses [8 g, 8 g + 8) packed into group g (12 bits each,
// slot i at bits [12 i, 12 i + 12); a tiled block's slots are < kTileCap)
static __global__ void k_pack_slots(long ngroups, long n, const unsigned short *__restrict__ d2,
                                    Slots12 *__restrict__ out) {
    const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ngroups) return;
    unsigned long long lo = 0, hi = 0;  // bits 0..63, 64..95
#pragma unroll
    for (int q = 0; q < kSlotGroup; q++) {
        const long p = g * kSlotGroup + q;
        const unsigned long long x = p < n ? (d2[p] & 0xfffu) : 0u;
        const int bit = 12 * q;
        if (bit + 12 <= 64) {
            lo |= x << bit;
        } else if (bit >= 64) {
            hi |= x << (bit - 64);
        } else {
            lo |= x << bit;
            hi |= x >> (64 - bit);
        }
    }
    Slots12 r;
    r.w[0] = (unsigned)lo;
    r.w[1] = (unsigned)(lo >> 32);
    r.w[2] = (unsigned)hi;
    out[g] = r;
}

// ustart[b] = first position whose u end is in block >= b (tile order sorts by
// u block), ustart[nb] = E
static __global__ void k_tile_ustart(long E, int nb, const int *__restrict__ Eu,
                                     int *__restrict__ ustart) {
    const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p > E) return;
    const int lo = p == 0 ? 0 : Eu[p - 1] / kBlock + 1;
    const int hi = p == E ? nb : Eu[p] / kBlock;
    for (int b = lo; b <= hi; b++) ustart[b] = (int)p;
}

// Runs of a vertex block's contributions outside its u run, each a maximal
// stretch of entries i of one source whose vertex lies in that block:
//   v ends (a = Ev over [0, E), rs = 0): wz[E + i];
//   u ends of a partitioned rank's boundary edges (a = Eu + Eint, rs = Eint - E):
//     wz[Eint + i];
//   received contributions (keys = the halo's recv_keys, rs = E): wz[2E + i];
// vertices >= V (ghosts) belong to no block.  A run is stored as its start
// relative to E (tstart = rs + i: the vertex sweep reads wz[E + tstart + k])
// and its length.
__device__ __forceinline__ int run_block(long i, const int *__restrict__ a,
                                         const unsigned long long *__restrict__ keys, int V) {
    const int x = keys ? (int)(keys[i] >> 32) : a[i];
    return x < V ? x / kBlock : -1;
}
static __global__ void k_tile_runs_count(long n, const int *__restrict__ a,
                                         const unsigned long long *__restrict__ keys, int V,
                                         int *__restrict__ cnt) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int b = run_block(i, a, keys, V);
    if (b >= 0 && (i == 0 || run_block(i - 1, a, keys, V) != b)) atomicAdd(cnt + b, 1);
}

// each run at its block's next slot (the order of a block's runs does not
// matter: every entry carries its slot), with its length
static __global__ void k_tile_runs_fill(long n, const int *__restrict__ a,
                                        const unsigned long long *__restrict__ keys, int V,
                                        long rs, const int *__restrict__ tptr,
                                        int *__restrict__ fill, int *__restrict__ tstart,
                                        int *__restrict__ tlen) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int b = run_block(i, a, keys, V);
    if (b < 0 || (i != 0 && run_block(i - 1, a, keys, V) == b)) return;
    long q = i + 1;
    while (q < n && run_block(q, a, keys, V) == b) q++;
    const int j = tptr[b] + atomicAdd(fill + b, 1);
    tstart[j] = (int)(rs + i);
    tlen[j] = (int)(q - i);
}

// tok[b] = 1 when block b's entries fit the LDS list and its runs the table
// tok[b] = 1: block b's list fits the LDS (cap entries), its runs the run
// table, and every degree a byte (deg8, tile_sum)
static __global__ void k_tile_ok(int V, int nb, const int *__restrict__ ptr,
                                 const int *__restrict__ tptr, int cap, int *__restrict__ tok) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const int v0 = b * kBlock, v1 = min(v0 + kBlock, V);
    bool ok = ptr[v1] - ptr[v0] <= cap && tptr[b + 1] - tptr[b] <= kTileRuns;
    for (int v = v0; ok && v < v1; v++) ok = ptr[v + 1] - ptr[v] < 256;
    tok[b] = ok ? 1 : 0;
}

// the per-block records of tile_sum_rec for tiled blocks with at most
// kRecRuns v-end runs (tok 1 -> 2)
static __global__ void k_tile_rec(int nb, const int *__restrict__ ustart,
                                  const int *__restrict__ tptr, const int *__restrict__ tstart,
                                  const int *__restrict__ tlen, int *__restrict__ tok,
                                  int *__restrict__ rec) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const int t0 = tptr[b], nt = tptr[b + 1] - t0;
    int *r = rec + (long)b * kTileRec;
    for (int q = 0; q < kTileRec; q++) r[q] = 0;
    if (!tok[b] || nt > kRecRuns) return;
    r[0] = ustart[b];
    r[1] = ustart[b + 1] - ustart[b];
    r[2] = nt;
    for (int q = 0; q < nt; q++) {
        r[3 + 2 * q] = tstart[t0 + q];
        r[4 + 2 * q] = tlen[t0 + q];
    }
    tok[b] = 2;
}

// ------------------------------------------------ slot patterns -------
// On regular graphs most record blocks' runs carry the same slot sequences
// (on C2 every interior block is one x-row of the grid; on C5 the 640-vertex
// rows give five phases).  A run's PATTERN = (its first address mod 8, its
// length, its slots); the distinct patterns go to a small table of packed
// groups (ptab, aligned as each run's groups are) and each record block gets
// the table offset of every run (prec: 16 ints beside its record), so the
// vertex sweep reads no per-entry slot stream (12 B per 8 contributions).
__device__ __forceinline__ bool rec_run(const int *r, long E, int q, long &A, int &len) {
    const int nt = r[2];
    if (q == 0) {
        A = r[0];
        len = r[1];
    } else if (q <= nt) {
        A = E + r[1 + 2 * q];
        len = r[2 + 2 * q];
    } else {
        return false;
    }
    return true;
}

// hash of run q of record block b (~0: no run / not a record block)
static __global__ void k_run_hash(int nb, long E, const int *__restrict__ tok,
                                  const int *__restrict__ trec, const unsigned short *__restrict__ d2,
                                  unsigned long long *__restrict__ h) {
    const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= (long)nb * kPrec) return;
    const int b = (int)(id / kPrec), q = (int)(id - (long)b * kPrec);
    unsigned long long x = ~0ull;
    long A;
    int len;
    if (tok[b] == 2 && rec_run(trec + (long)b * kTileRec, E, q, A, len)) {
        x = 0x9e3779b97f4a7c15ull * (unsigned long long)((A & 7) + 1) ^ (unsigned long long)len << 20;
        for (int i = 0; i < len; i++) {
            x ^= d2[A + i] + 0x9e3779b97f4a7c15ull + (x << 6) + (x >> 2);
            x *= 0xbf58476d1ce4e5b9ull;
        }
        if (x == ~0ull) x = 0;
    }
    h[id] = x;
}

// every run's slots equal those of its pattern's representative (else *bad)
static __global__ void k_run_verify(int nb, long E, const int *__restrict__ tok,
                                    const int *__restrict__ trec,
                                    const unsigned short *__restrict__ d2,
                                    const long long *__restrict__ repA, int *__restrict__ bad) {
    const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= (long)nb * kPrec) return;
    const int b = (int)(id / kPrec), q = (int)(id - (long)b * kPrec);
    long A;
    int len;
    if (tok[b] != 2 || !rec_run(trec + (long)b * kTileRec, E, q, A, len)) return;
    const long R = repA[id];
    bool ok = R >= 0 && (R & 7) == (A & 7);
    for (int i = 0; ok && i < len; i++) ok = d2[A + i] == d2[R + i];
    if (!ok) atomicAdd(bad, 1);
}

// deg8[v] = the vertex's CSR entries (clamped; blocks with a larger one are
// not tiled)
static __global__ void k_tile_deg(int V, const int *__restrict__ ptr,
                                  unsigned char *__restrict__ deg8) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < V) deg8[v] = (unsigned char)min(ptr[v + 1] - ptr[v], 255);
}

// ------------------------------------------------ split incidence setup --
// counts edges out of u order or with a u end outside [0, V)
static __global__ void k_u_order_check(long E, int V, const int *__restrict__ Eu,
                                unsigned long long *__restrict__ bad) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int u = Eu[e];
    if (u < 0 || u >= V || (e + 1 < E && u > Eu[e + 1])) atomicAdd(bad, 1ull);
}

// uptr[v] = first edge whose u end is >= v, v in [0, V] (Eu sorted)
static __global__ void k_uptr(long E, int V, const int *__restrict__ Eu, int *__restrict__ uptr) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e > E) return;
    const int lo = e == 0 ? 0 : Eu[e - 1] + 1;
    const int hi = e == E ? V : Eu[e];
    for (int v = lo; v <= hi; v++) uptr[v] = (int)e;
}

// One lane per vertex: code (bit i: the i-th CSR entry is the vertex's next
// own u-run contribution; terminator bit at the degree) and the other
// entries' addresses in CSR order.  blkok[b] = 1 when every vertex of block
// b has <= 31 entries with its u-run in edge order, and the block's runs
// fit the LDS halves (cap).
static __global__ __launch_bounds__(256) void k_split_build(int V, long E, const int *__restrict__ ptr,
                                                     const unsigned *__restrict__ idx,
                                                     const int *__restrict__ uptr, long ototal,
                                                     unsigned *__restrict__ mask,
                                                     unsigned *__restrict__ oidx,
                                                     int *__restrict__ blkok, int cap) {
    const int v0 = blockIdx.x * kBlock;
    const int v = v0 + threadIdx.x;
    int ok = 1;
    if (v < V) {
        const int p0 = ptr[v], p1 = ptr[v + 1], u0 = uptr[v], u1 = uptr[v + 1];
        const long o0 = (long)p0 - u0;
        unsigned m = 0u;
        int cu = 0, co = 0;
        if (p1 - p0 > 31) ok = 0;
        for (int j = p0; j < p1; j++) {
            const unsigned id = idx[j];
            if ((long)id < E) {
                if ((long)id != (long)u0 + cu) ok = 0;
                if (j - p0 < 32) m |= 1u << (j - p0);
                cu++;
            } else {
                if (o0 + co >= 0 && o0 + co < ototal) oidx[o0 + co] = id;
                co++;
            }
        }
        if (cu != u1 - u0) ok = 0;
        mask[v] = (p1 - p0 <= 31) ? (m | (1u << (p1 - p0))) : 0u;
    }
    const int all = __syncthreads_and(ok);
    if (threadIdx.x == 0) {
        const int vend = min(v0 + kBlock, V);
        const int nu = uptr[vend] - uptr[v0];
        const int no = (ptr[vend] - uptr[vend]) - (ptr[v0] - uptr[v0]);
        blkok[blockIdx.x] = (all && nu <= cap && no >= 0 && no <= cap) ? 1 : 0;
    }
}

// ====================================================================== //
//                                kernels                                  //
// ====================================================================== //

template <typename real>
__global__ void k_xp_init(int V, const real *__restrict__ X, R2<real> *xp) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    R2<real> o;
    o.x = X[v];
    o.y = real(0);
    xp[v] = o;
}

template <typename real>
__global__ void k_x_extract(int V, const R2<real> *__restrict__ xp,
                            real *__restrict__ X) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < V) X[v] = xp[v].x;
}

// X in the caller's labels from a relabelled session: X[v] = xp[where[v]].x
template <typename real>
__global__ void k_x_extract_perm(int V, const R2<real> *__restrict__ xp,
                                 const int *__restrict__ where, real *__restrict__ X) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < V) X[v] = xp[where[v]].x;
}

// dst[i] = src[map[i]] (relabelling gathers)
template <typename T>
__global__ void k_gather(long n, const T *__restrict__ src, const int *__restrict__ map,
                         T *__restrict__ dst) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[map[i]];
}

// dst[map[i]] = src[i] (a relabelled partition's amplitudes in the caller's order)
template <typename T>
__global__ void k_scatter(long n, const T *__restrict__ src, const int *__restrict__ map,
                          T *__restrict__ dst) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[map[i]] = src[i];
}

// edge variable (e, side): half-edge layout Z2[2e + side] (zs = 0), or
// side-major Z[side * zs + e] (zs = E: tile-ordered sessions)
__device__ __forceinline__ long zat(long e, int side, long zs) {
    return zs ? side * zs + e : 2 * e + side;
}

// Z_u = X[Eu], Z_v = X[Ev]   (ref :320-324)
template <typename real>
__global__ void k_z_init(long E, const int *__restrict__ Eu,
                         const int *__restrict__ Ev,
                         const R2<real> *__restrict__ xp,
                         real *__restrict__ Z2, long zs) {
    long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    Z2[zat(e, 0, zs)] = xp[Eu[e]].x;
    Z2[zat(e, 1, zs)] = xp[Ev[e]].x;
}

// diagonal of A^t A for the identity / diagonal / A^tA modes (ref :101-122)
// (A^tA: local column v of a column block starting at global row row0,
// column length ld)
template <typename real>
__global__ void k_diag(int V, int mode, const real *__restrict__ A, long ld, long row0,
                       real *__restrict__ diag) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    real d = real(1);
    if (mode == A_DIAG) d = A[v];
    else if (mode == A_ATA) d = A[(size_t)ld * v + row0 + v];
    diag[v] = d;
}

// --------------------------------------------------- dense column dots --
enum ColEpi : int { EPI_STORE = 0, EPI_SELF = 1, EPI_DIV = 2,
                    EPI_FWD_DIRECT = 3, EPI_FWD_ATA = 4,
                    EPI_GRAD_DIRECT = 5, EPI_GRAD_ATA = 6 };

template <typename real>
struct ColArgs {
    const real *A;        // column major, column c at A + len*c
    int ncols, len;
    const real *w;        // vector dotted with every column (len)
    real *out;            // STORE/SELF/DIV/GRAD_*
    const real *div;      // DIV
    R2<real> *xp;         // FWD_*
    const real *Ga, *Y;   // FWD_*, GRAD_ATA
    const Ctrl<real> *ctrl;
    int gate;
};

// acc + x y in double: f32 operands multiply exactly in double, so one fma
// rounds as the product and the sum would; f64 keeps the multiply and add
template <typename real>
__device__ __forceinline__ double dacc(double acc, double x, double y) {
    if (sizeof(real) == 4) return fma(x, y, acc);
    return acc + x * y;
}

template <typename real, int EPI>
__device__ __forceinline__ void col_epilogue(const ColArgs<real> &a, long col, real acc) {
    if (EPI == EPI_STORE || EPI == EPI_SELF) {
        a.out[col] = acc;
    } else if (EPI == EPI_DIV) {
        a.out[col] = acc / a.div[col];
    } else if (EPI == EPI_GRAD_DIRECT) {
        a.out[col] = -acc;
    } else if (EPI == EPI_GRAD_ATA) {
        real p = acc;
        p -= a.Y[col];
        a.out[col] = p;
    } else {
        real p;
        if (EPI == EPI_FWD_DIRECT) {
            p = -acc;
        } else {
            p = acc;
            p -= a.Y[col];
        }
        R2<real> q = a.xp[col];
        q.y = real(2) * q.x - a.Ga[col] * p;
        a.xp[col] = q;
    }
}

// One wave64 per column: 16-byte loads of the column (and of w, which
// every wave re-reads from L2), wave-shuffle reduction, fused epilogue.
// The products and sums run in double whatever `real` (HBM-bound), so a
// tree-reduced f32 dot product lies closer to the exact one than the
// reference's sequential f32 sum, not just as close (tests/
// test_fullsize_pin_gpu.py: the yardstick is the reference's f64 run).  The
// product of two f32 values is exact in double, so one fma per term rounds
// exactly as a multiply and an add would (f64 fma: one instruction, not two).
// ref: diag of A^tA :102-110, pseudo-inverse :126-134, apply A^tA
// :368-376, gradient -A^t R :432-440, forward :462-464.
template <typename real, int EPI>
__global__ __launch_bounds__(256) void k_col_dot(ColArgs<real> a) {
    if (gated(a.ctrl, a.gate)) return;
    const int lane = threadIdx.x & 63;
    const long col = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (col >= a.ncols) return;
    const real *c = a.A + (size_t)a.len * col;
    const real *w = (EPI == EPI_SELF) ? c : a.w;
    constexpr int VW = Vec<real>::kPer16B;
    double acc = 0.0;
    if ((a.len % VW) == 0) {
        const int nv = a.len / VW;
        for (int i = lane; i < nv; i += 64) {
            Pk<real, VW> x = ldv<real, VW>(c + (size_t)i * VW);
            Pk<real, VW> y = ldv<real, VW>(w + (size_t)i * VW);
#pragma unroll
            for (int j = 0; j < VW; j++) acc = dacc<real>(acc, x.v[j], y.v[j]);
        }
    } else {
        for (int i = lane; i < a.len; i += 64) acc = dacc<real>(acc, c[i], w[i]);
    }
    acc = wave_sum(acc);
    if (lane != 0) return;
    col_epilogue<real, EPI>(a, col, (real)acc);
}

// Sequential-order column dots for small dense problems (the reduced
// problems cut pursuit hands over): one lane per column adds c[i] w[i] for
// i = 0, 1, ... exactly as the reference's loops do (:102-110, :126-134,
// :368-376, :432-440), so the dense modes round like the reference, bit for
// bit.  The chain is `len` dependent adds per lane, hence only below the
// session's exact-dense limit; 4 x 16-byte loads in flight ahead of the adds.
template <typename real, int EPI>
__global__ __launch_bounds__(256) void k_col_seq(ColArgs<real> a) {
    if (gated(a.ctrl, a.gate)) return;
    const long col = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (col >= a.ncols) return;
    const real *c = a.A + (size_t)a.len * col;
    const real *w = (EPI == EPI_SELF) ? c : a.w;
    constexpr int VW = Vec<real>::kPer16B, U = 4;
    real acc = real(0);
    int i = 0;
    if ((a.len % VW) == 0 && ((uintptr_t)a.A % 16) == 0 && ((uintptr_t)w % 16) == 0) {
        for (; i + U * VW <= a.len; i += U * VW) {
            Pk<real, VW> x[U], y[U];
#pragma unroll
            for (int q = 0; q < U; q++) {
                x[q] = ldv<real, VW>(c + i + q * VW);
                y[q] = ldv<real, VW>(w + i + q * VW);
            }
#pragma unroll
            for (int q = 0; q < U; q++)
#pragma unroll
                for (int j = 0; j < VW; j++) acc += x[q].v[j] * y[q].v[j];
        }
    }
    for (; i < a.len; i++) acc += c[i] * w[i];
    col_epilogue<real, EPI>(a, col, acc);
}

// R[n] = Y[n] - sum_v A[n + N v] X[v], v ascending in one lane per row
// (ref :356-367 order; loads coalesced across the lanes), single GPU
template <typename real>
__global__ __launch_bounds__(256) void k_rows_seq(int N, int V, const real *__restrict__ A,
                                                  const R2<real> *__restrict__ xp,
                                                  const real *__restrict__ Y,
                                                  real *__restrict__ R, const Ctrl<real> *ctrl,
                                                  int gate) {
    if (gated(ctrl, gate)) return;
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    constexpr int U = 8;
    real acc = real(0);
    int v = 0;
    for (; v + U <= V; v += U) {
        real c[U], x[U];
#pragma unroll
        for (int q = 0; q < U; q++) {
            c[q] = A[(size_t)N * (v + q) + n];
            x[q] = xp[v + q].x;
        }
#pragma unroll
        for (int q = 0; q < U; q++) acc += c[q] * x[q];
    }
    for (; v < V; v++) acc += A[(size_t)N * v + n] * xp[v].x;
    R[n] = Y[n] - acc;
}

// ------------------------------------------- symmetric A^tA products --
// A^tA is symmetric, so y = (A^tA) w needs only its block upper triangle:
// half the HBM bytes of one wave per column (k_col_dot).  Tile (bi, bj),
// bi <= bj, is T x T entries (32 row groups of one 16-byte vector: T = 128
// f32 / 64 f64, 64 KB / 32 KB); its row part A_IJ w_J goes to part[bj][I],
// its column part A_IJ^t w_I (bi < bj) to part[bi][J]; every (block, row)
// slot has exactly one writer and k_symv_finish sums part[0..nb)[r] in that
// fixed order (deterministic; a regrouping of the reference's column dot
// products :368-376, :432-440, :462-464 like k_col_dot's).  Taken only when
// the caller's matrix is exactly symmetric (k_sym_check), V % VW == 0 and
// A is 16-byte aligned.
template <typename real>
struct SymT {
    static constexpr int VW = Vec<real>::kPer16B, T = 32 * VW, CPT = T / 8;
};

// t = bj (bj + 1) / 2 + bi with 0 <= bi <= bj (column-major upper triangle)
__device__ __forceinline__ void tri_index(long t, int &bi, int &bj) {
    long j = (long)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while (j * (j + 1) / 2 > t) j--;
    while ((j + 1) * (j + 2) / 2 <= t) j++;
    bj = (int)j;
    bi = (int)(t - j * (j + 1) / 2);
}

template <typename real>
__global__ __launch_bounds__(256) void k_symv_tiles(int V, const real *__restrict__ A,
                                                    const real *__restrict__ w,
                                                    real *__restrict__ part,
                                                    const Ctrl<real> *ctrl, int gate) {
    if (gated(ctrl, gate)) return;
    using S = SymT<real>;
    constexpr int VW = S::VW, T = S::T, CPT = S::CPT;
    __shared__ real wI[T], wJ[T], csum[T];
    __shared__ real rsum[8][T];
    int bi, bj;
    tri_index(blockIdx.x, bi, bj);
    const int I0 = bi * T, J0 = bj * T;
    const int tid = threadIdx.x;
    const int rg = tid & 31, cg = tid >> 5;  // row group (16 B of a column), column group
    const int r0 = I0 + rg * VW;
    const bool rok = r0 < V;  // V % VW == 0: the lane's whole vector is in range
    Pk<real, VW> a[CPT];
#pragma unroll
    for (int k = 0; k < CPT; k++) {
        const int c = J0 + cg * CPT + k;
        if (rok && c < V) {
            a[k] = ldv<real, VW>(A + (size_t)V * c + r0);
        } else {
#pragma unroll
            for (int j = 0; j < VW; j++) a[k].v[j] = real(0);
        }
    }
    if (tid < T) {
        wI[tid] = (I0 + tid < V) ? w[I0 + tid] : real(0);
        wJ[tid] = (J0 + tid < V) ? w[J0 + tid] : real(0);
    }
    __syncthreads();
    // row part: this lane's VW rows over its CPT columns
    real racc[VW];
#pragma unroll
    for (int j = 0; j < VW; j++) racc[j] = real(0);
#pragma unroll
    for (int k = 0; k < CPT; k++) {
        const real wc = wJ[cg * CPT + k];
#pragma unroll
        for (int j = 0; j < VW; j++) racc[j] += a[k].v[j] * wc;
    }
#pragma unroll
    for (int j = 0; j < VW; j++) rsum[cg][rg * VW + j] = racc[j];
    // column part: column dots over the tile's rows, summed across the 32
    // row groups of the half-wave (xor butterfly: every lane holds the same sum)
    const bool offdiag = bi != bj;
    if (offdiag) {
        real wr[VW];
#pragma unroll
        for (int j = 0; j < VW; j++) wr[j] = wI[rg * VW + j];
#pragma unroll
        for (int k = 0; k < CPT; k++) {
            real s = real(0);
#pragma unroll
            for (int j = 0; j < VW; j++) s += a[k].v[j] * wr[j];
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 32);
            if (rg == k) csum[cg * CPT + k] = s;
        }
    }
    __syncthreads();
    if (tid < T) {
        const int r = I0 + tid;
        if (r < V) {
            real s = rsum[0][tid];
#pragma unroll
            for (int g = 1; g < 8; g++) s += rsum[g][tid];
            part[(size_t)bj * V + r] = s;
        }
        const int c = J0 + tid;
        if (offdiag && c < V) part[(size_t)bi * V + c] = csum[tid];
    }
}

// 64 rows per block, the nb slots of a row split over 4 waves (8 loads in
// flight per lane; one lane walking all nb slots was latency bound), the
// four quarter sums added in a fixed order
template <typename real, int EPI>
__global__ __launch_bounds__(256) void k_symv_finish(int nb, const real *__restrict__ part,
                                                     ColArgs<real> a) {
    if (gated(a.ctrl, a.gate)) return;
    __shared__ real q4[4][64];
    const int rl = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int r = blockIdx.x * 64 + rl;
    const int per = (nb + 3) / 4, b0 = g * per, b1 = min(nb, b0 + per);
    real acc = real(0);
    if (r < a.ncols) {
#pragma unroll 8
        for (int b = b0; b < b1; b++) acc += part[(size_t)b * a.ncols + r];
    }
    q4[g][rl] = acc;
    __syncthreads();
    if (g == 0 && r < a.ncols)
        col_epilogue<real, EPI>(a, r, ((q4[0][rl] + q4[1][rl]) + q4[2][rl]) + q4[3][rl]);
}

// flag[0] = 1 unless A (V x V, column major) is exactly symmetric: tile
// (bi, bj), bi <= bj, of 64 x 64 entries against the mirror tile staged in LDS
template <typename real>
__global__ __launch_bounds__(256) void k_sym_check(int V, const real *__restrict__ A,
                                                   int *__restrict__ flag) {
    constexpr int T = 64;
    __shared__ real m[T][T + 1];
    int bi, bj;
    tri_index(blockIdx.x, bi, bj);
    const int I0 = bi * T, J0 = bj * T;
    for (int i = threadIdx.x; i < T * T; i += blockDim.x) {
        const int r = i & (T - 1), c = i >> 6;  // mirror tile: rows J, columns I
        if (J0 + r < V && I0 + c < V) m[c][r] = A[(size_t)V * (I0 + c) + J0 + r];
    }
    __syncthreads();
    bool bad = false;
    for (int i = threadIdx.x; i < T * T; i += blockDim.x) {
        const int r = i & (T - 1), c = i >> 6;  // tile: rows I, columns J
        if (I0 + r < V && J0 + c < V) {
            const real x = A[(size_t)V * (J0 + c) + I0 + r];
            bad |= !(x == m[r][c]);
        }
    }
    if (bad) flag[0] = 1;
}

// R partials: part[b][n] = sum_{v in block b} A[n + N v] X[v]
// (column-major A streamed once, 16-byte loads, 4 columns in flight);
// products and partials in double (as k_col_dot)
template <typename real>
__global__ __launch_bounds__(256) void k_rows_partial(
    int N, int V, const real *__restrict__ A, const R2<real> *__restrict__ xp,
    int cpb, double *__restrict__ part, const Ctrl<real> *ctrl, int gate) {
    if (gated(ctrl, gate)) return;
    const int b = blockIdx.x;
    const int v0 = b * cpb, v1 = min(v0 + cpb, V);
    constexpr int VW = Vec<real>::kPer16B;
    if ((N % VW) == 0) {
        for (int n0 = threadIdx.x * VW; n0 < N; n0 += kBlock * VW) {
            double acc[VW];
#pragma unroll
            for (int j = 0; j < VW; j++) acc[j] = 0.0;
            int v = v0;
            for (; v + 4 <= v1; v += 4) {
                Pk<real, VW> c[4];
                double x[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    c[q] = ldv<real, VW>(A + (size_t)N * (v + q) + n0);
                    x[q] = (double)xp[v + q].x;
                }
#pragma unroll
                for (int q = 0; q < 4; q++)
#pragma unroll
                    for (int j = 0; j < VW; j++) acc[j] = dacc<real>(acc[j], c[q].v[j], x[q]);
            }
            for (; v < v1; v++) {
                Pk<real, VW> c = ldv<real, VW>(A + (size_t)N * v + n0);
                const double x = (double)xp[v].x;
#pragma unroll
                for (int j = 0; j < VW; j++) acc[j] = dacc<real>(acc[j], c.v[j], x);
            }
#pragma unroll
            for (int j = 0; j < VW; j++) part[(size_t)b * N + n0 + j] = acc[j];
        }
    } else {
        for (int n = threadIdx.x; n < N; n += kBlock) {
            double acc = 0.0;
            for (int v = v0; v < v1; v++) acc = dacc<real>(acc, A[(size_t)N * v + n], xp[v].x);
            part[(size_t)b * N + n] = acc;
        }
    }
}

// R[n] = Y[n] - sum_b part[b][n]   (ref :356-367), in double, rounded once
template <typename real>
__global__ void k_rows_finish(int N, int nb, const double *__restrict__ part,
                              const real *__restrict__ Y,
                              real *__restrict__ R, const Ctrl<real> *ctrl,
                              int gate) {
    if (gated(ctrl, gate)) return;
    int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    double s = 0.0;
    int b = 0;
    for (; b + 8 <= nb; b += 8) {
        double t[8];
#pragma unroll
        for (int q = 0; q < 8; q++) t[q] = part[(size_t)(b + q) * N + n];
#pragma unroll
        for (int q = 0; q < 8; q++) s += t[q];
    }
    for (; b < nb; b++) s += part[(size_t)b * N + n];
    // Y == NULL: this rank's partial A X (all-reduced next)
    R[n] = Y ? (real)((double)Y[n] - s) : (real)s;
}

// R = Y - (A X summed over the ranks)
template <typename real>
__global__ void k_rows_residual(int N, const real *__restrict__ Y, const real *__restrict__ S,
                                real *__restrict__ R, const Ctrl<real> *ctrl, int gate) {
    if (gated(ctrl, gate)) return;
    int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n < N) R[n] = Y[n] - S[n];
}

// ---------------------------------------------------- preconditioning --
// |amplitude| per vertex and block counts of nonzero amplitudes (ref
// :124-153).  src 0: pseudo-inverse Y/diag (N <= 0); 1: precomputed (N > 0);
// 2: current iterate (reconditioning).
template <typename real>
__global__ __launch_bounds__(256) void k_amp(int V, int src,
                                             const real *__restrict__ Y,
                                             const real *__restrict__ diag,
                                             const real *__restrict__ pre,
                                             const R2<real> *__restrict__ xp,
                                             real *__restrict__ absval,
                                             int *__restrict__ cnt_part) {
    __shared__ int red[kBlock / kWave];
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    real a = real(0);
    if (v < V) {
        if (src == 0) {
            real g = diag[v];
            a = (g > real(0)) ? Y[v] / g : real(0);
        } else if (src == 1) {
            a = pre[v];
        } else {
            a = xp[v].x;
        }
        // c += a for a > 0, c -= a for a < 0 (identical to adding -a)
        absval[v] = (a > real(0)) ? a : ((a < real(0)) ? -a : real(0));
    }
    int nz = (v < V) && (a > real(0) || a < real(0));
    nz = block_sum(nz, red);
    if (threadIdx.x == 0) cnt_part[blockIdx.x] = nz;
}

// c = n / sum|a| (first call) or sum|a| / n (reconditioning) (ref :154)
template <typename real>
__global__ void k_set_c(const real *__restrict__ sum, const long long *__restrict__ cnt,
                        int init, Ctrl<real> *ctrl) {
    if (threadIdx.x != 0) return;
    const real n = (real)(int)*cnt;
    const real s = *sum;
    ctrl->c = init ? n / s : s / n;
    ctrl->cnt = (int)*cnt;
}

// Splitting weights.  The reference stores Wu[e] = a_e Aux[u]^-1 and
// Wv[e] = a_e Aux[v]^-1 (ref :156-203), a_e = c La_d1[e] at the first
// conditioning, La_d1[e] / d_e at a reconditioning.  This build keeps only
// the factors: a_e is recomputed from La_d1 and the scalar c of the first
// conditioning (cw), or read from A1 after a reconditioning; invAux per
// vertex (with Ga in the packed gi pair).  Every product a_e * invAux is
// the reference's own operation, so the weights are identical bit for bit.
template <typename real>
__device__ __forceinline__ real edge_a(long e, const real *__restrict__ A1,
                                       const real *__restrict__ La_d1, real cw) {
    return A1 ? A1[e] : cw * La_d1[e];
}

// La_d1[e] of the iteration kernels: a null array means every edge weighs
// la0 (a uniform La_d1 detected at setup, k_uniform_check: the 4-byte
// stream is not read; the value, and so every operation, is the same)
template <typename real>
__device__ __forceinline__ real la_at(long e, const real *__restrict__ La_d1, real la0) {
    return La_d1 ? La_d1[e] : la0;
}
template <typename real, int N>
__device__ __forceinline__ Pk<real, N> la_vec(long e0, const real *__restrict__ La_d1, real la0) {
    Pk<real, N> la;
#pragma unroll
    for (int j = 0; j < N; j++) la.v[j] = la0;
    if (La_d1) {
        const Pk<real, N> x = ldv<real, N>(La_d1 + e0);
#pragma unroll
        for (int j = 0; j < N; j++) la.v[j] = x.v[j];
    }
    return la;
}

// nonzero *bad when some La_d1[e] differs from La_d1[0] (bitwise)
template <typename real>
__global__ void k_uniform_check(long E, const real *__restrict__ La_d1, int *__restrict__ bad) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    using U = typename std::conditional<sizeof(real) == 4, unsigned, unsigned long long>::type;
    const U x = *reinterpret_cast<const U *>(La_d1 + e), x0 = *reinterpret_cast<const U *>(La_d1);
    if (__any(x != x0) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(bad, 1);
}

// d1 contributions a_e to the per-vertex sums (both ends through the CSR,
// like the DR average; ref :156-192).  On reconditioning, first turn the
// auxiliary variables into subgradients with the OLD weights and metric
// (ref :89-99), then store the new a_e in A1 (A1old: null while the old
// a_e are still cw La_d1).
template <typename real>
__global__ void k_d1_weights(long E, const int *__restrict__ Eu,
                             const int *__restrict__ Ev,
                             const real *__restrict__ La_d1,
                             const Ctrl<real> *__restrict__ ctrl, int init,
                             real condMin, const R2<real> *__restrict__ xp,
                             const real *A1old, real cw, const real *__restrict__ invAux,
                             real *A1, real *__restrict__ wz,
                             const real *__restrict__ Ga,
                             const real *__restrict__ grad,
                             real *__restrict__ Z2, long zs) {
    long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const real c = ctrl->c;
    real w;
    if (init) {
        w = c * La_d1[e];
    } else {
        const int u = Eu[e], v = Ev[e];
        const real xu = xp[u].x, xv = xp[v].x;
        const real gu = Ga[u], gv = Ga[v];
        const real a0 = edge_a(e, A1old, La_d1, cw);
        const real wu = a0 * invAux[u], wv = a0 * invAux[v];
        const long iu = zat(e, 0, zs), iv = zat(e, 1, zs);
        Z2[iu] = (wu / gu) * (xu - gu * grad[u] - Z2[iu]);
        Z2[iv] = (wv / gv) * (xv - gv * grad[v] - Z2[iv]);
        real a = xu, b = xv, d = a - b;
        if (a < real(0)) a = -a;
        if (b < real(0)) b = -b;
        if (d < real(0)) d = -d;
        if (a < b) a = b;
        if (a < c) a = c;
        a *= condMin;
        if (d < a) d = a;
        w = La_d1[e] / d;
        A1[e] = w;
    }
    wz[e] = w;      // per-vertex sums go through the same CSR as the DR average
    wz[E + e] = w;
}

template <typename real>
__global__ __launch_bounds__(256) void k_precond_vertex(
    int V, const int *__restrict__ ptr, const unsigned *__restrict__ idx,
    const real *__restrict__ wz, const real *__restrict__ diag,
    const real *__restrict__ La_l1, const R2<real> *__restrict__ xp,
    const Ctrl<real> *__restrict__ ctrl, int init, real condMin, real cap,
    const real *__restrict__ Ldiag, real *__restrict__ Ga,
    real *__restrict__ invAux, real *__restrict__ Th_l1) {
    __shared__ real lds[GatherCap<real>::v];
    const int v0 = blockIdx.x * kBlock;
    const real s = gather_sum<real, GatherCap<real>::v>(V, v0, ptr, idx, wz, lds);
    const int v = v0 + threadIdx.x;
    if (v >= V) return;
    real g = diag[v];
    g += s;
    invAux[v] = real(1) / s;
    if (La_l1) {
        const real c = ctrl->c;
        if (init) {
            g += c * La_l1[v];
        } else {
            const real cm = c * condMin;
            real d = xp[v].x;
            if (d < real(0)) d = -d;
            if (d < cm) d = cm;
            g += La_l1[v] / d;
        }
    }
    g = real(1) / g;
    if (!Ldiag) {
        if (g > cap) g = cap;
    } else {
        const real L = Ldiag[v];
        if (L > real(0)) {
            const real b = cap / L;
            if (g > b) g = b;
        }
    }
    Ga[v] = g;
    if (La_l1) Th_l1[v] = g * La_l1[v];
}

// reconditioning: auxiliary variables back from subgradients with the new
// weights and metric (ref :241-250)
template <typename real>
__global__ void k_recond_edge(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                              const real *__restrict__ A1, const real *__restrict__ invAux,
                              const real *__restrict__ Ga, const R2<real> *__restrict__ xp,
                              const real *__restrict__ grad, real *__restrict__ Z2, long zs) {
    long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int u = Eu[e], v = Ev[e];
    const real wu = A1[e] * invAux[u];
    const real wv = A1[e] * invAux[v];
    const real gu = Ga[u], gv = Ga[v];
    const long iu = zat(e, 0, zs), iv = zat(e, 1, zs);
    Z2[iu] = xp[u].x - gu * (grad[u] + Z2[iu] / wu);
    Z2[iv] = xp[v].x - gv * (grad[v] + Z2[iv] / wv);
}

// (Ga, invAux) pairs of owned and ghost vertices: one 8/16-byte gather per
// edge end in the edge sweeps
template <typename real>
__global__ void k_gi_pack(int n, const real *__restrict__ Ga, const real *__restrict__ invAux,
                          R2<real> *__restrict__ gi) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    R2<real> q;
    q.x = Ga[v];
    q.y = invAux[v];
    gi[v] = q;
}

// per-vertex ratio of the RAT edge sweeps: the splitting weight of every
// edge at v over v's metric, (cw * la0 * invAux) / Ga -- bit for bit the
// quotient prox_weights forms from edge_full's wu when a_e = cw * la0
template <typename real>
__global__ void k_ratio_vertex(int n, real cw, real la0, const real *__restrict__ Ga,
                               const real *__restrict__ invAux, real *__restrict__ rr) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const real a0 = cw * la0;
    rr[v] = (a0 * invAux[v]) / Ga[v];
}

// the prox weights and threshold of an edge from its splitting weights,
// the metric of its ends and its TV weight — the operations of the
// reference's precomputation (ref :252-259), recomputed in every edge sweep
// (bit for bit the values the reference stores in W_d1u, W_d1v, Th_d1)
template <typename real>
__device__ __forceinline__ void prox_weights(real wu, real wv, real gu, real gv, real la,
                                             real &du, real &dv, real &th) {
    const real a = wu / gu, b = wv / gv, s = a + b;
    th = la * s / (a * b);
    du = a / s;
    dv = b / s;
}

// gradient A X - Y of the identity / diagonal modes (ref :377-385, :441-445)
template <typename real>
__global__ void k_grad_vertex(int V, int mode, const real *__restrict__ A,
                              const real *__restrict__ Y,
                              const R2<real> *__restrict__ xp,
                              real *__restrict__ grad) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const real x = xp[v].x;
    real p = (mode == A_DIAG) ? A[v] * x : x;
    p -= Y[v];
    grad[v] = p;
}

// forward step from the gradient: P = 2 X - Ga grad   (ref :462-464)
template <typename real>
__global__ void k_forward_grad(int V, const real *__restrict__ Ga,
                               const real *__restrict__ grad, R2<real> *xp) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    R2<real> q = xp[v];
    q.y = real(2) * q.x - Ga[v] * grad[v];
    xp[v] = q;
}

// ---------------------------------------------------------- iteration --
// TV prox on every edge (ref :466-489) + the two DR contributions W*Z.
// 16 bytes per lane on every edge stream: 4 (f32) / 2 (f64) edges per lane.
template <typename real>
__device__ __forceinline__ void edge_update(const R2<real> &pu,
                                            const R2<real> &pv, real &zu,
                                            real &zv, real wu, real wv,
                                            real th, real rho) {
    // pu.x = X[u], pu.y = P[u] (forward step)
    const real a = wu * (pu.y - zu) + wv * (pv.y - zv);
    real b = (pu.y - zu) - (pv.y - zv);
    if (b > th) {
        b -= th;
        zu += rho * (a + wv * b - pu.x);
        zv += rho * (a - wu * b - pv.x);
    } else if (b < -th) {
        b += th;
        zu += rho * (a + wv * b - pu.x);
        zv += rho * (a - wu * b - pv.x);
    } else {
        zu += rho * (a - pu.x);
        zv += rho * (a - pv.x);
    }
}

// one edge: splitting weights from a_e and the ends' invAux, prox weights
// from them and the ends' metric, TV prox + relaxed Z update, the two DR
// contributions W*Z
template <typename real>
__device__ __forceinline__ void edge_full(const R2<real> &pu, const R2<real> &pv,
                                          const R2<real> &giu, const R2<real> &giv, real a,
                                          real la, real &zu, real &zv, real &ou, real &ov,
                                          real rho) {
    const real wu = a * giu.y, wv = a * giv.y;
    real du, dv, th;
    prox_weights<real>(wu, wv, giu.x, giv.x, la, du, dv, th);
    edge_update<real>(pu, pv, zu, zv, du, dv, th, rho);
    ou = wu * zu;
    ov = wv * zv;
}

// iterate evolution and loop control (ref :514-529, :424-429, :447-460);
// red[0..1] = (sum (X - X_)^2, sum X^2) over all ranks
template <typename real>
__device__ __forceinline__ void decide_step(Ctrl<real> *ctrl, real num, real den,
                                            real *__restrict__ Dif, int track) {
    int it = ctrl->it;
    if (track) {
        const real eps = ctrl->eps;
        const real dif = (den > eps) ? num / den : num / eps;
        ctrl->dif = dif;
        if (Dif) Dif[it] = dif;
    }
    it++;
    ctrl->it = it;
    const real dif = ctrl->dif;
    if (it >= ctrl->itMax || dif < ctrl->difTol) {
        ctrl->stop = 1;
        ctrl->halt = 1;
    } else if (dif < ctrl->difRcd) {
        ctrl->recond = 1;
        ctrl->halt = 1;
    }
}

// Loop control of small single-GPU graphs (at most kFuseBlocks vertex
// blocks, dif tracked, no objective record), two launches per iteration
// instead of three (the sweeps' FD = true instances):
//  * the decision on iteration t is taken by the edge sweep of iteration
//    t + 1: EVERY workgroup sums the vertex sweep's partials with
//    k_reduce_decide's loop and tree and runs decide_step on its own copy
//    of the control block `src`; the workgroup of logical block 0 alone
//    writes the result (and Dif, red) to `dst`, a DIFFERENT control block
//    (the readers of this launch never see the update; the host alternates
//    the two blocks), and every workgroup skips its stores when the
//    decision halts -- so the iterates, iteration counts and Dif are those
//    of the three-launch loop, bit for bit;
//  * the halt flag (or the decision) is tested before the sweep's first
//    store instead of ahead of everything: one dependent round trip less at
//    the start of each launch (a halted launch then reads its operands
//    once, which only small launches can afford).
// The partials are loaded into registers before the sweep's own loads and
// added only after them, so their latency hides under the edge streams.
constexpr int kFuseBlocks = 1024;
constexpr int kFusePer = kFuseBlocks / kBlock;  // partial pairs per lane

template <typename real>
struct FuseDecide {
    const Ctrl<real> *src;  // null: no decision in this launch (halt of `ctrl` tested late)
    Ctrl<real> *dst;
    const real *part;       // 2 per vertex block
    real *red, *Dif;
    int nparts;             // <= kFuseBlocks
};

template <typename real>
struct FdRegs {
    real a[kFusePer], b[kFusePer];
    Ctrl<real> c;  // src, loaded with the partials (no dependent load later)
};

// a lane's operands of k_reduce_decide's fixed-order loop (i = tid + k kBlock)
template <typename real>
__device__ __forceinline__ void fd_load(const FuseDecide<real> &fd, FdRegs<real> &r) {
    r.c = *fd.src;
#pragma unroll
    for (int k = 0; k < kFusePer; k++) {
        const int i = threadIdx.x + k * kBlock;
        r.a[k] = i < fd.nparts ? fd.part[2 * i] : real(0);
        r.b[k] = i < fd.nparts ? fd.part[2 * i + 1] : real(0);
    }
}

// the loop's adds, block sums (k_reduce_decide's tree), the decision on a
// copy of src, the writer's stores; returns the (block-uniform) halt flag.
// Every lane calls.
template <typename real>
__device__ __forceinline__ int fd_decide(const FuseDecide<real> &fd, const FdRegs<real> &r,
                                         bool writer, real (*red)[kBlock / kWave], int *s_halt) {
    real a = real(0), b = real(0);
#pragma unroll
    for (int k = 0; k < kFusePer; k++)
        if ((int)threadIdx.x + k * kBlock < fd.nparts) { a += r.a[k]; b += r.b[k]; }
    a = block_sum(a, red[0]);
    b = block_sum(b, red[1]);
    if (threadIdx.x == 0) {
        Ctrl<real> c = r.c;
        const int was = c.halt;
        if (!was) decide_step(&c, a, b, writer ? fd.Dif : nullptr, 1);
        if (writer) {
            *fd.dst = c;
            if (!was) { fd.red[0] = a; fd.red[1] = b; }
        }
        *s_halt = c.halt;
    }
    __syncthreads();
    return *s_halt;
}

// One or two edge ranges of one launch: logical blocks [0, nb0) sweep
// [b0, e0), the others [b1, e1) (a partitioned session's two boundary
// ranges, before and after the interior run, in a single launch)
struct ERange {
    long b0, e0, b1, e1;
    int nb0;
    __device__ __forceinline__ void pick(int &blk, long &ebeg, long &eend) const {
        if (blk < nb0) { ebeg = b0; eend = e0; }
        else { blk -= nb0; ebeg = b1; eend = e1; }
    }
};

// Contributions of a small graph stored where its vertex sweep reads them
// (k_vertex_sweep_pad): the contribution of (e, side) goes to wzp[sl[2e +
// side]], the slot of that entry in its vertex block's CSR list, each block's
// list at a fixed stride.  Null sl: side-major wz as below.
template <typename real>
struct PadOut {
    const int *sl;
    real *wzp;
};

// Edge sweep over the edges [ebeg, eend) (ebeg a multiple of the lane
// width); writes the DR contributions W*Z side-major: wz[e] (u end),
// wz[E + e] (v end), so the u-side run of a vertex is contiguous.  Streams
// per edge: Eu, Ev, Z (r/w), La_d1, the two contributions (+ A1 after a
// reconditioning); gathers (X, P) and (Ga, invAux) of both ends.
// one lane's EPT edges [e0, e0 + EPT) of the edges [.., eend): the lane
// body of k_edge_sweep, shared with the one-workgroup k_tiny_iterate (whose
// xp is rewritten between its edge passes: no __restrict__ on it)
template <typename real>
__device__ __forceinline__ void edge_lane(long e0, long eend, long E, const int *__restrict__ Eu,
                                          const int *__restrict__ Ev, const R2<real> *xp,
                                          real *Z2, const real *A1, real cw, const R2<real> *gi,
                                          const real *__restrict__ La_d1, real la0, real *wz,
                                          real rho,
                                          PadOut<real> pd = PadOut<real>{nullptr, nullptr}) {
    constexpr int EPT = Vec<real>::kPer16B;
    if (e0 >= eend) return;
    if (e0 + EPT <= eend) {
        const Pk<int, EPT> iu = ldv<int, EPT>(Eu + e0);
        const Pk<int, EPT> iv = ldv<int, EPT>(Ev + e0);
        Pk<int, 2 * EPT> sv{};
        if (pd.sl) sv = ldv<int, 2 * EPT>(pd.sl + 2 * e0);
        R2<real> pu[EPT], pv[EPT], gu[EPT], gv[EPT];
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            pu[j] = xp[iu.v[j]]; pv[j] = xp[iv.v[j]];
            gu[j] = gi[iu.v[j]]; gv[j] = gi[iv.v[j]];
        }
        Pk<real, 2 * EPT> z = ldv<real, 2 * EPT>(Z2 + 2 * e0);
        const Pk<real, EPT> la = la_vec<real, EPT>(e0, La_d1, la0);
        Pk<real, EPT> a;
        if (A1) a = ldv<real, EPT>(A1 + e0);
        else {
#pragma unroll
            for (int j = 0; j < EPT; j++) a.v[j] = cw * la.v[j];
        }
        Pk<real, EPT> ou, ov;
#pragma unroll
        for (int j = 0; j < EPT; j++)
            edge_full<real>(pu[j], pv[j], gu[j], gv[j], a.v[j], la.v[j], z.v[2 * j],
                            z.v[2 * j + 1], ou.v[j], ov.v[j], rho);
        stv<real, 2 * EPT>(Z2 + 2 * e0, z);
        if (pd.sl) {
#pragma unroll
            for (int j = 0; j < EPT; j++) {
                pd.wzp[sv.v[2 * j]] = ou.v[j];
                pd.wzp[sv.v[2 * j + 1]] = ov.v[j];
            }
        } else {
            stv<real, EPT>(wz + e0, ou);
            stv<real, EPT>(wz + E + e0, ov);
        }
    } else {
        for (long e = e0; e < eend; e++) {
            const int u = Eu[e], v = Ev[e];
            real zu = Z2[2 * e], zv = Z2[2 * e + 1], ou, ov;
            const real l = la_at(e, La_d1, la0);
            edge_full<real>(xp[u], xp[v], gi[u], gi[v], A1 ? A1[e] : cw * l, l, zu, zv, ou, ov,
                            rho);
            Z2[2 * e] = zu;
            Z2[2 * e + 1] = zv;
            if (pd.sl) {
                pd.wzp[pd.sl[2 * e]] = ou;
                pd.wzp[pd.sl[2 * e + 1]] = ov;
            } else {
                wz[e] = ou;
                wz[E + e] = ov;
            }
        }
    }
}

template <typename real, bool FD>
__global__ __launch_bounds__(256) void k_edge_sweep(
    long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
    const R2<real> *__restrict__ xp, real *__restrict__ Z2, const real *__restrict__ A1, real cw,
    const R2<real> *__restrict__ gi, const real *__restrict__ La_d1, real la0,
    real *__restrict__ wz, real rho, const Ctrl<real> *ctrl, int nb, int xcd, ERange rg,
    FuseDecide<real> fd, PadOut<real> pdx) {
    if (!FD && ctrl && ctrl->halt) return;
    constexpr int EPT = Vec<real>::kPer16B;
    const PadOut<real> pd = FD ? pdx : PadOut<real>{nullptr, nullptr};
    int blk = xcd_block(blockIdx.x, nb, xcd);
    if (blk >= nb) return;
    if (FD) {
        __shared__ real red[2][kBlock / kWave];
        __shared__ int s_halt;
        if (fd.src) {
            FdRegs<real> r;
            fd_load(fd, r);
            if (fd_decide(fd, r, blk == 0, red, &s_halt)) return;
        } else if (ctrl && ctrl->halt) {
            return;
        }
    }
    long ebeg, eend;
    rg.pick(blk, ebeg, eend);
    const long e0 = ebeg + ((long)blk * blockDim.x + threadIdx.x) * EPT;
    edge_lane<real>(e0, eend, E, Eu, Ev, xp, Z2, A1, cw, gi, La_d1, la0, wz, rho, pd);
}

// Edge sweep of a tile-ordered graph (see tile_sum): sorted by u block, so
// the u ends of a block's edges lie in a few consecutive u blocks, and
// inside a (u block, v block) tile every v end lies in one 256-vertex block.
// Each workgroup reads a 192-byte record of its edges (erec, built at
// setup, scalar loads): the first u block, how many it spans and where in
// the block each further u block starts, and the runs of equal v block
// (start, v block base) -- at most kEbRuns; positions are relative to the
// block's first edge, so every lookup is a 32-bit compare against scalars
// in groups of four runs.  Every edge names both ends by one byte each
// (luv: u mod 256 | v mod 256 << 8), so neither Eu nor Ev is streamed: the
// u ends come from the block's staged u range of (X, P) and (Ga, invAux) in
// LDS, the v ends are gathered (a run's gathers share their lines) at v
// block base + byte.  A block with more runs reads Ev, one spanning more
// than TlBlocks u blocks reads Eu.  Z is side-major (Z[e], Z[E + e]); wz
// null (Z-direct, see tile_sum's ZD) leaves the W * Z products to the
// vertex sweep.
// u range staged: at most 16 KB of LDS (f64 blocks cover 512 edges)
template <typename real> struct TlBlocks { static constexpr int v = 16384 / (2 * 256 * sizeof(R2<real>)) ; };
constexpr int kEbRuns = 20;  // v-block runs in an edge block's record
constexpr int kErecU = 4;    // rec[4]: staged span; rec[4 + q]: start of u block ub0 + q
                             // (q = 1..3; INT_MAX if q >= nub)
constexpr int kErecS = 8;    // rec[kErecS + 2r]: start of run r (INT_MAX if r >= nruns), + 1: its v base
// rec[0..3]: ub0, nub, nruns (0: read Ev), uoff (smallest u end - ub0 * 256);
// the staged u range is [ub0 * 256 + uoff, + span), span = largest - smallest + 1
constexpr int kErec = kErecS + 2 * kEbRuns;
// UNI: one weight La_d1 for every edge (la0) and no A1 (before any
// reconditioning): a_e = cw * la0 is one value, computed once per lane.
// RAT (UNI, Z-direct): each end's ratio (cw * la0 / Aux) / Ga comes formed
// (k_ratio_vertex) -- one 4/8-byte gather per end instead of the (Ga,
// invAux) pair, and three divisions per edge instead of five
template <typename real>
__device__ __forceinline__ void edge_ratio(const R2<real> &pu, const R2<real> &pv, real a, real b,
                                           real la, real &zu, real &zv, real rho) {
    const real s = a + b, th = la * s / (a * b);
    edge_update<real>(pu, pv, zu, zv, a / s, b / s, th, rho);
}

template <typename real, bool UNI, bool RAT = false>
__device__ __forceinline__ void tl_gather(
    long E, int V, const int *__restrict__ Eu, const unsigned short *__restrict__ luv,
    const int *__restrict__ rec, const int *__restrict__ Ev,
    const R2<real> *__restrict__ xp, real *__restrict__ Z2, const real *__restrict__ A1, real cw,
    const R2<real> *__restrict__ gi, const real *__restrict__ La_d1, real la0,
    real *__restrict__ wz, real rho, int blk, R2<real> *s_xp, R2<real> *s_gi,
    const real *__restrict__ rr = nullptr) {
    static_assert(!RAT || UNI, "ratios need one edge weight");
    real *s_r = reinterpret_cast<real *>(s_gi);  // RAT: the staged ratios
    constexpr int EPT = Vec<real>::kPer16B;
    constexpr int NUB = TlBlocks<real>::v, SPAN = NUB * kBlock;
    const int tid = threadIdx.x;
    const int ub0 = rec[0], nub = rec[1], nr = rec[2];
    const int uoff = rec[3], span = rec[kErecU];  // staged u range: ub0 * 256 + uoff, span
    const bool staged = nub <= NUB && span <= SPAN;  // block-uniform
    const int rel = tid * EPT;       // first edge of the lane, relative to the block's
    const long e0 = (long)blk * kBlock * EPT + rel;
    const bool full = e0 + EPT <= E;
    // streams first, then the staging loads of the block's u range (the
    // first NS0 per lane issued unconditionally, clamped into the range, so
    // the load counts stay static), then the v-end gathers once the end
    // bytes are in: the three round trips overlap
    constexpr int NS0 = SPAN / kBlock / 2;
    Pk<unsigned short, EPT> ib{};
    Pk<real, 2 * EPT> z{};
    Pk<real, EPT> la{}, a{};
    R2<real> pu[EPT], pv[EPT], gu[EPT], gv[EPT];
    real ru[EPT], rv[EPT];
    if (full) {  // Z side-major (tiled sessions): zu at e, zv at E + e
        ib = ldv<unsigned short, EPT>(luv + e0);
        const Pk<real, EPT> zu = ldv<real, EPT>(Z2 + e0), zv = ldv<real, EPT>(Z2 + E + e0);
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            z.v[2 * j] = zu.v[j];
            z.v[2 * j + 1] = zv.v[j];
        }
        if (!UNI) {
            la = la_vec<real, EPT>(e0, La_d1, la0);
            if (A1) a = ldv<real, EPT>(A1 + e0);
        }
    }
    const int su = ub0 * kBlock + uoff;  // first staged vertex
    // f32: the staged (X, P) and (Ga, invAux) pairs are loaded two vertices
    // per 16-byte access from the even vertex at or below su (one load per
    // array and lane covers 512 vertices: the headline's u range is ~170) --
    // the texture addresser, not HBM, bounds this sweep, so its load
    // instructions are what counts.  f64 pairs are 16 bytes already.
    constexpr bool PAIRS = sizeof(real) == 4;
    const int sb = su & ~1, so = su - sb;  // PAIRS: entries counted from sb
    R2<real> sx[NS0], sg[NS0];
    real sr[NS0];
    Pk<real, 4> px{}, pg{};
    Pk<real, 2> pr{};
    if (staged) {
        if (PAIRS) {
            const int j = min(tid, (span + so - 1) >> 1);  // (the arrays carry 2 spare vertices)
            px = ldv<real, 4>(reinterpret_cast<const real *>(xp + sb) + 4 * j);
            if (RAT) pr = ldv<real, 2>(rr + sb + 2 * j);
            else pg = ldv<real, 4>(reinterpret_cast<const real *>(gi + sb) + 4 * j);
        } else {
#pragma unroll
            for (int q = 0; q < NS0; q++) {
                const int i = su + min(q * kBlock + tid, span - 1);
                sx[q] = xp[i];
                if (RAT) sr[q] = rr[i];
                else sg[q] = gi[i];
            }
        }
    }
    if (full) {
        int iv[EPT];
        if (nr) {  // block-uniform: v ends from the record's runs
            int vb[EPT];
#pragma unroll
            for (int j = 0; j < EPT; j++) vb[j] = rec[kErecS + 1];
            // runs in groups of four (one 32-byte scalar load each; starts
            // past the block's last run are padded, never reached)
#pragma unroll
            for (int g = 1; g < kEbRuns; g += 4) {
                if (g < nr) {  // block-uniform
#pragma unroll
                    for (int r = g; r < g + 4 && r < kEbRuns; r++) {
                        const int st = rec[kErecS + 2 * r], bs = rec[kErecS + 2 * r + 1];
#pragma unroll
                        for (int j = 0; j < EPT; j++) vb[j] = rel + j >= st ? bs : vb[j];
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < EPT; j++) iv[j] = vb[j] + (ib.v[j] >> 8);
        } else {
            const Pk<int, EPT> x = ldv<int, EPT>(Ev + e0);
#pragma unroll
            for (int j = 0; j < EPT; j++) iv[j] = x.v[j];
        }
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            pv[j] = xp[iv[j]];
            if (RAT) rv[j] = rr[iv[j]];
            else gv[j] = gi[iv[j]];
        }
    }
    if (staged) {
        if (PAIRS) {
            const int i0 = 2 * tid - so;  // LDS slot of the pair's first vertex
            if (2 * tid < span + so) {       // the pair starts inside the staged range
                if (i0 >= 0) {
                    s_xp[i0].x = px.v[0]; s_xp[i0].y = px.v[1];
                    if (RAT) s_r[i0] = pr.v[0];
                    else { s_gi[i0].x = pg.v[0]; s_gi[i0].y = pg.v[1]; }
                }
                if (i0 + 1 < span) {
                    s_xp[i0 + 1].x = px.v[2]; s_xp[i0 + 1].y = px.v[3];
                    if (RAT) s_r[i0 + 1] = pr.v[1];
                    else { s_gi[i0 + 1].x = pg.v[2]; s_gi[i0 + 1].y = pg.v[3]; }
                }
            }
            for (int i = 2 * kBlock - so + tid; i < span; i += kBlock) {  // wide ranges
                s_xp[i] = xp[su + i];
                if (RAT) s_r[i] = rr[su + i];
                else s_gi[i] = gi[su + i];
            }
        } else {
#pragma unroll
            for (int q = 0; q < NS0; q++) {
                const int i = q * kBlock + tid;
                if (i < span) {
                    s_xp[i] = sx[q];
                    if (RAT) s_r[i] = sr[q];
                    else s_gi[i] = sg[q];
                }
            }
            for (int i = NS0 * kBlock + tid; i < span; i += kBlock) {  // wide ranges
                s_xp[i] = xp[su + i];
                if (RAT) s_r[i] = rr[su + i];
                else s_gi[i] = gi[su + i];
            }
        }
    }
    __syncthreads();
    if (e0 >= E) return;
    if (full) {
        if (staged) {
            int ku[EPT];  // staged u block of each edge, then its LDS slot
#pragma unroll
            for (int j = 0; j < EPT; j++) ku[j] = (ib.v[j] & 0xff) - uoff;
            if (nub > 1) {  // block-uniform; starts of absent blocks padded
#pragma unroll
                for (int q = 1; q < NUB; q++) {
                    const int st = rec[kErecU + q];
#pragma unroll
                    for (int j = 0; j < EPT; j++) ku[j] += rel + j >= st ? kBlock : 0;
                }
            }
#pragma unroll
            for (int j = 0; j < EPT; j++) {
                pu[j] = s_xp[ku[j]];
                if (RAT) ru[j] = s_r[ku[j]];
                else gu[j] = s_gi[ku[j]];
            }
        } else {
            const Pk<int, EPT> iu = ldv<int, EPT>(Eu + e0);
#pragma unroll
            for (int j = 0; j < EPT; j++) {
                pu[j] = xp[iu.v[j]];
                if (RAT) ru[j] = rr[iu.v[j]];
                else gu[j] = gi[iu.v[j]];
            }
        }
        if (UNI) {
            const real a0 = cw * la0;
#pragma unroll
            for (int j = 0; j < EPT; j++) {
                a.v[j] = a0;
                la.v[j] = la0;
            }
        } else if (!A1) {
#pragma unroll
            for (int j = 0; j < EPT; j++) a.v[j] = cw * la.v[j];
        }
        Pk<real, EPT> ou, ov;
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            if (RAT)
                edge_ratio<real>(pu[j], pv[j], ru[j], rv[j], la0, z.v[2 * j], z.v[2 * j + 1], rho);
            else
                edge_full<real>(pu[j], pv[j], gu[j], gv[j], a.v[j], la.v[j], z.v[2 * j],
                                z.v[2 * j + 1], ou.v[j], ov.v[j], rho);
        }
        Pk<real, EPT> zu, zv;
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            zu.v[j] = z.v[2 * j];
            zv.v[j] = z.v[2 * j + 1];
        }
        stv<real, EPT>(Z2 + e0, zu);
        stv<real, EPT>(Z2 + E + e0, zv);
        if (!RAT && wz) {  // block-uniform; null: the vertex sweep forms W * Z itself
            stv<real, EPT>(wz + e0, ou);
            stv<real, EPT>(wz + E + e0, ov);
        }
    } else {
        for (long e = e0; e < E; e++) {
            const int u = Eu[e], v = Ev[e];
            real zu = Z2[e], zv = Z2[E + e], ou, ov;
            const real l = la_at(e, La_d1, la0);
            if (RAT)
                edge_ratio<real>(xp[u], xp[v], rr[u], rr[v], la0, zu, zv, rho);
            else
                edge_full<real>(xp[u], xp[v], gi[u], gi[v], A1 ? A1[e] : cw * l, l, zu, zv, ou,
                                ov, rho);
            Z2[e] = zu;
            Z2[E + e] = zv;
            if (!RAT && wz) {
                wz[e] = ou;
                wz[E + e] = ov;
            }
        }
    }
}


template <typename real, bool UNI, bool RAT = false>
__global__ __launch_bounds__(256) void k_edge_sweep_tl(
    long E, int V, const int *__restrict__ Eu, const unsigned short *__restrict__ luv,
    const int *__restrict__ erec, const int *__restrict__ Ev,
    const R2<real> *__restrict__ xp, real *__restrict__ Z2, const real *__restrict__ A1, real cw,
    const R2<real> *__restrict__ gi, const real *__restrict__ La_d1, real la0,
    real *__restrict__ wz, real rho, const Ctrl<real> *ctrl, int b0, int nb, int xcd,
    const real *__restrict__ rr = nullptr) {
    if (ctrl && ctrl->halt) return;
    constexpr int SPAN = TlBlocks<real>::v * kBlock;
    __shared__ R2<real> s_xp[SPAN];
    __shared__ R2<real> s_gi[SPAN];
    int blk = xcd_block(blockIdx.x, nb, xcd);
    if (blk >= nb) return;  // whole block
    blk += b0;  // edge blocks [b0, b0 + nb) of this launch
    tl_gather<real, UNI, RAT>(E, V, Eu, luv, erec + (long)blk * kErec, Ev, xp, Z2, A1, cw, gi,
                              La_d1, la0, wz, rho, blk, s_xp, s_gi, rr);
}

// luv[p] = (Eu[p] mod 256) | (Ev[p] mod 256) << 8: both ends within their blocks
static __global__ void k_tile_luv(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                                  unsigned short *__restrict__ luv) {
    const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < E) luv[p] = (unsigned short)((Eu[p] % kBlock) | ((Ev[p] % kBlock) << 8));
}

// nub of a block whose u blocks are not nondecreasing: never staged
constexpr int kErecNoStage = 1 << 30;

// the record of every edge block of k_edge_sweep_tl (EB edges; one wave per
// block): first u block, span and the smallest / largest u end, where each
// further u block starts, then the runs of equal v block in edge order
// (nruns = 0 when there are more than kEbRuns: the block reads Ev); starts
// relative to the block's first edge, padded past the last run.  Blocks
// [b0, nblk).  Only the block's own record is written.
//
// A partitioned rank's edge block that straddles its interior / boundary cut
// (the edges with a ghost end are sorted after the interior ones, each part
// by u block) sees the u block DROP inside the block.  Its u ends are not a
// few consecutive blocks from ub0 on, so the block is marked unstaged (nub =
// kErecNoStage: k_edge_sweep_tl reads Eu) and no u-block start is recorded
// -- u blocks below ub0 would otherwise index before the record.
static __global__ void k_tile_erec(long E, int EB, int b0, int nblk, const int *__restrict__ Eu,
                                   const int *__restrict__ Ev, int *__restrict__ erec) {
    const int blk = b0 + blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    const int lane = threadIdx.x & (kWave - 1);
    if (blk >= nblk) return;  // whole wave
    const long eb = (long)blk * EB, ee = min(eb + EB, E);
    int *r = erec + (long)blk * kErec;
    const int ub0 = Eu[eb] / kBlock;
    bool drop = false;
    for (long p = eb + 1 + lane; p < ee; p += kWave) drop |= Eu[p] / kBlock < Eu[p - 1] / kBlock;
    drop = __ballot(drop) != 0;  // wave-uniform
    int count = 0, umin = 0x7fffffff, umax = -1;
    for (long c = eb; c < ee; c += kWave) {
        const long p = c + lane;
        bool st = false;
        int vb = 0;
        if (p < ee) {
            vb = Ev[p] / kBlock;
            st = p == eb || Ev[p - 1] / kBlock != vb;
            const int u = Eu[p];
            umin = min(umin, u);
            umax = max(umax, u);
            // u blocks ub0 + q starting here (edges sorted by u block: q1 >= q0 >= 0)
            const int q1 = u / kBlock - ub0;
            const int q0 = p == eb ? q1 : Eu[p - 1] / kBlock - ub0;
            if (!drop)
                for (int q = q0 + 1; q <= q1 && q < kErecS - kErecU; q++)
                    r[kErecU + q] = (int)(p - eb);
        }
        const unsigned long long m = __ballot(st);
        const int k = count + __popcll(m & ((1ull << lane) - 1));
        if (st && k < kEbRuns) {
            r[kErecS + 2 * k] = (int)(p - eb);
            r[kErecS + 2 * k + 1] = vb * kBlock;
        }
        count += __popcll(m);
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        umin = min(umin, __shfl_xor(umin, o, kWave));
        umax = max(umax, __shfl_xor(umax, o, kWave));
    }
    const int nub = drop ? kErecNoStage : Eu[ee - 1] / kBlock - ub0 + 1;
    for (int k = count + lane; k < kEbRuns; k += kWave) {  // padding: never reached
        r[kErecS + 2 * k] = 0x7fffffff;
        r[kErecS + 2 * k + 1] = 0;
    }
    if (lane == 0) {
        r[0] = ub0;
        r[1] = nub;
        r[2] = count <= kEbRuns ? count : 0;
        r[3] = umin - ub0 * kBlock;
        r[kErecU] = umax - umin + 1;
        for (int q = drop ? 1 : max(nub, 1); q < kErecS - kErecU; q++) r[kErecU + q] = 0x7fffffff;
    }
}

// Edge sweep of a graph whose edges are sorted by their u end (uptr: first
// edge of each u, see k_uptr).  The u ends of a block's edges are a short
// vertex range [ua, ub]: the block stages their edge offsets, (X, P) and
// (Ga, invAux) pairs in LDS with coalesced loads, so the Eu stream is not
// read and only the v ends are gathered (issued before the staging, so
// the two round trips overlap); each lane finds the u end of its edges by
// a binary search of the staged offsets.  A block whose u range exceeds
// the LDS cap reads Eu.
template <typename real> struct USpan { static constexpr int v = 1024; };
// Occupancy: 86 VGPRs (f32) = 5 waves/SIMD.  Forcing 6 (80 VGPRs) or 7 (68)
// waves was slower on the headline (0.442 -> 0.450 / 0.462 ms): more loads
// in flight per SIMD only adds cache pressure here.
template <typename real, bool FD>
__global__ __launch_bounds__(256) void k_edge_sweep_us(
    long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
    const int *__restrict__ uptr, const R2<real> *__restrict__ xp, real *__restrict__ Z2,
    const real *__restrict__ A1, real cw, const R2<real> *__restrict__ gi,
    const real *__restrict__ La_d1, real la0, real *__restrict__ wz, real rho,
    const Ctrl<real> *ctrl, int nb, int xcd, ERange rg, FuseDecide<real> fd, PadOut<real> pdx) {
    if (!FD && ctrl && ctrl->halt) return;
    constexpr int EPT = Vec<real>::kPer16B;
    constexpr int CAP = USpan<real>::v;
    const PadOut<real> pd = FD ? pdx : PadOut<real>{nullptr, nullptr};
    __shared__ int s_ptr[CAP + 1];
    __shared__ R2<real> s_xp[CAP];
    __shared__ R2<real> s_gi[CAP];
    __shared__ real s_red[2][kBlock / kWave];
    __shared__ int s_halt;
    int blk = xcd_block(blockIdx.x, nb, xcd);
    if (blk >= nb) return;  // whole block
    const bool writer = blk == 0;
    // loop control (FD): its loads in flight under the edge streams
    FdRegs<real> fr;
    int halt = 0;
    if (FD) {
        if (fd.src) fd_load(fd, fr);
        else if (ctrl) halt = ctrl->halt;
    }
    long ebeg, eend;
    rg.pick(blk, ebeg, eend);
    const int tid = threadIdx.x;
    const long eb = ebeg + (long)blk * kBlock * EPT;
    const long el = min(eb + (long)kBlock * EPT, eend) - 1;  // block's last edge
    const int ua = Eu[eb], ub = Eu[el];
    const int span = ub - ua + 1;
    const bool staged = span <= CAP;  // block-uniform
    const long e0 = eb + (long)tid * EPT;
    const bool full = e0 + EPT <= eend;
    // streams and v-end gathers first: their latency hides under the staging
    Pk<int, EPT> iv{};
    Pk<real, 2 * EPT> z{};
    Pk<real, EPT> la{}, a{};
    Pk<int, 2 * EPT> sv{};
    R2<real> pu[EPT], pv[EPT], gu[EPT], gv[EPT];
    if (full) {
        iv = ldv<int, EPT>(Ev + e0);
        z = ldv<real, 2 * EPT>(Z2 + 2 * e0);
        la = la_vec<real, EPT>(e0, La_d1, la0);
        if (A1) a = ldv<real, EPT>(A1 + e0);
        if (pd.sl) sv = ldv<int, 2 * EPT>(pd.sl + 2 * e0);
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            pv[j] = xp[iv.v[j]];
            gv[j] = gi[iv.v[j]];
        }
    }
    if (staged) {
        for (int i = tid; i <= span; i += kBlock) s_ptr[i] = uptr[ua + i];
        for (int i = tid; i < span; i += kBlock) {
            s_xp[i] = xp[ua + i];
            s_gi[i] = gi[ua + i];
        }
    }
    __syncthreads();
    if (FD && fd.src) halt = fd_decide(fd, fr, writer, s_red, &s_halt);
    if (FD && halt) return;  // block-uniform
    if (e0 >= eend) return;
    if (full) {
        if (staged) {
            int lo = 0, hi = span - 1;  // largest k with s_ptr[k] <= e0
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if ((long)s_ptr[mid] <= e0) lo = mid;
                else hi = mid - 1;
            }
#pragma unroll
            for (int j = 0; j < EPT; j++) {
                while (lo + 1 < span && (long)s_ptr[lo + 1] <= e0 + j) lo++;
                pu[j] = s_xp[lo];
                gu[j] = s_gi[lo];
            }
        } else {
            const Pk<int, EPT> iu = ldv<int, EPT>(Eu + e0);
#pragma unroll
            for (int j = 0; j < EPT; j++) {
                pu[j] = xp[iu.v[j]];
                gu[j] = gi[iu.v[j]];
            }
        }
        if (!A1) {
#pragma unroll
            for (int j = 0; j < EPT; j++) a.v[j] = cw * la.v[j];
        }
        Pk<real, EPT> ou, ov;
#pragma unroll
        for (int j = 0; j < EPT; j++)
            edge_full<real>(pu[j], pv[j], gu[j], gv[j], a.v[j], la.v[j], z.v[2 * j],
                            z.v[2 * j + 1], ou.v[j], ov.v[j], rho);
        stv<real, 2 * EPT>(Z2 + 2 * e0, z);
        if (pd.sl) {
#pragma unroll
            for (int j = 0; j < EPT; j++) {
                pd.wzp[sv.v[2 * j]] = ou.v[j];
                pd.wzp[sv.v[2 * j + 1]] = ov.v[j];
            }
        } else {
            stv<real, EPT>(wz + e0, ou);
            stv<real, EPT>(wz + E + e0, ov);
        }
    } else {
        for (long e = e0; e < eend; e++) {
            const int u = Eu[e], v = Ev[e];
            real zu = Z2[2 * e], zv = Z2[2 * e + 1], ou, ov;
            const real l = la_at(e, La_d1, la0);
            edge_full<real>(xp[u], xp[v], gi[u], gi[v], A1 ? A1[e] : cw * l, l, zu, zv, ou, ov,
                            rho);
            Z2[2 * e] = zu;
            Z2[2 * e + 1] = zv;
            if (pd.sl) {
                pd.wzp[pd.sl[2 * e]] = ou;
                pd.wzp[pd.sl[2 * e + 1]] = ov;
            } else {
                wz[e] = ou;
                wz[E + e] = ov;
            }
        }
    }
}

template <typename real>
struct VArgs {
    int V;
    int nb, xcd;            // logical blocks of this launch, XCD-aware order
    int bbeg;               // first block of this launch (vertex block bbeg*256)
    int bsplit, bjump;      // logical blocks >= bsplit skip bjump blocks (two ranges)
    const int *ptr;
    const unsigned *idx;
    const int *uptr;        // split incidence (null: CSR gather everywhere)
    const unsigned *mask, *oidx;
    const int *blkok;       // per block: 1 = split path
    const real *wz;         // contributions (local side-major, then received)
    R2<real> *xp;
    R2<real> *xpo;          // where the new (X, P) go (null: xp, in place)
    const real *Y, *A, *Ga, *Th_l1;
    int prox, positivity;
    real lo, hi;
    int fwd;        // 0: keep P (dense modes), 1: identity, 2: diagonal A
    int track;      // iterate-evolution partials
    real *part;     // 2 per block
    const Ctrl<real> *ctrl;
    int late;       // halt of ctrl tested after the sum, before the stores (small launches)
    // tiled contributions (null d2: off; see tile_sum)
    long E;
    const Slots12 *slots;
    const int *trec;        // per-block records (tile_sum_rec; tok == 2)
    const Slots12 *ptab;    // slot patterns (null: per-entry slots; see k_run_hash)
    const int *prec;        // per record block: its runs' pattern offsets
    const unsigned char *deg8;
    const int *ustart, *tptr, *tstart, *tlen, *tok;
    // Z-direct (tiled single-GPU sessions with one edge weight, no A1): the
    // lists hold Z (side-major, zs) and each term is (a0 * invAux[v]) * z
    const real *zs;
    const real *invAux;
    real a0;
    // per-vertex constants: gi = (Ga, invAux) pairs (null: the separate
    // arrays); l1uni: La_l1 is one value l1u, so Th_l1 = Ga * l1u (the
    // preconditioner's own product, k_precond_vertex) is not read
    const R2<real> *gi;
    int l1uni;
    real l1u;
    // sequential evolution statistic (null: off): the terms (X_ - X)^2 at
    // terms[i] and X^2 at terms[tstride + i], i = the vertex's label in the
    // caller's order (tmap[v] for a relabelled session, else v), summed
    // afterwards in that order with the reference's rounding (mono_sum)
    real *terms;
    const int *tmap;
    long tstride;
};

// DR average (ordered), prox on the iterate, evolution partials, next
// forward step (ref :491-529 then :355-464 of the next iteration)
// occupancy target of the vertex sweep: 8 waves/SIMD in f32 (LDS allows 9
// blocks per CU), 4 in f64 (32 KiB of LDS per block)
template <typename real> struct VSweep;
template <> struct VSweep<float> { static constexpr int waves = 8; };
template <> struct VSweep<double> { static constexpr int waves = 4; };

// per-vertex operands of the vertex sweep (loaded before the sum: their
// latency hides under the gather)
template <typename real>
struct VOps {
    R2<real> q{};
    real th = real(0), yv = real(0), gv = real(0), av = real(0), ia = real(0);
};
// The old iterate (X_, P_) is read only where it is used: the evolution
// terms (tracked) or the dense modes (P kept until their forward step); an
// untracked identity / diagonal-A sweep overwrites both (8 B per vertex).
template <typename real>
__device__ __forceinline__ VOps<real> vertex_ops(const VArgs<real> &a, int v,
                                                 const R2<real> *gpre = nullptr) {
    VOps<real> o;
    if (v < a.V) {
        if (a.track || !a.fwd) o.q = a.xp[v];
        real g = real(0);
        if (a.gi) {
            const R2<real> p = gpre ? *gpre : a.gi[v];  // (gpre: loaded by the caller)
            g = p.x;
            o.ia = p.y;
        } else if (a.fwd || a.l1uni) {
            g = a.Ga[v];
        }
        if (a.prox == PROX_L1) o.th = a.l1uni ? g * a.l1u : a.Th_l1[v];
        if (a.fwd) { o.yv = a.Y[v]; o.gv = g; }
        if (a.fwd == 2) o.av = a.A[v];
    }
    return o;
}

// after the ordered sum x of vertex v: prox, evolution terms, next forward
// step (ref :499-529 then :355-464 of the next iteration)
template <typename real>
__device__ __forceinline__ R2<real> vertex_finish(const VArgs<real> &a, int v, real x,
                                                  const VOps<real> &o, real &num, real &den) {
    num = real(0);
    den = real(0);
    R2<real> q = o.q;
    const real th = o.th, yv = o.yv, gv = o.gv, av = o.av;
    if (v < a.V) {
        switch (a.prox) {
            case PROX_L1: {
                if (x > th) x -= th;
                else if (!a.positivity && (x < -th)) x += th;
                else x = real(0);
            } break;
            case PROX_POS:
                if (x < real(0)) x = real(0);
                break;
            case PROX_BOX:
                if (x < a.lo) x = a.lo;
                else if (x > a.hi) x = a.hi;
                break;
            case PROX_LO:
                if (x < a.lo) x = a.lo;
                break;
            case PROX_HI:
                if (x > a.hi) x = a.hi;
                break;
            default:
                break;
        }
        if (a.track) {
            const real d = q.x - x;
            num = d * d;
            den = x * x;
            if (a.terms) {
                const long i = a.tmap ? a.tmap[v] : v;
                a.terms[i] = num;
                a.terms[a.tstride + i] = den;
            }
        }
        q.x = x;
        if (a.fwd) {
            real p = (a.fwd == 2) ? av * x : x;
            p -= yv;
            q.y = real(2) * x - gv * p;
        }
        (a.xpo ? a.xpo : a.xp)[v] = q;
    }
    return q;
}

// one vertex block `blk` (all 256 lanes of the calling block take part)
template <typename real, int GB, bool ZD = false>
__device__ __forceinline__ void vertex_block(const VArgs<real> &a, int blk, real *lds,
                                             real (*red)[kBlock / kWave], int *scan,
                                             int halt = 0) {
    const int v0 = blk * kBlock;
    const int v = v0 + threadIdx.x;
    const VOps<real> o = vertex_ops(a, v);
    // ZD: the vertex's splitting weight, as the edge sweep forms it (a * invAux)
    const real wv = ZD && v < a.V ? a.a0 * (a.gi ? o.ia : a.invAux[v]) : real(1);
    real x;
    // the block's record, pattern offsets and degree in the same load round
    // as its tok and the vertex operands (every block has a record slot; only
    // tok == 2 blocks read it): two dependent rounds to the contributions
    // instead of three
    const bool pre = a.slots && a.trec;  // launch-uniform
    int pre_rv = 0, pre_pr = 0, pre_dg = 0;
    if (pre) {
        const int lane = threadIdx.x & (kWave - 1);
        pre_rv = lane < kTileRec ? a.trec[(long)blk * kTileRec + lane] : 0;
        pre_pr = a.prec && lane < kPrec ? a.prec[(long)blk * kPrec + lane] : 0;
        pre_dg = v < a.V ? a.deg8[v] : 0;
    }
    const int tk = a.slots ? a.tok[blk] : 0;  // block-uniform
    if (tk == 2)
        x = tile_sum_rec<real, ZD>(a.V, a.E, blk, v, a.deg8, a.slots, a.trec, ZD ? a.zs : a.wz,
                                   lds, scan + 3 * kTileRuns, wv, a.ptab, a.prec, pre, pre_rv,
                                   pre_pr, pre_dg);
    else if (tk)
        x = tile_sum<real, GB, ZD>(a.V, a.E, blk, v, a.deg8, a.slots, a.ustart, a.tptr, a.tstart,
                                   a.tlen, ZD ? a.zs : a.wz, lds, scan, wv);
    else if (!ZD && a.blkok && a.blkok[blk])
        x = split_sum<real, GB>(a.V, v0, v, a.ptr, a.uptr, a.mask, a.oidx, a.wz, lds, scan);
    else
        x = gather_sum<real, GatherCap<real>::v, GB, ZD>(a.V, v0, a.ptr, a.idx,
                                                         ZD ? a.zs : a.wz, lds, wv);
    if (halt) return;  // block-uniform (a.late)
    real num, den;
    vertex_finish(a, v, x, o, num, den);
    if (a.track) {
        num = block_sum(num, red[0]);
        den = block_sum(den, red[1]);
        if (threadIdx.x == 0) {
            a.part[2 * blk] = num;
            a.part[2 * blk + 1] = den;
        }
    }
}

template <typename real, int GB, bool ZD = false>
__global__ __launch_bounds__(256, VSweep<real>::waves) void k_vertex_sweep(VArgs<real> a) {
    int halt = 0;
    if (a.ctrl) {
        if (!a.late) {
            if (a.ctrl->halt) return;
        } else {
            halt = a.ctrl->halt;  // waited for only after the sum's loads
        }
    }
    __shared__ real lds[GatherCap<real>::v];
    __shared__ real red[2][kBlock / kWave];
    __shared__ int scan[3 * kTileRuns + kBlock / kWave];  // block scan (split_sum) / run table
                                                         // and degree totals (tile_sum)
    // the logical blocks LAST to first: the edge sweep before this one walked
    // its tiles first to last, so the contributions it wrote last are the
    // ones still in the 256 MB Infinity Cache when this sweep starts, and the
    // blocks this sweep ends on are the ones the next edge sweep starts with
    // (headline: vertex sweep 0.180 -> 0.167 ms, edge sweep 0.283 -> 0.277;
    // C2 0.482 -> 0.468 ms/iter, r6a / r6c)
    int lb = xcd_block(blockIdx.x, a.nb, a.xcd);
    if (lb >= a.nb) return;
    lb = a.nb - 1 - lb;
    if (lb >= a.bsplit) lb += a.bjump;
    vertex_block<real, GB, ZD>(a, a.bbeg + lb, lds, red, scan, halt);
}

// The pair vertex sweep (single-GPU or one range of record blocks only,
// every block a record block, f32): a workgroup takes the consecutive
// blocks 2p, 2p + 1 of the launch (pairs walked last to first, as
// k_vertex_sweep walks blocks), both blocks' contributions staged together
// (tile_sum_rec2) into a dynamic LDS list of 2 cap entries, cap = the
// largest record block's entry count; an odd last block is launched on its
// own (k_vertex_sweep).  Block partials stay per vertex block.
template <typename real, bool ZD = false>
__global__ __launch_bounds__(256, 7) void k_vertex_sweep_pair(VArgs<real> a, int cap) {
    int halt = 0;
    if (a.ctrl) {
        if (!a.late) {
            if (a.ctrl->halt) return;
        } else {
            halt = a.ctrl->halt;
        }
    }
    extern __shared__ __attribute__((aligned(16))) unsigned char vpair_lds[];
    real *lds = reinterpret_cast<real *>(vpair_lds);
    __shared__ real red[2][kBlock / kWave];
    __shared__ int scan[3 * kTileRuns + 2 * (kBlock / kWave)];  // (the degree totals)
    const int np = a.nb / 2;  // (an odd last block: a k_vertex_sweep launch of its own)
    int lp = xcd_block(blockIdx.x, np, a.xcd);
    if (lp >= np) return;
    lp = np - 1 - lp;
    const int b0 = a.bbeg + 2 * lp;
    const int v0 = b0 * kBlock + threadIdx.x, v1 = v0 + kBlock;
    const VOps<real> o0 = vertex_ops(a, v0);
    const real wv0 = ZD && v0 < a.V ? a.a0 * (a.gi ? o0.ia : a.invAux[v0]) : real(1);
    real x0, x1;
    // block b0 + 1's metric pair now (its weight), its other operands after
    // the sum (registers)
    R2<real> g1{};
    if (a.gi && v1 < a.V) g1 = a.gi[v1];
    const real wv1 = ZD && v1 < a.V ? a.a0 * (a.gi ? g1.y : a.invAux[v1]) : real(1);
    tile_sum_rec2<real, ZD>(a.V, a.E, b0, v0, v1, a.deg8, a.slots, a.trec, ZD ? a.zs : a.wz, lds,
                            cap, scan + 3 * kTileRuns, wv0, wv1, a.ptab, a.prec, x0, x1);
    if (halt) return;  // block-uniform (a.late)
    const VOps<real> o1 = vertex_ops(a, v1, a.gi ? &g1 : nullptr);
    real n0, d0, n1, d1;
    vertex_finish(a, v0, x0, o0, n0, d0);
    vertex_finish(a, v1, x1, o1, n1, d1);
    if (a.track) {
        n0 = block_sum(n0, red[0]);
        d0 = block_sum(d0, red[1]);
        n1 = block_sum(n1, red[0]);
        d1 = block_sum(d1, red[1]);
        if (threadIdx.x == 0) {
            a.part[2 * b0] = n0;
            a.part[2 * b0 + 1] = d0;
            a.part[2 * b0 + 2] = n1;
            a.part[2 * b0 + 3] = d1;
        }
    }
}

// entries of each record block's list (0 for the others): the pair sweep's
// LDS list per block is the largest
static __global__ void k_rec_entries(int V, int nb, const int *__restrict__ ptr,
                                     const int *__restrict__ tok, int *__restrict__ out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    out[b] = tok[b] == 2 ? ptr[min((b + 1) * kBlock, V)] - ptr[b * kBlock] : 0;
}

// Vertex sweep of a small graph (the fused-decision range) whose edge sweep
// stores the contributions block by block (PadOut): vertex block b's CSR
// entries are wzp[b * nmax ...) in CSR order, so the block stages them with
// loads whose addresses depend on nothing loaded, issued together with the
// per-vertex operands and the CSR pointers -- one dependent round trip
// instead of three (pointers -> other-entry addresses -> gathered
// contributions), which is what a latency-bound launch pays for.  Each lane
// then adds its vertex's entries in CSR order from LDS (the sums of
// split_sum / gather_sum, bit for bit) and finishes as vertex_block does.
constexpr int kPadPer = 16;  // staged entries per lane: nmax <= kPadPer * kBlock
template <typename real>
__global__ __launch_bounds__(256) void k_vertex_sweep_pad(VArgs<real> a,
                                                          const real *__restrict__ wzp, int nmax,
                                                          const int *__restrict__ pidx,
                                                          R2<real> *__restrict__ xpe) {
    static_assert(kPadPer * kBlock <= GatherCap<real>::v, "staged list fits the LDS chunk");
    int halt = 0;
    if (a.ctrl) {
        if (!a.late) {
            if (a.ctrl->halt) return;
        } else {
            halt = a.ctrl->halt;  // waited for only after the sum's loads
        }
    }
    __shared__ real lds[kPadPer * kBlock];
    __shared__ int sidx[kPadPer * kBlock];
    __shared__ real red[2][kBlock / kWave];
    const int lb = xcd_block(blockIdx.x, a.nb, a.xcd);
    if (lb >= a.nb) return;
    const int blk = a.bbeg + lb;
    const int tid = threadIdx.x, v0 = blk * kBlock, v = v0 + tid;
    const VOps<real> o = vertex_ops(a, v);
    const int p0 = a.ptr[v0];
    const int my0 = v < a.V ? a.ptr[v] : 0, my1 = v < a.V ? a.ptr[v + 1] : 0;
    const real *src = wzp + (long)blk * nmax;
    const int per = nmax / kBlock;  // block-uniform
    real w[kPadPer];
    int pe[kPadPer];
#pragma unroll
    for (int k = 0; k < kPadPer; k++)
        if (k < per) {
            w[k] = src[k * kBlock + tid];
            if (xpe) pe[k] = pidx[(long)blk * nmax + k * kBlock + tid];
        }
#pragma unroll
    for (int k = 0; k < kPadPer; k++)
        if (k < per) {
            lds[k * kBlock + tid] = w[k];
            if (xpe) sidx[k * kBlock + tid] = pe[k];
        }
    __syncthreads();
    real x = real(0);
    for (int j = my0; j < my1; j++) x += lds[j - p0];
    if (halt) return;  // block-uniform
    real num, den;
    const R2<real> q = vertex_finish(a, v, x, o, num, den);
    // (X, P) to the copies the next edge sweep streams: entry j of this
    // vertex is the end (e, side) = pidx of the edge that contributed it
    if (xpe && v < a.V)
        for (int j = my0; j < my1; j++) xpe[sidx[j - p0]] = q;
    if (a.track) {
        num = block_sum(num, red[0]);
        den = block_sum(den, red[1]);
        if (tid == 0) {
            a.part[2 * blk] = num;
            a.part[2 * blk + 1] = den;
        }
    }
}

// Edge sweep of a padded session whose endpoint data arrive as per-edge
// copies (written by the previous vertex sweep / k_pad_ends): (X, P) and
// (Ga, 1/Aux) of both ends of edge e at xpe / gie [2e + side], so every
// load of the sweep is a stream (no endpoint index, no gather: one
// dependent round trip); contributions stored through sl as in PadOut.
// Fused decision as k_edge_sweep<real, true>.
template <typename real>
__global__ __launch_bounds__(256) void k_edge_sweep_ends(
    long E, const R2<real> *__restrict__ xpe, const R2<real> *__restrict__ gie,
    real *__restrict__ Z2, const real *__restrict__ A1, real cw,
    const real *__restrict__ La_d1, real la0, real rho, const Ctrl<real> *ctrl, int nb, int xcd,
    FuseDecide<real> fd, PadOut<real> pd) {
    constexpr int EPT = Vec<real>::kPer16B;
    const int blk = xcd_block(blockIdx.x, nb, xcd);
    if (blk >= nb) return;
    __shared__ real red[2][kBlock / kWave];
    __shared__ int s_halt;
    FdRegs<real> fr;
    int halt = 0;
    if (fd.src) fd_load(fd, fr);
    else if (ctrl) halt = ctrl->halt;
    const long e0 = ((long)blk * blockDim.x + threadIdx.x) * EPT;
    const bool full = e0 + EPT <= E;
    R2<real> pu[EPT], pv[EPT], gu[EPT], gv[EPT];
    Pk<real, 2 * EPT> z{};
    Pk<real, EPT> la{}, a{};
    Pk<int, 2 * EPT> sv{};
    if (full) {
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            pu[j] = xpe[2 * (e0 + j)]; pv[j] = xpe[2 * (e0 + j) + 1];
            gu[j] = gie[2 * (e0 + j)]; gv[j] = gie[2 * (e0 + j) + 1];
        }
        z = ldv<real, 2 * EPT>(Z2 + 2 * e0);
        la = la_vec<real, EPT>(e0, La_d1, la0);
        if (A1) a = ldv<real, EPT>(A1 + e0);
        sv = ldv<int, 2 * EPT>(pd.sl + 2 * e0);
    }
    if (fd.src) halt = fd_decide(fd, fr, blk == 0, red, &s_halt);
    if (halt || e0 >= E) return;  // halt is block-uniform
    if (full) {
        if (!A1) {
#pragma unroll
            for (int j = 0; j < EPT; j++) a.v[j] = cw * la.v[j];
        }
        Pk<real, EPT> ou, ov;
#pragma unroll
        for (int j = 0; j < EPT; j++)
            edge_full<real>(pu[j], pv[j], gu[j], gv[j], a.v[j], la.v[j], z.v[2 * j],
                            z.v[2 * j + 1], ou.v[j], ov.v[j], rho);
        stv<real, 2 * EPT>(Z2 + 2 * e0, z);
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            pd.wzp[sv.v[2 * j]] = ou.v[j];
            pd.wzp[sv.v[2 * j + 1]] = ov.v[j];
        }
    } else {
        for (long e = e0; e < E; e++) {
            real zu = Z2[2 * e], zv = Z2[2 * e + 1], ou, ov;
            const real l = la_at(e, La_d1, la0);
            edge_full<real>(xpe[2 * e], xpe[2 * e + 1], gie[2 * e], gie[2 * e + 1],
                            A1 ? A1[e] : cw * l, l, zu, zv, ou, ov, rho);
            Z2[2 * e] = zu;
            Z2[2 * e + 1] = zv;
            pd.wzp[pd.sl[2 * e]] = ou;
            pd.wzp[pd.sl[2 * e + 1]] = ov;
        }
    }
}

// the per-edge endpoint copies from the vertex arrays (setup, and after a
// reconditioning rewrote (X, P) and (Ga, 1/Aux))
template <typename real>
__global__ void k_pad_ends(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                           const R2<real> *__restrict__ xp, const R2<real> *__restrict__ gi,
                           R2<real> *__restrict__ xpe, R2<real> *__restrict__ gie) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int u = Eu[e], v = Ev[e];
    xpe[2 * e] = xp[u];
    xpe[2 * e + 1] = xp[v];
    gie[2 * e] = gi[u];
    gie[2 * e + 1] = gi[v];
}

// largest CSR entry count of a vertex block (atomicMax into *out)
static __global__ void k_pad_nmax(int V, int nb, const int *__restrict__ ptr, int *out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    atomicMax(out, ptr[min(V, (b + 1) * kBlock)] - ptr[b * kBlock]);
}

// slot of every contribution (e, side) in its vertex block's padded list:
// sl[2e + side] = b * nmax + (CSR position - first position of block b)
// and, with pidx, the end 2e + side of each list entry
static __global__ void k_pad_slots(int V, long E, const int *__restrict__ ptr,
                                   const unsigned *__restrict__ idx, int nmax, int *__restrict__ sl,
                                   int *__restrict__ pidx) {
    const int v = blockIdx.x * kBlock + threadIdx.x;
    if (v >= V) return;
    const int b = v / kBlock, base = ptr[b * kBlock];
    for (int j = ptr[v]; j < ptr[v + 1]; j++) {
        const long addr = idx[j];
        const long side = addr >= E ? 1 : 0;
        const long end = 2 * (addr - side * E) + side;
        sl[end] = b * nmax + (j - base);
        if (pidx) pidx[(long)b * nmax + (j - base)] = (int)end;
    }
}

// fixed-order sum of per-block partial pairs into out[0..1]
template <typename real>
__global__ __launch_bounds__(256) void k_reduce_pairs(int nparts, const real *__restrict__ part,
                                                      real *__restrict__ out, int stride) {
    __shared__ real red[2][kBlock / kWave];
    real a = real(0), b = real(0);
    for (int i = threadIdx.x; i < nparts; i += kBlock) {
        a += part[2 * i];
        b += part[2 * i + 1];
    }
    a = block_sum(a, red[0]);
    b = block_sum(b, red[1]);
    if (threadIdx.x == 0) { out[0] = a; out[stride] = b; }
}

// single GPU: the fixed-order partial sums of k_reduce_pairs and the
// decision of k_decide in one launch (one kernel boundary less per
// iteration, which counts for small graphs)
template <typename real>
__device__ __forceinline__ void reduce_decide_block(int nparts, const real *__restrict__ part,
                                                    real *__restrict__ out, Ctrl<real> *ctrl,
                                                    real *__restrict__ Dif, int track,
                                                    real (*red)[kBlock / kWave]) {
    real a = real(0), b = real(0);
    if (track) {
        for (int i = threadIdx.x; i < nparts; i += kBlock) {
            a += part[2 * i];
            b += part[2 * i + 1];
        }
        a = block_sum(a, red[0]);
        b = block_sum(b, red[1]);
    }
    if (threadIdx.x == 0) {
        if (track) { out[0] = a; out[1] = b; }
        decide_step(ctrl, a, b, Dif, track);
    }
}

template <typename real>
__global__ __launch_bounds__(256) void k_reduce_decide(int nparts, const real *__restrict__ part,
                                                       real *__restrict__ out, Ctrl<real> *ctrl,
                                                       real *__restrict__ Dif, int track) {
    __shared__ real red[2][kBlock / kWave];
    if (ctrl->halt) return;  // uniform
    reduce_decide_block(nparts, part, out, ctrl, Dif, track, red);
}

// ------------------------------------------------ small graphs, one launch --
// Up to `iters` whole iterations of a small single-GPU graph in ONE
// workgroup: edge pass (per-edge edge_full, as the sweeps' lanes do), the
// vertex pass (the ordered sums, vertex_finish and the per-block evolution
// partials), the fixed-order reduction and decision (decide_step), with
// workgroup barriers between the phases.  Every value is computed by the
// same device code or the same sequence of operations as the multi-launch
// path, so the iterates are identical bit for bit; what goes is the 2-3
// launches per iteration that bound CP's reduced problems (~10 us each).
template <typename real>
struct TinyArgs {
    long E;
    const int *Eu, *Ev;
    real *Z2;
    const real *A1, *La_d1;
    real la0;           // every edge's weight when La_d1 is null
    real cw, rho;
    const R2<real> *gi;
    real *wz;
    VArgs<real> va;     // nb = every vertex block, bbeg 0
    real *red;          // (num, den) of the last evolution
    Ctrl<real> *ctrl;   // null: no tracking, run exactly `iters`
    real *Dif;
    int track, iters;
};

// 1024 lanes: four vertex blocks at a time; each lane adds its vertex's
// CSR entries in order directly (the sequence gather_sum / split_sum add),
// then vertex_finish; the evolution partials of each 256-vertex block and
// the reduction before the decision repeat block_sum's tree exactly
// (wave_sum, then the block's 4 wave sums in order).
constexpr int kTiny = 1024;

// Memory-level parallelism inside the one workgroup (everything it touches
// sits in its XCD's L2, so each dependent round trip is an L2 latency): the
// edge pass runs k_edge_sweep's lane body (EPT edges per lane, 16-byte
// streams, the endpoint gathers of all EPT edges issued together), the
// vertex pass loads 8 CSR addresses, then 8 contributions, at a time and
// adds them in order, and the loop control stays in registers / LDS (the
// control block is stored each iteration, never re-read; the per-block
// partials are summed from LDS).
constexpr int kTinyMaxBlocks = 32;

template <typename real>
__global__ __launch_bounds__(kTiny) void k_tiny_iterate(TinyArgs<real> t) {
    constexpr int EPT = Vec<real>::kPer16B;
    __shared__ real wred[2][kTiny / kWave];
    __shared__ real bpart[2][kTinyMaxBlocks];
    __shared__ int halt;
    const int tid = threadIdx.x;
    const VArgs<real> &a = t.va;
    R2<real> *xp = a.xp;
    Ctrl<real> c{};
    if (tid == 0) {
        if (t.ctrl) c = *t.ctrl;
        halt = t.ctrl ? c.halt : 0;
    }
    __syncthreads();
    for (int it = 0; it < t.iters; it++) {
        if (halt) break;  // uniform (set by lane 0 before the last barrier)
        for (long e0 = (long)tid * EPT; e0 < t.E; e0 += (long)kTiny * EPT)
            edge_lane<real>(e0, t.E, t.E, t.Eu, t.Ev, xp, t.Z2, t.A1, t.cw, t.gi, t.La_d1, t.la0, t.wz,
                            t.rho);
        __syncthreads();
        for (int b0 = 0; b0 < a.nb; b0 += kTiny / kBlock) {
            const int blk = b0 + tid / kBlock;
            const int v = blk * kBlock + (tid & (kBlock - 1));
            real num = real(0), den = real(0);
            if (blk < a.nb) {
                const VOps<real> o = vertex_ops(a, v);
                real x = real(0);
                if (v < a.V) {
                    const int j1 = a.ptr[v + 1];
                    for (int j = a.ptr[v]; j < j1; j += 8) {
                        unsigned id[8];
                        real w[8];
#pragma unroll
                        for (int q = 0; q < 8; q++) id[q] = j + q < j1 ? a.idx[j + q] : 0u;
#pragma unroll
                        for (int q = 0; q < 8; q++) w[q] = j + q < j1 ? a.wz[id[q]] : real(0);
#pragma unroll
                        for (int q = 0; q < 8; q++)
                            if (j + q < j1) x += w[q];
                    }
                }
                vertex_finish(a, v, x, o, num, den);
            }
            if (a.track) {
                num = wave_sum(num);
                den = wave_sum(den);
                if ((tid & (kWave - 1)) == 0) { wred[0][tid / kWave] = num; wred[1][tid / kWave] = den; }
                __syncthreads();
                if ((tid & (kBlock - 1)) == 0 && blk < a.nb) {
                    real sn = real(0), sd = real(0);
                    const int w0 = tid / kWave;
                    for (int i = 0; i < kBlock / kWave; i++) { sn += wred[0][w0 + i]; sd += wred[1][w0 + i]; }
                    bpart[0][blk] = sn;
                    bpart[1][blk] = sd;
                    a.part[2 * blk] = sn;
                    a.part[2 * blk + 1] = sd;
                }
                __syncthreads();
            }
        }
        __syncthreads();
        if (t.ctrl) {  // k_reduce_decide on the first 256 lanes, its tree exactly
            real sa = real(0), sb = real(0);
            if (t.track && tid < kBlock)
                for (int i = tid; i < a.nb; i += kBlock) { sa += bpart[0][i]; sb += bpart[1][i]; }
            sa = wave_sum(sa);
            sb = wave_sum(sb);
            if ((tid & (kWave - 1)) == 0 && tid < kBlock) { wred[0][tid / kWave] = sa; wred[1][tid / kWave] = sb; }
            __syncthreads();
            if (tid == 0) {
                real na = real(0), nb = real(0);
                if (t.track)
                    for (int i = 0; i < kBlock / kWave; i++) { na += wred[0][i]; nb += wred[1][i]; }
                if (t.track) { t.red[0] = na; t.red[1] = nb; }
                decide_step(&c, na, nb, t.Dif, t.track);
                *t.ctrl = c;
                halt = c.halt;
            }
        }
        __syncthreads();
    }
}

// the decision closing a chunk of fused bodies (FuseDecide): one workgroup,
// k_reduce_decide's loop and tree, from fd.src into fd.dst
template <typename real>
__global__ __launch_bounds__(256) void k_decide_fused(FuseDecide<real> fd) {
    __shared__ real red[2][kBlock / kWave];
    __shared__ int s_halt;
    FdRegs<real> r;
    fd_load(fd, r);
    (void)fd_decide(fd, r, true, red, &s_halt);
}

template <typename real>
__global__ void k_decide(Ctrl<real> *ctrl, const real *__restrict__ red,
                         real *__restrict__ Dif, int track) {
    if (threadIdx.x != 0 || ctrl->halt) return;
    decide_step(ctrl, track ? red[0] : real(0), track ? red[1] : real(0), Dif, track);
}

// ------------------------------------------------------------ objective --
// partials: [0, nbv) data term, [nbv, 2 nbv) l1 term, [2 nbv, 2 nbv + nbe)
// TV term, then the squared residual partials (direct mode).
template <typename real>
__global__ __launch_bounds__(256) void k_obj_vertex(
    int V, int mode, const R2<real> *__restrict__ xp,
    const real *__restrict__ A, const real *__restrict__ papp,
    const real *__restrict__ Y, const real *__restrict__ La_l1,
    real *__restrict__ part, int nbv, const Ctrl<real> *ctrl) {
    if (gated(ctrl, GATE_OBJ)) return;
    __shared__ real red[2][kBlock / kWave];
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    real dat = real(0), l1 = real(0);
    if (v < V) {
        const real x = xp[v].x;
        if (mode != A_DIRECT) {
            const real p = (mode == A_IDENT) ? x : (mode == A_DIAG ? A[v] * x : papp[v]);
            dat = x * (real(0.5) * p - Y[v]);
        }
        if (La_l1) l1 = (x < real(0)) ? -(La_l1[v] * x) : La_l1[v] * x;
    }
    dat = block_sum(dat, red[0]);
    l1 = block_sum(l1, red[1]);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = dat;
        part[nbv + blockIdx.x] = l1;
    }
}

template <typename real>
__global__ __launch_bounds__(256) void k_obj_edge(
    long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
    const R2<real> *__restrict__ xp, const real *__restrict__ La_d1,
    real *__restrict__ part, const Ctrl<real> *ctrl) {
    if (gated(ctrl, GATE_OBJ)) return;
    __shared__ real red[kBlock / kWave];
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    real t = real(0);
    if (e < E) {
        const real b = xp[Eu[e]].x - xp[Ev[e]].x;
        t = (b < real(0)) ? -(La_d1[e] * b) : La_d1[e] * b;
    }
    t = block_sum(t, red);
    if (threadIdx.x == 0) part[blockIdx.x] = t;
}

template <typename real>
__global__ __launch_bounds__(256) void k_obj_rsq(int N,
                                                 const real *__restrict__ R,
                                                 real *__restrict__ part,
                                                 const Ctrl<real> *ctrl) {
    if (gated(ctrl, GATE_OBJ)) return;
    __shared__ real red[kBlock / kWave];
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    real t = (n < N) ? R[n] * R[n] : real(0);
    t = block_sum(t, red);
    if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// objective partials -> red[0..2] = (data, l1, tv)
template <typename real>
__global__ __launch_bounds__(256) void k_obj_reduce(
    const real *__restrict__ part, int nbv, int nbe, int nbn, int direct,
    const Ctrl<real> *ctrl, real *__restrict__ red3) {
    __shared__ real red[3][kBlock / kWave];
    if (ctrl && ctrl->obj_it >= ctrl->it) return;
    real dat = real(0), l1 = real(0), tv = real(0);
    if (direct) {
        for (int i = threadIdx.x; i < nbn; i += kBlock) dat += part[2 * nbv + nbe + i];
    } else {
        for (int i = threadIdx.x; i < nbv; i += kBlock) dat += part[i];
    }
    for (int i = threadIdx.x; i < nbv; i += kBlock) l1 += part[nbv + i];
    for (int i = threadIdx.x; i < nbe; i += kBlock) tv += part[2 * nbv + i];
    dat = block_sum(dat, red[0]);
    l1 = block_sum(l1, red[1]);
    tv = block_sum(tv, red[2]);
    if (threadIdx.x == 0) { red3[0] = dat; red3[1] = l1; red3[2] = tv; }
}

template <typename real>
__global__ void k_obj_write(const real *__restrict__ red3, int direct, int has_l1,
                            Ctrl<real> *ctrl, real *__restrict__ Obj) {
    if (threadIdx.x != 0) return;
    if (ctrl && ctrl->obj_it >= ctrl->it) return;
    real o = direct ? real(0.5) * red3[0] : red3[0];
    o += red3[2];
    if (has_l1) o += red3[1];
    const int it = ctrl ? ctrl->it : 0;
    Obj[it] = o;
    if (ctrl) ctrl->obj_it = it;
}

}  // namespace pfdr
