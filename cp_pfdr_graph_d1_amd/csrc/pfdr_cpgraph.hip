// Cut-pursuit graph steps on the GPU: the
// full-graph work the reference's CP driver does around every reduced PFDR
// solve, src/CP_PFDR_graph_quadratic_d1_l1.cpp:
//
//   gradient      DfS = smooth gradient at the piecewise-constant iterate +
//                 the d1 and l1 directional terms                 :339-413
//   capacities    source/sink capacities of the single (differentiable) or
//                 the first / second cut, edge capacities         :402-535
//   activate      activate the inactive edges a maxflow cut separates
//                                                         :430-440, :519-556
//   components    connected components of the graph minus its active edges,
//                 in the reference's queue order (Cv, Vc, rVc)     :566-597
//   reduced graph reduced edges (discovery order), summed TV weights, eps
//                 self-loops of isolated components, summed l1 weights
//                                                                  :599-661
//   merge         deactivate edges between (relatively) equal components
//                                                                  :863-886
//
// The maxflow itself (Boykov-Kolmogorov, sequential) stays with the caller
// on the host: capacities go out, segments come back.
//
// Graph state lives in HBM for the whole CP run: endpoints, TV / l1
// weights, the incidence CSR (arc ids 2e + side ascending per vertex, i.e.
// the maxflow graph's adjacency lists REVERSED: include/graph.hpp:405-408
// prepends), edge activity bytes, components.  Every result is identical
// to the reference's (integer work exactly, and every floating sum in the
// reference's order):
//   * components: union-find gives each component's smallest vertex (the
//     reference's root, its outer loop runs u = 0..V-1); then a
//     level-synchronous BFS from all roots at once reproduces the
//     reference's queue exactly: a vertex is claimed by the smallest
//     (queue position of the parent, rank of the arc in the parent's list)
//     with a 64-bit atomicMin, and the winners of each level are emitted in
//     that order (count, scan, emit); a stable sort of the concatenated
//     levels by component gives Vc.
//   * reduced graph: candidate arcs are emitted in the reference's visiting
//     order (Vc position, arc rank), stably sorted by (ru, rv), summed
//     sequentially per group, and the groups ordered by (ru, first visit).
#include <climits>
#include <cstring>
#include <memory>
#include <vector>
#include <rocprim/rocprim.hpp>
#include <stdexcept>

#include "pfdr_graph.hpp"
#include "pfdr_monosum.hpp"

namespace pfdr {

// ------------------------------------------------------------- helpers --
__device__ __forceinline__ int arc_head(unsigned a, const int *__restrict__ Eu,
                                        const int *__restrict__ Ev) {
    return (a & 1u) ? Eu[a >> 1] : Ev[a >> 1];
}

// grow-only temporary storage for rocPRIM calls
struct Tmp {
    DevBuf<char> b;
    void *get(size_t n) {
        if (n > b.n) b.alloc(n + (n >> 2) + 256);
        return b.p;
    }
};

template <typename T>
static void excl_scan(Tmp &t, const T *in, T *out, long n, hipStream_t s) {
    size_t bytes = 0;
    PFDR_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, T(0), (size_t)n, rocprim::plus<T>(),
                                     s));
    void *p = t.get(bytes);
    PFDR_HIP(rocprim::exclusive_scan(p, bytes, in, out, T(0), (size_t)n, rocprim::plus<T>(), s));
}

template <typename K, typename V>
static void sort_pairs(Tmp &t, K *kin, K *kout, V *vin, V *vout, long n, int bits,
                       hipStream_t s) {
    size_t bytes = 0;
    PFDR_HIP(rocprim::radix_sort_pairs(nullptr, bytes, kin, kout, vin, vout, (size_t)n, 0, bits, s));
    void *p = t.get(bytes);
    PFDR_HIP(rocprim::radix_sort_pairs(p, bytes, kin, kout, vin, vout, (size_t)n, 0, bits, s));
}

static int bits_for(long n) {  // smallest b with 2^b >= n (at least 1)
    int b = 1;
    while (b < 62 && (1L << b) < n) b++;
    return b;
}

template <typename T>
static T d2h_scalar(const T *p, hipStream_t s) {
    T h;
    PFDR_HIP(hipMemcpyAsync(&h, p, sizeof(T), hipMemcpyDeviceToHost, s));
    PFDR_HIP(hipStreamSynchronize(s));
    return h;
}

// grid of the counting edge kernels (activation, merge): a grid-stride loop
// and one atomic per block -- one block per 256 edges put 234K atomics on
// one word at the headline size (2.3 ms of serialised adds)
inline int count_grid(long n) { return std::min(grid_for(n), 2048); }

// per-block partial count -> one atomicAdd (integer: order-free)
__device__ __forceinline__ void block_count(int c, int *total) {
    __shared__ int red[kBlock / kWave];
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int i = 0; i < kBlock / kWave; i++) t += red[i];
        if (t) atomicAdd(total, t);
    }
}

// ------------------------------------------------ ordered segment sums --
// out[g] = (((0 + x[o0]) + x[o0+1]) + ...) over [off[g], off[g+1]), with
// x[i] = val[idx[i]] (idx may be null: x[i] = val[i]).  Short segments:
// one lane each; long ones (> kWave entries) are appended to a list and
// summed by one workgroup each (k_segsum_long).
constexpr int kSegShort = kWave;

template <typename real>
__global__ void k_segsum_short(int G, const int *__restrict__ off, const int *__restrict__ idx,
                               const real *__restrict__ val, real *__restrict__ out,
                               int *__restrict__ longs, int *__restrict__ nlong, long vstride) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    const int a = off[g], b = off[g + 1];
    if (b - a > kSegShort) {
        if (blockIdx.y == 0) longs[atomicAdd(nlong, 1)] = g;
        return;
    }
    // grid.y = several value arrays val + y * vstride (the same segments),
    // results at out + y * G
    const real *vv = val + (long)blockIdx.y * vstride;
    real s = real(0);
    for (int i = a; i < b; i++) s += vv[idx ? idx[i] : i];
    out[(long)blockIdx.y * G + g] = s;
}

// one workgroup per long segment: waves 1-3 stage the next chunk in LDS
// (double buffered, coalesced / gathered loads) while lane 0 of wave 0 adds
// the current one in order, 16-byte LDS reads issued ahead of its chain
template <typename real, bool GATHER>
__global__ __launch_bounds__(kBlock) void k_segsum_long(int n, const int *__restrict__ longs,
                                                       const int *__restrict__ off,
                                                       const int *__restrict__ idx,
                                                       const real *__restrict__ val_,
                                                       real *__restrict__ out_, int G,
                                                       long vstride) {
    constexpr int CH = 4096;
    __shared__ alignas(16) real buf[2][CH];
    if ((int)blockIdx.x >= n) return;
    const real *__restrict__ val = val_ + (long)blockIdx.y * vstride;
    real *__restrict__ out = out_ + (long)blockIdx.y * G;
    const int g = longs[blockIdx.x];
    const long a = off[g], b = off[g + 1];
    const int t = threadIdx.x;
    // loaders (waves 1-3): 16 independent loads in flight per lane
    // (indices clamped into the chunk, so every load is unconditional)
    auto load = [&](int which, long c0) {
        constexpr int B = 16, NL = kBlock - kWave;
        const int m = (int)min((long)CH, b - c0);
        for (int j0 = t - kWave; j0 < m; j0 += B * NL) {
            int id[B];
            real x[B];
#pragma unroll
            for (int u = 0; u < B; u++) {
                const long j = c0 + min(j0 + u * NL, m - 1);
                id[u] = GATHER ? idx[j] : (int)j;
            }
#pragma unroll
            for (int u = 0; u < B; u++) x[u] = val[id[u]];
#pragma unroll
            for (int u = 0; u < B; u++)
                if (j0 + u * NL < m) buf[which][j0 + u * NL] = x[u];
        }
    };
    real s = real(0);
    int cur = 0;
    if (t >= kWave) load(0, a);
    __syncthreads();
    for (long c0 = a; c0 < b; c0 += CH) {
        const int m = (int)min((long)CH, b - c0);
        if (t == 0) {
            s = ordered_add(s, buf[cur], m);
        } else if (t >= kWave && c0 + CH < b) {
            load(cur ^ 1, c0 + CH);
        }
        __syncthreads();
        cur ^= 1;
    }
    if (t == 0) out[g] = s;
}

// [off[g], off[g + 1]) of the listed long segments, for the host
__global__ void k_seg_bounds(int n, const int *__restrict__ longs, const int *__restrict__ off,
                             int *__restrict__ b) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    b[2 * i] = off[longs[i]];
    b[2 * i + 1] = off[longs[i] + 1];
}

// *bad = 1 when a term x[i] = val[idx ? idx[i] : i], i < n, is negative, NaN
// or infinite (outside mono_sum's domain); with tmp, the terms are also
// gathered there in order
template <typename real>
__global__ void k_seg_terms(long n, const int *__restrict__ idx, const real *__restrict__ val,
                            real *__restrict__ tmp, int *__restrict__ bad) {
    int b = 0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long)gridDim.x * blockDim.x) {
        const real x = idx ? val[idx[i]] : val[i];
        if (tmp) tmp[i] = x;
        if (!(x >= real(0) && isfinite(x))) b = 1;
    }
    if (bad && __syncthreads_or(b) && threadIdx.x == 0) atomicOr(bad, 1);
}

// Segments of at least kSegMono nonnegative finite terms are summed by the
// binade scan of pfdr_monosum.hpp (mono_sum: the rounding of the sequential
// loop, bit for bit, in parallel) instead of one lane's dependent adds
// (~4.5 ns per term: 36 ms for a giant component's 8M l1 weights).
constexpr long kSegMono = 32768;

// nv value arrays val + j * vstride (j < nv) over the same segments: out[j * G + g]
template <typename real>
static void segsum(int G, const int *off, const int *idx, const real *val, real *out,
                   DevBuf<int> &longs, DevBuf<int> &nlong, hipStream_t s, int nv = 1,
                   long vstride = 0) {
    if (G <= 0 || nv <= 0) return;
    if (nv > 65535) throw std::runtime_error("segsum: too many value arrays");
    if (longs.n < (size_t)G) longs.alloc(G);
    if (!nlong.p) nlong.alloc(1);
    PFDR_HIP(hipMemsetAsync(nlong.p, 0, sizeof(int), s));
    k_segsum_short<real><<<dim3(grid_for(G), nv), kBlock, 0, s>>>(G, off, idx, val, out, longs.p,
                                                                  nlong.p, vstride);
    int nl = d2h_scalar(nlong.p, s);
    if (nl) {
        std::vector<int> hl(nl), hb(2 * (size_t)nl);
        DevBuf<int> db(2 * (size_t)nl);
        k_seg_bounds<<<grid_for(nl), kBlock, 0, s>>>(nl, longs.p, off, db.p);
        PFDR_HIP(hipGetLastError());
        PFDR_HIP(hipMemcpyAsync(hl.data(), longs.p, sizeof(int) * nl, hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipMemcpyAsync(hb.data(), db.p, sizeof(int) * 2 * nl, hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
        std::vector<int> cand;
        long maxlen = 0;
        for (int i = 0; i < nl; i++)
            if ((long)hb[2 * i + 1] - hb[2 * i] >= kSegMono) {
                cand.push_back(i);
                maxlen = std::max(maxlen, (long)hb[2 * i + 1] - hb[2 * i]);
            }
        if (!cand.empty()) {
            const size_t nc = cand.size();
            DevBuf<int> bad(nc * nv);
            PFDR_HIP(hipMemsetAsync(bad.p, 0, sizeof(int) * nc * nv, s));
            for (size_t c = 0; c < nc; c++) {
                const long a = hb[2 * cand[c]], n = hb[2 * cand[c] + 1] - a;
                for (int y = 0; y < nv; y++)
                    k_seg_terms<real><<<(int)std::min<long>(grid_for(n), 1024), kBlock, 0, s>>>(
                        n, idx ? idx + a : nullptr, val + y * vstride + (idx ? 0 : a), nullptr,
                        bad.p + c * nv + y);
            }
            PFDR_HIP(hipGetLastError());
            std::vector<int> hbad(nc * nv);
            PFDR_HIP(hipMemcpyAsync(hbad.data(), bad.p, sizeof(int) * nc * nv,
                                    hipMemcpyDeviceToHost, s));
            PFDR_HIP(hipStreamSynchronize(s));
            DevBuf<real> tmp(idx ? (size_t)maxlen : 1);
            DevBuf<char> ws(mono_ws_bytes<real>(maxlen));
            std::vector<char> done(nl, 0);
            for (size_t c = 0; c < nc; c++) {
                bool ok = true;
                for (int y = 0; y < nv; y++) ok = ok && !hbad[c * nv + y];
                if (!ok) continue;  // a negative / non-finite term: one workgroup below
                const int i = cand[c], g = hl[i];
                const long a = hb[2 * i], n = hb[2 * i + 1] - a;
                for (int y = 0; y < nv; y++) {
                    const real *terms = val + y * vstride + a;
                    if (idx) {  // gathered in order into tmp (stream-ordered reuse)
                        k_seg_terms<real><<<(int)std::min<long>(grid_for(n), 1024), kBlock, 0, s>>>(
                            n, idx + a, val + y * vstride, tmp.p, nullptr);
                        terms = tmp.p;
                    }
                    mono_sum<real>(n, terms, nullptr, 0, nullptr, out + (long)y * G + g, nullptr,
                                   ws.p, s);
                }
                done[i] = 1;
            }
            PFDR_HIP(hipGetLastError());
            // the remaining long segments, one workgroup each
            std::vector<int> rest;
            for (int i = 0; i < nl; i++)
                if (!done[i]) rest.push_back(hl[i]);
            nl = (int)rest.size();
            if (nl)
                PFDR_HIP(hipMemcpyAsync(longs.p, rest.data(), sizeof(int) * nl,
                                        hipMemcpyHostToDevice, s));
            PFDR_HIP(hipStreamSynchronize(s));  // rest, tmp and ws leave scope
        }
    }
    if (nl && idx)
        k_segsum_long<real, true><<<dim3(nl, nv), kBlock, 0, s>>>(nl, longs.p, off, idx, val, out,
                                                                   G, vstride);
    else if (nl)
        k_segsum_long<real, false><<<dim3(nl, nv), kBlock, 0, s>>>(nl, longs.p, off, idx, val, out,
                                                                    G, vstride);
    PFDR_HIP(hipGetLastError());
}

template <typename real>
void ordered_segment_sums(int G, const int *off, const int *idx, const real *val, real *out,
                          hipStream_t s) {
    DevBuf<int> longs, nlong;
    segsum<real>(G, off, idx, val, out, longs, nlong, s);
    PFDR_HIP(hipStreamSynchronize(s));  // scratch freed at scope exit
}
template void ordered_segment_sums<float>(int, const int *, const int *, const float *, float *,
                                          hipStream_t);
template void ordered_segment_sums<double>(int, const int *, const int *, const double *,
                                           double *, hipStream_t);

// ----------------------------------------------------------- components --
__device__ __forceinline__ int uf_root(const int *parent, int v) {
    for (;;) {
        const int p = __hip_atomic_load(parent + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p == v) return v;
        v = p;
    }
}

__global__ void k_uf_init(int V, int *parent) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < V) parent[v] = v;
}

// union over the inactive edges: hook the larger root under the smaller one
// by CAS on the root (a lost race retries from the new roots), so every
// tree's root is its component's smallest vertex
__global__ void k_uf_hook(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                          const uint8_t *__restrict__ active, int *parent) {
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < E;
         e += (long)gridDim.x * blockDim.x) {
        if (active[e]) continue;
        int a = Eu[e], b = Ev[e];
        for (;;) {
            a = uf_root(parent, a);
            b = uf_root(parent, b);
            if (a == b) break;
            const int hi = max(a, b), lo = min(a, b);
            if (atomicCAS(parent + hi, hi, lo) == hi) break;
        }
    }
}

__global__ void k_uf_flatten(int V, int *parent, int *is_root) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const int r = uf_root(parent, v);
    parent[v] = r;
    is_root[v] = (r == v) ? 1 : 0;
}

// level 0: the roots in increasing order (= component order); Cv of every
// other vertex -1 (unvisited), claims cleared
__global__ void k_bfs_roots(int V, const int *__restrict__ is_root, const int *__restrict__ rid,
                            int *__restrict__ L, int *__restrict__ Cv,
                            unsigned long long *__restrict__ claim) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    claim[v] = ~0ull;
    if (is_root[v]) {
        L[rid[v]] = v;
        Cv[v] = rid[v];
    } else {
        Cv[v] = -1;
    }
}

__device__ __forceinline__ unsigned long long claim_key(int i, int j) {
    return ((unsigned long long)(unsigned)i << 32) | (unsigned)j;
}

// A frontier vertex's arcs are handled by a subgroup of kSub lanes (arc j
// by lane j mod kSub), so the dependent gathers of an arc (slot, activity,
// endpoint, component) run for up to kSub arcs at once instead of one
// after the other.
constexpr int kSub = 16;

// ---- breadth-first levels driven from the device.  Frontier L[lo, hi):
// every unvisited neighbour through an inactive edge is claimed by its first
// visit in the reference's order (queue position i, then the arc's rank j in
// the maxflow graph's list: slots descending); the winners are counted,
// scanned and appended in arc order.  The frontier bounds live in a control
// block (lo, hi, done, overflow), every kernel of a level reads them, fixed
// grids loop over the frontier, and a one-lane kernel advances the bounds;
// the host enqueues levels in batches (one hipGraph replay each) and reads
// the control block once per batch instead of once per level (a host round
// trip per level cost ~40 us of a ~60 us level).
struct BfsCtl {
    int lo, hi, done, overflow;
};

__device__ __forceinline__ void bfs_chunk(int n, int nblk, int b, int &c0, int &c1) {
    // frontier positions [c0, c1) of block b: whole steps of kBlock / kSub vertices
    constexpr int step = kBlock / kSub;
    const int per = ((n + nblk - 1) / nblk + step - 1) / step * step;
    c0 = min(n, b * per);
    c1 = min(n, c0 + per);
}

__global__ void k_bfsd_claim(const BfsCtl *__restrict__ ctl, const int *__restrict__ L,
                             const int *__restrict__ ptr, const unsigned *__restrict__ slot,
                             const int *__restrict__ Eu, const int *__restrict__ Ev,
                             const uint8_t *__restrict__ active, const int *__restrict__ Cv,
                             unsigned long long *claim) {
    const BfsCtl c = *ctl;
    if (c.done) return;
    const long nt = (long)(c.hi - c.lo) * kSub;
    for (long gt = (long)blockIdx.x * blockDim.x + threadIdx.x; gt < nt;
         gt += (long)gridDim.x * blockDim.x) {
        const int i = c.lo + (int)(gt / kSub), l = (int)(gt % kSub);
        const int v = L[i];
        const int top = ptr[v + 1] - 1, deg = top + 1 - ptr[v];
        for (int j = l; j < deg; j += kSub) {
            const unsigned a = slot[top - j];
            if (active[a >> 1]) continue;
            const int w = arc_head(a, Eu, Ev);
            if (Cv[w] != -1) continue;
            atomicMin(claim + w, claim_key(i, j));
        }
    }
}

// claims won by frontier vertex i (the whole subgroup returns the count;
// EMIT: appended in arc order at base, Cv set)
template <bool EMIT>
__device__ __forceinline__ int bfs_take_one(int i, int l, int sh, const int *__restrict__ L,
                                            const int *__restrict__ ptr,
                                            const unsigned *__restrict__ slot,
                                            const int *__restrict__ Eu, const int *__restrict__ Ev,
                                            const uint8_t *__restrict__ active,
                                            const unsigned long long *__restrict__ claim,
                                            bool valid, int base, int *Lo, int *Cv) {
    int v = 0, deg = 0, top = 0, cv = 0;
    if (valid) {
        v = L[i];
        top = ptr[v + 1] - 1;
        deg = top + 1 - ptr[v];
        if (EMIT) cv = Cv[v];
    }
    int c = 0;
    // every lane of the wave runs the same number of ballots
    int dmax = deg;
    for (int o = 1; o < kWave; o <<= 1) dmax = max(dmax, __shfl_xor(dmax, o, kWave));
    for (int j0 = 0; j0 < dmax; j0 += kSub) {
        const int j = j0 + l;
        bool win = false;
        int w = 0;
        if (j < deg) {
            const unsigned a = slot[top - j];
            if (!active[a >> 1]) {
                w = arc_head(a, Eu, Ev);
                win = claim[w] == claim_key(i, j);
            }
        }
        const unsigned long long m = __ballot(win);
        const unsigned mine = (unsigned)(m >> sh) & ((1u << kSub) - 1);
        if (EMIT && win) {
            Lo[base + c + __builtin_popcount(mine & ((1u << l) - 1))] = w;
            Cv[w] = cv;
        }
        c += __builtin_popcount(mine);
    }
    return c;
}

// counts of the block's chunk into cnt[i - lo], the chunk's total into bsum[b]
__global__ __launch_bounds__(kBlock) void k_bfsd_count(
    const BfsCtl *__restrict__ ctl, const int *__restrict__ L, const int *__restrict__ ptr,
    const unsigned *__restrict__ slot, const int *__restrict__ Eu, const int *__restrict__ Ev,
    const uint8_t *__restrict__ active, const unsigned long long *__restrict__ claim,
    int *__restrict__ cnt, int *__restrict__ bsum) {
    __shared__ int red[kBlock / kWave];
    const BfsCtl c = *ctl;
    if (c.done) return;
    int c0, c1;
    bfs_chunk(c.hi - c.lo, gridDim.x, blockIdx.x, c0, c1);
    const int t = threadIdx.x, l = t % kSub, sh = (t & (kWave - 1)) & ~(kSub - 1);
    if (c0 >= c1) {  // past the frontier (block-uniform)
        if (t == 0) bsum[blockIdx.x] = 0;
        return;
    }
    int tot = 0;
    for (int q = c0; q < c1; q += kBlock / kSub) {
        const int fi = q + t / kSub;
        const bool valid = fi < c1;
        const int k = bfs_take_one<false>(c.lo + fi, l, sh, L, ptr, slot, Eu, Ev, active, claim,
                                          valid, 0, nullptr, nullptr);
        if (valid && l == 0) {
            cnt[fi] = k;
            tot += k;
        }
    }
    tot = block_sum(tot, red);
    if (t == 0) bsum[blockIdx.x] = tot;
}

// emission: the block's base is the sum of the earlier blocks' totals, each
// step's 16 vertices are offset by an exclusive scan of their counts
__global__ __launch_bounds__(kBlock) void k_bfsd_emit(
    const BfsCtl *__restrict__ ctl, const int *__restrict__ ptr, const unsigned *__restrict__ slot,
    const int *__restrict__ Eu, const int *__restrict__ Ev, const uint8_t *__restrict__ active,
    const unsigned long long *__restrict__ claim, const int *__restrict__ cnt,
    const int *__restrict__ bsum, int *L, int *Cv) {
    constexpr int step = kBlock / kSub;
    __shared__ int red[kBlock / kWave];
    __shared__ int off[step + 1];
    __shared__ int s_pre;
    const BfsCtl c = *ctl;
    if (c.done) return;
    const int t = threadIdx.x, l = t % kSub, sh = (t & (kWave - 1)) & ~(kSub - 1);
    int c0, c1;
    bfs_chunk(c.hi - c.lo, gridDim.x, blockIdx.x, c0, c1);
    if (c0 >= c1) return;  // past the frontier (block-uniform)
    int pre = 0;
    for (int b = t; b < (int)blockIdx.x; b += kBlock) pre += bsum[b];
    pre = block_sum(pre, red);  // valid in thread 0
    if (t == 0) s_pre = pre;
    __syncthreads();
    int base = c.hi + s_pre;
    for (int q = c0; q < c1; q += step) {
        __syncthreads();
        if (t == 0) {
            int a = 0;
            for (int k = 0; k < step; k++) {
                off[k] = a;
                if (q + k < c1) a += cnt[q + k];
            }
            off[step] = a;
        }
        __syncthreads();
        const int fi = q + t / kSub;
        const bool valid = fi < c1;
        (void)bfs_take_one<true>(c.lo + fi, l, sh, L, ptr, slot, Eu, Ev, active, claim, valid,
                                 base + off[t / kSub], L, Cv);
        base += off[step];
    }
}

// lo <- hi, hi += this level's total; done when it is 0 or every vertex is queued
__global__ void k_bfsd_advance(BfsCtl *ctl, const int *__restrict__ bsum, int nblk, int V) {
    __shared__ int red[kBlock / kWave];
    const BfsCtl c = *ctl;
    if (c.done) return;
    int tot = 0;
    for (int b = threadIdx.x; b < nblk; b += kBlock) tot += bsum[b];
    tot = block_sum(tot, red);
    if (threadIdx.x == 0) {
        BfsCtl n = c;
        if (tot > V - c.hi) {
            n.overflow = 1;
            n.done = 1;
        } else {
            n.lo = c.hi;
            n.hi = c.hi + tot;
            n.done = (tot == 0 || n.hi >= V) ? 1 : 0;
        }
        *ctl = n;
    }
}

__global__ void k_gather_keys(int V, const int *__restrict__ L, const int *__restrict__ Cv,
                              unsigned *__restrict__ key) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < V) key[i] = (unsigned)Cv[L[i]];
}

// rVc[c] = first position of component c in the sorted keys, rVc[rV] = V
__global__ void k_comp_ptr(int V, int rV, const unsigned *__restrict__ skey, int *__restrict__ rVc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > V) return;
    if (i == V) { rVc[rV] = V; return; }
    if (i == 0 || skey[i] != skey[i - 1]) rVc[skey[i]] = i;
}

// -------------------------------------------------------- reduced graph --
// per Vc position s: candidate arcs of u = Vc[s] (active, nonzero weight,
// neighbour component rv >= ru) in the reference's visiting order; any
// active nonzero arc makes the component non-isolated (:626-633)
template <typename real, bool EMIT>
__global__ void k_rg_scan(int V, int rbits, const int *__restrict__ Vc, const int *__restrict__ Cv,
                          const int *__restrict__ ptr, const unsigned *__restrict__ slot,
                          const int *__restrict__ Eu, const int *__restrict__ Ev,
                          const uint8_t *__restrict__ active, const real *__restrict__ La,
                          int *__restrict__ cnt, uint8_t *__restrict__ nonIso,
                          unsigned long long *__restrict__ key, unsigned *__restrict__ pos,
                          int *__restrict__ cand_e) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= V) return;
    const int u = Vc[s], ru = Cv[u];
    const int b = ptr[u];
    int c = 0, base = EMIT ? cnt[s] : 0;
    bool any = false;
    for (int k = ptr[u + 1] - 1; k >= b; k--) {
        const unsigned a = slot[k];
        const int e = (int)(a >> 1);
        if (!active[e]) continue;
        if (La[e] == real(0)) continue;
        any = true;
        const int rv = Cv[arc_head(a, Eu, Ev)];
        if (rv < ru) continue;
        if (EMIT) {
            const int p = base + c;
            key[p] = ((unsigned long long)ru << rbits) | (unsigned long long)rv;
            pos[p] = (unsigned)p;
            cand_e[p] = e;
        }
        c++;
    }
    if (!EMIT) {
        cnt[s] = c;
        if (any) nonIso[ru] = 1;
    }
}

// group heads of the sorted (ru, rv) keys
__global__ void k_rg_heads(long M, const unsigned long long *__restrict__ skey,
                           int *__restrict__ head) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) head[i] = (i == 0 || skey[i] != skey[i - 1]) ? 1 : 0;
}

// per group: start offset, (ru, rv); per entry: its weight in sorted order
template <typename real>
__global__ void k_rg_groups(long M, int rbits, const unsigned long long *__restrict__ skey,
                            const unsigned *__restrict__ spos, const int *__restrict__ cand_e,
                            const real *__restrict__ La, const int *__restrict__ head,
                            const int *__restrict__ gid, int *__restrict__ goff,
                            int *__restrict__ gru, int *__restrict__ grv,
                            unsigned *__restrict__ gfirst, real *__restrict__ wsorted) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const unsigned p = spos[i];
    wsorted[i] = La[cand_e[p]];
    if (head[i]) {
        const int g = gid[i];
        const unsigned long long k = skey[i];
        goff[g] = (int)i;
        gru[g] = (int)(k >> rbits);
        grv[g] = (int)(k & ((1ull << rbits) - 1));
        gfirst[g] = p;  // stable sort: the group's first visit
    }
}

// final order keys: groups by (ru, first visit); isolated components'
// eps self-loop at (ru, 0) (they own no group)
__global__ void k_rg_order_keys(int G, int rV, const int *__restrict__ gru,
                                const unsigned *__restrict__ gfirst,
                                const uint8_t *__restrict__ nonIso, const int *__restrict__ isoid,
                                unsigned long long *__restrict__ key, int *__restrict__ val) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < G) {
        key[i] = ((unsigned long long)gru[i] << 32) | gfirst[i];
        val[i] = i;
    } else if (i < G + rV) {
        const int ru = i - G;
        if (!nonIso[ru]) {
            const int t = G + isoid[ru];
            key[t] = (unsigned long long)ru << 32;
            val[t] = -1 - ru;
        }
    }
}

// outputs; an isolated component's self-loop goes to the next non-isolated
// component when there is one (the reference's rEc reset, :645-656)
template <typename real>
__global__ void k_rg_write(int rE, int nNI, const int *__restrict__ sval,
                           const int *__restrict__ gru, const int *__restrict__ grv,
                           const real *__restrict__ gw, const int *__restrict__ NI, real eps,
                           int *__restrict__ rEu, int *__restrict__ rEv, real *__restrict__ rLa) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= rE) return;
    const int g = sval[t];
    if (g >= 0) {
        rEu[t] = gru[g];
        rEv[t] = grv[g];
        rLa[t] = gw[g];
        return;
    }
    const int ru = -1 - g;
    int lo = 0, hi = nNI;  // first non-isolated component > ru
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (NI[m] > ru) hi = m; else lo = m + 1;
    }
    rEu[t] = (lo < nNI) ? NI[lo] : ru;
    rEv[t] = ru;
    rLa[t] = eps;
}

__global__ void k_flag_to_int(int n, const uint8_t *__restrict__ f, int neg, int *__restrict__ o) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = neg ? (f[i] ? 0 : 1) : (f[i] ? 1 : 0);
}

__global__ void k_compact_ids(int n, const uint8_t *__restrict__ f, const int *__restrict__ pos,
                              int *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && f[i]) out[pos[i]] = i;
}

// -------------------------------------------------------------- merge --
template <typename real>
__global__ void k_cp_merge(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                           const int *__restrict__ Cv, const real *__restrict__ rX, real eps,
                           real difTol, uint8_t *__restrict__ active, int *__restrict__ count) {
    int c = 0;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < E;
         e += (long)gridDim.x * blockDim.x) {
        if (!active[e]) continue;
        real a = rX[Cv[Eu[e]]], b = rX[Cv[Ev[e]]], d = a - b;
        if (a < real(0)) a = -a;
        if (b < real(0)) b = -b;
        if (d < real(0)) d = -d;
        if (a < b) a = b;
        d = (a > eps) ? d / a : d / eps;
        if (d <= difTol) {
            active[e] = 0;
            c++;
        }
    }
    block_count(c, count);
}

// ------------------------------------------------------------ gradient --
// DfS base of the N = 0 modes (:369-376), then the d1 term over the active
// arcs in the maxflow graph's order and the l1 term (:379-413); N != 0:
// the base is already in DfS
template <typename real>
__global__ void k_cp_grad(int V, int base_mode, const real *__restrict__ A,
                          const real *__restrict__ Y, const int *__restrict__ ptr,
                          const unsigned *__restrict__ slot, const int *__restrict__ Eu,
                          const int *__restrict__ Ev, const uint8_t *__restrict__ active,
                          const real *__restrict__ La, const real *__restrict__ L1,
                          const int *__restrict__ Cv, const real *__restrict__ rX,
                          real *__restrict__ DfS) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= V) return;
    const real xu = rX[Cv[u]];
    real g;
    if (base_mode == 1) g = A[u] * xu - Y[u];
    else if (base_mode == 0) g = xu - Y[u];
    else g = DfS[u];
    const int b = ptr[u];
    for (int k = ptr[u + 1] - 1; k >= b; k--) {
        const unsigned a = slot[k];
        const int e = (int)(a >> 1);
        if (!active[e]) continue;
        const real d = xu - rX[Cv[arc_head(a, Eu, Ev)]];
        if (d > real(0)) g += La[e];
        else if (d < real(0)) g -= La[e];
    }
    if (L1) {
        if (xu > real(0)) g += L1[u];
        else if (xu < real(0)) g -= L1[u];
    }
    DfS[u] = g;
}

// N > 0: DfS[v] = -(sum_n A[n, v] R[n]) in n order (:342-352).  One wave
// per 64 columns: 64 x 64 tiles staged through LDS (coalesced column
// reads), then each lane adds its column's entries in order.
template <typename real>
__global__ __launch_bounds__(kWave) void k_cp_grad_direct(int N, int V, const real *__restrict__ A,
                                                         const real *__restrict__ R,
                                                         real *__restrict__ DfS) {
    __shared__ real t[kWave][kWave + 1];
    const int lane = threadIdx.x;
    const int v0 = blockIdx.x * kWave;
    real s = real(0);
    for (int n0 = 0; n0 < N; n0 += kWave) {
        const int n = n0 + lane;
        const real r = (n < N) ? R[n] : real(0);
        for (int c = 0; c < kWave; c++) {
            const int v = v0 + c;
            t[c][lane] = (v < V && n < N) ? A[(size_t)N * v + n] * r : real(0);
        }
        __syncthreads();
        const int m = min(kWave, N - n0);
        for (int k = 0; k < m; k++) s += t[lane][k];
        __syncthreads();
    }
    if (v0 + lane < V) DfS[v0 + lane] = -s;
}

// N < 0: DfS[u] = sum over components with rX != 0 of (component sum of
// column u of A^tA, in Vc order) * rX, minus Y[u] (:353-368); one lane per u
template <typename real>
__global__ void k_cp_grad_ata(int V, int rV, const real *__restrict__ A, const real *__restrict__ Y,
                              const int *__restrict__ Vc, const int *__restrict__ rVc,
                              const real *__restrict__ rX, real *__restrict__ DfS) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= V) return;
    const real *Av = A + (size_t)V * u;
    real b = real(0);
    for (int rv = 0; rv < rV; rv++) {
        const real x = rX[rv];
        if (x == real(0)) continue;
        real a = real(0);
        for (int s = rVc[rv], t = rVc[rv + 1]; s < t; s++) a += Av[Vc[s]];
        b += a * x;
    }
    DfS[u] = b - Y[u];
}

// ---------------------------------------------------------- capacities --
template <typename real>
__global__ void k_cp_trcap(int V, int cut, int positivity, const real *__restrict__ L1,
                           const int *__restrict__ Cv, const real *__restrict__ rX,
                           const real *__restrict__ DfS, real *__restrict__ tr) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const bool zero = rX[Cv[v]] == real(0);
    real t = DfS[v];
    if (cut == 1 && L1 && zero) t = DfS[v] + L1[v];
    else if (cut == 2 && zero) t = positivity ? -Lim<real>::huge : DfS[v] - L1[v];
    tr[v] = t;
}

// the bounds driver's cuts (src/CP_PFDR_graph_quadratic_d1_bounds.cpp:386-534):
// cut 1 +inf on components at max (max < inf), else DfS; cut 2 +inf on
// components at min (-inf < min), else -DfS; cut 0 DfS
template <typename real>
__global__ void k_cp_trcap_bounds(int V, int cut, real mn, real mx, const int *__restrict__ Cv,
                                  const real *__restrict__ rX, const real *__restrict__ DfS,
                                  real *__restrict__ tr) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const real inf = Lim<real>::huge, x = rX[Cv[v]];
    real t = DfS[v];
    if (cut == 1) t = (mx < inf && x == mx) ? inf : DfS[v];
    else if (cut == 2) t = (-inf < mn && x == mn) ? inf : -DfS[v];
    tr[v] = t;
}

template <typename real>
__global__ void k_cp_rcap(long E, const uint8_t *__restrict__ active, const real *__restrict__ La,
                          real *__restrict__ rc) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < E) rc[e] = active[e] ? real(0) : La[e];
}

__global__ void k_cp_activate(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                              const uint8_t *__restrict__ seg, uint8_t *__restrict__ active,
                              int *__restrict__ count) {
    int c = 0;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < E;
         e += (long)gridDim.x * blockDim.x)
        if (seg[Eu[e]] != seg[Ev[e]] && !active[e]) {
            active[e] = 1;
            c++;
        }
    block_count(c, count);
}


// ------------------------------------------------- the simplex driver --
// src/CP_PFDR_graph_loss_d1_simplex.cpp: K labels, Q[v*K + k] and the
// component label vectors rP[rv*K + k] (the reference's layouts).

// Q (V x K, vertex-major) -> Qt (K x V): each label's column contiguous,
// for the ordered component sums of the reduced observations
template <typename real>
__global__ void k_sx_transpose(int V, int K, const real *__restrict__ Q, real *__restrict__ Qt) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)V * K) return;
    const long v = i / K, k = i - v * K;
    Qt[k * V + v] = Q[i];
}

// :739-766 from the ordered sums S[k*rV + rv]: linear loss: rQ = sums, rP =
// the corner of the first largest sum; else rQ = rP = sums / size, rLa_f =
// size
template <typename real>
__global__ void k_sx_observations(int rV, int K, int linear, const real *__restrict__ S,
                                  const int *__restrict__ rVc, real *__restrict__ rP,
                                  real *__restrict__ rQ, real *__restrict__ rLa_f) {
    const int rv = blockIdx.x * blockDim.x + threadIdx.x;
    if (rv >= rV) return;
    real *P = rP + (size_t)rv * K, *Qo = rQ + (size_t)rv * K;
    if (linear) {
        int i = 0;
        real a = S[rv];
        for (int k = 1; k < K; k++) {
            const real x = S[(size_t)k * rV + rv];
            if (x > a) { a = x; i = k; }
        }
        for (int k = 0; k < K; k++) {
            Qo[k] = S[(size_t)k * rV + rv];
            P[k] = (k == i) ? real(1) : real(0);
        }
    } else {
        const int n = rVc[rv + 1] - rVc[rv];
        for (int k = 0; k < K; k++) {
            const real q = S[(size_t)k * rV + rv] / (real)n;
            Qo[k] = q;
            P[k] = q;
        }
        if (rLa_f) rLa_f[rv] = (real)n;
    }
}

// :327-376, one lane per (v, k): the loss gradient at the component's label
// vector, then the d1 term over v's active arcs, newest first (the maxflow
// graph's list order); the adds of one (v, k) are independent of the
// other labels
template <typename real>
__global__ void k_sx_gradient(int V, int K, int loss, real alK, real al1, real alKal1,
                              const real *__restrict__ Q, const int *__restrict__ ptr,
                              const unsigned *__restrict__ slot, const int *__restrict__ Eu,
                              const int *__restrict__ Ev, const uint8_t *__restrict__ active,
                              const real *__restrict__ La, const int *__restrict__ Cv,
                              const real *__restrict__ rP, real eps, real *__restrict__ DfS) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)V * K) return;
    const int v = (int)(i / K), k = (int)(i - (long)v * K);
    const real q = Q[i], p = rP[(size_t)Cv[v] * K + k];
    real g;
    if (loss == 0) g = -q;
    else if (loss == 1) g = p - q;
    else g = -(alK + al1 * q) / (alKal1 + p);
    const int b = ptr[v];
    for (int j = ptr[v + 1] - 1; j >= b; j--) {
        const unsigned a = slot[j];
        const int e = (int)(a >> 1);
        if (!active[e]) continue;
        const real d = p - rP[(size_t)Cv[arc_head(a, Eu, Ev)] * K + k];
        if (d > eps) g += La[e];
        else if (d < -eps) g -= La[e];
    }
    DfS[i] = g;
}

// :525-536 the most confident label of each component (first on ties)
template <typename real>
__global__ void k_sx_best(int rV, int K, const real *__restrict__ rP, int *__restrict__ rDi) {
    const int rv = blockIdx.x * blockDim.x + threadIdx.x;
    if (rv >= rV) return;
    const real *P = rP + (size_t)rv * K;
    int i = 0;
    real a = P[0];
    for (int k = 1; k < K; k++)
        if (P[k] > a) { a = P[k]; i = k; }
    rDi[rv] = i;
}

// :542-595 alpha-expansion n: per vertex the source/sink capacity from its
// component's label and its current alternative, then the d1 terms of its
// inactive edges in edge order (incidence slots ascending: the reference's
// sequential edge loop adds c - a at the u end and -c at the v end)
template <typename real>
__global__ void k_sx_trcap(int V, int K, int n, const int *__restrict__ ptr,
                           const unsigned *__restrict__ slot, const int *__restrict__ Eu,
                           const int *__restrict__ Ev, const uint8_t *__restrict__ active,
                           const real *__restrict__ La, const int *__restrict__ Cv,
                           const int *__restrict__ rDi, const int *__restrict__ Djv,
                           const real *__restrict__ DfS, real *__restrict__ tr) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const int i = rDi[Cv[v]], j = n > i ? n : n - 1, k = Djv[v];
    const real *D = DfS + (size_t)v * K;
    real t;
    if (k == 0) t = D[j] - D[i];
    else if (k == n) t = real(0);
    else if (k > i) t = D[j] - D[k];
    else t = D[j] - D[k - 1];
    for (int q = ptr[v], qe = ptr[v + 1]; q < qe; q++) {
        const unsigned a = slot[q];
        const int e = (int)(a >> 1);
        if (active[e]) continue;
        const real w = real(2) * La[e];
        const real aa = (Djv[Eu[e]] == Djv[Ev[e]]) ? real(0) : w;
        if (a & 1u) t -= w;
        else t += w - aa;
    }
    tr[v] = t;
}

// arc 2e's capacity b + c - a (arc 2e + 1 has none, :592-593)
template <typename real>
__global__ void k_sx_rcap(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                          const uint8_t *__restrict__ active, const real *__restrict__ La,
                          const int *__restrict__ Djv, real *__restrict__ rc) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    if (active[e]) { rc[e] = real(0); return; }
    const real w = real(2) * La[e];
    const real a = (Djv[Eu[e]] == Djv[Ev[e]]) ? real(0) : w;
    rc[e] = w + w - a;
}

// :600-604 the sink side takes alternative n
__global__ void k_sx_expand(int V, int n, const uint8_t *__restrict__ seg, int *__restrict__ Djv) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < V && seg[v]) Djv[v] = n;
}

// :608-618 activate the inactive edges whose ends took different alternatives
__global__ void k_sx_activate(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                              const int *__restrict__ Djv, uint8_t *__restrict__ active,
                              int *__restrict__ count) {
    int c = 0;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < E;
         e += (long)gridDim.x * blockDim.x)
        if (!active[e] && Djv[Eu[e]] != Djv[Ev[e]]) {
            active[e] = 1;
            c++;
        }
    block_count(c, count);
}

// :782-803 deactivate the active edges whose components' label vectors
// differ by at most eps in every label
template <typename real>
__global__ void k_sx_merge(long E, int K, const int *__restrict__ Eu, const int *__restrict__ Ev,
                           const int *__restrict__ Cv, const real *__restrict__ rP, real eps,
                           uint8_t *__restrict__ active, int *__restrict__ count) {
    int c = 0;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < E;
         e += (long)gridDim.x * blockDim.x) {
        if (!active[e]) continue;
        const real *Pu = rP + (size_t)Cv[Eu[e]] * K, *Pv = rP + (size_t)Cv[Ev[e]] * K;
        real a = real(0);
        for (int k = 0; k < K; k++) {
            real d = Pu[k] - Pv[k];
            if (d < real(0)) d = -d;
            if (d > a) a = d;
        }
        if (a <= eps) {
            active[e] = 0;
            c++;
        }
    }
    block_count(c, count);
}


// the duplex driver's two-layer cut (src/CP_PFDR_graph_quadratic_d1_l1_duplex.cpp:469-527,
// non-differentiable case): directional derivatives up / down per vertex
// (:473-502; without La_l1 both are DfS -- the reference leaves them unset
// there), m = MAX(0, MAX(-up, down)) with the reference's macro,
// tr_cap[v1] = -down + m, tr_cap[v2] = -(up + m), arc v1 -> v2 of capacity m
template <typename real>
__global__ void k_cp_trcap_duplex(int V, int positivity, const real *__restrict__ L1,
                                  const int *__restrict__ Cv, const real *__restrict__ rX,
                                  const real *__restrict__ DfS, real *__restrict__ tr,
                                  real *__restrict__ link) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const real x = rX[Cv[v]], g = DfS[v];
    real up = g, dn = g;
    if (L1 && x == real(0)) {
        up = g + L1[v];
        dn = g - L1[v];
    }
    if (positivity && x == real(0)) dn = -Lim<real>::huge;
    const real in = ((-up) > (dn)) ? (-up) : (dn);
    const real m = (real(0) > in) ? real(0) : in;
    tr[v] = -dn + m;
    tr[V + v] = -(up + m);
    link[v] = m;
}

// :531-545 activate the inactive edges the cut separates in either layer
__global__ void k_cp_activate_duplex(int V, long E, const int *__restrict__ Eu,
                                     const int *__restrict__ Ev, const uint8_t *__restrict__ seg,
                                     uint8_t *__restrict__ active, int *__restrict__ count) {
    int c = 0;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < E;
         e += (long)gridDim.x * blockDim.x) {
        if (active[e]) continue;
        const int u = Eu[e], v = Ev[e];
        if (seg[u] != seg[v] || seg[V + u] != seg[V + v]) {
            active[e] = 1;
            c++;
        }
    }
    block_count(c, count);
}

// ================================================================ state --
struct CpGraphBase {
    virtual ~CpGraphBase() = default;
    int V = 0;
    long E = 0;
    int dtype = PFDR_F32;
    hipStream_t s = nullptr;
    int dev = 0;  // device of s (calls from any thread run on it)
    DevBuf<int> Eu, Ev;
    Incidence inc;
    DevBuf<uint8_t> active;
    DevBuf<int> Cv, Vc, rVc;
    int rV = 0, rE = 0;
    DevBuf<int> rEu, rEv;
    DevBuf<int> count;
    Tmp tmp;
    double last_ms = 0;
    // scratch
    DevBuf<int> i0, i1, i2, L;
    DevBuf<unsigned long long> claim;
    DevBuf<int> longs, nlong;

    void components();
    void bfs_device();  // the BFS levels of components(), driven from the device
    virtual void reduced_graph(double eps) = 0;
    virtual int merge(double eps, double difTol) = 0;
    virtual void gradient(int N, const void *A, const void *Y, const void *R, int mem) = 0;
    virtual void capacities(int cut, int positivity, void *tr, void *rc, int mem) = 0;
    // bounds driver: box [mn, mx] (+-HUGE_VAL for none) instead of l1 / positivity
    virtual void capacities_bounds(int cut, double mn, double mx, void *tr, void *rc,
                                   int mem) = 0;
    virtual void set_values(const void *rX, int mem) = 0;
    virtual void get_reduced(int *rEu_o, int *rEv_o, void *rLa_o, void *rL1_o, int mem) = 0;
    virtual void get_dfs(void *out, int mem) = 0;
    int activate(const uint8_t *seg, int mem);
    // the simplex driver (K labels)
    int K = 0;
    DevBuf<int> rDi, Djv;
    virtual void sx_setup(int K_, double al, const void *Q, int mem) = 0;
    virtual void sx_observations(void *rP, void *rQ, void *rLa_f, int mem) = 0;
    virtual void sx_set_values(const void *rP, int mem) = 0;
    virtual void sx_gradient(double eps, void *DfS, int *rDi_o, int mem) = 0;
    virtual void sx_capacities(int n, void *tr, void *rc, int mem) = 0;
    virtual int sx_merge(double eps) = 0;
    void sx_expand(int n, const uint8_t *seg, int mem);
    int sx_activate();
    // the duplex driver's two-layer cut
    virtual void capacities_duplex(int positivity, void *tr, void *link, void *rc, int mem) = 0;
    int activate_duplex(const uint8_t *seg, int mem);
};

static hipMemcpyKind kind_in(int mem) {
    return mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
}
static hipMemcpyKind kind_out(int mem) {
    return mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
}

void CpGraphBase::components() {
    const int Vn = V;
    i0.alloc(Vn);  // parent
    i1.alloc(Vn + 1);  // is_root, then scratch
    i2.alloc(Vn + 1);  // root ids
    L.alloc(Vn);
    claim.alloc(Vn);
    Cv.alloc(Vn);
    k_uf_init<<<grid_for(Vn), kBlock, 0, s>>>(Vn, i0.p);
    if (E > 0)
        k_uf_hook<<<std::min(grid_for(E), 8192), kBlock, 0, s>>>(E, Eu.p, Ev.p, active.p, i0.p);
    k_uf_flatten<<<grid_for(Vn), kBlock, 0, s>>>(Vn, i0.p, i1.p);
    PFDR_HIP(hipMemsetAsync(i1.p + Vn, 0, sizeof(int), s));
    excl_scan(tmp, i1.p, i2.p, Vn + 1, s);
    rV = d2h_scalar(i2.p + Vn, s);
    k_bfs_roots<<<grid_for(Vn), kBlock, 0, s>>>(Vn, i1.p, i2.p, L.p, Cv.p, claim.p);
    PFDR_HIP(hipGetLastError());
    bfs_device();
    // Vc = the concatenated levels stably sorted by component
    DevBuf<unsigned> key(Vn), skey(Vn);
    Vc.alloc(Vn);
    rVc.alloc(Vn + 1);
    k_gather_keys<<<grid_for(Vn), kBlock, 0, s>>>(Vn, L.p, Cv.p, key.p);
    sort_pairs(tmp, key.p, skey.p, L.p, Vc.p, Vn, bits_for(rV), s);
    k_comp_ptr<<<grid_for(Vn + 1), kBlock, 0, s>>>(Vn, rV, skey.p, rVc.p);
    PFDR_HIP(hipGetLastError());
    PFDR_HIP(hipStreamSynchronize(s));
}

// levels after the roots (L[0, rV)): batches of device-driven levels, the
// first few launched directly, the rest as replays of one captured batch
void CpGraphBase::bfs_device() {
    const int Vn = V;
    if (rV >= Vn) return;
    DevBuf<BfsCtl> ctl(1);
    PinnedSmall pin(s);
    BfsCtl *h = static_cast<BfsCtl *>(pin.p);
    *h = BfsCtl{0, rV, 0, 0};
    PFDR_HIP(hipMemcpyAsync(ctl.p, h, sizeof(BfsCtl), hipMemcpyHostToDevice, s));
    constexpr int step = kBlock / kSub;
    const int gc = std::min(2048, grid_for((long)Vn * kSub));
    const int ge = std::max(1, std::min(1024, (Vn + step - 1) / step));
    DevBuf<int> bsum(ge);
    auto level = [&]() {
        k_bfsd_claim<<<gc, kBlock, 0, s>>>(ctl.p, L.p, inc.ptr.p, inc.idx.p, Eu.p, Ev.p, active.p,
                                           Cv.p, claim.p);
        k_bfsd_count<<<ge, kBlock, 0, s>>>(ctl.p, L.p, inc.ptr.p, inc.idx.p, Eu.p, Ev.p, active.p,
                                           claim.p, i1.p, bsum.p);
        k_bfsd_emit<<<ge, kBlock, 0, s>>>(ctl.p, inc.ptr.p, inc.idx.p, Eu.p, Ev.p, active.p,
                                          claim.p, i1.p, bsum.p, L.p, Cv.p);
        k_bfsd_advance<<<1, kBlock, 0, s>>>(ctl.p, bsum.p, ge, Vn);
    };
    auto poll = [&]() {
        PFDR_HIP(hipMemcpyAsync(h, ctl.p, sizeof(BfsCtl), hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
        return h->done != 0;
    };
    constexpr int kFirst = 8, kBatch = 32;
    for (int i = 0; i < kFirst; i++) level();
    PFDR_HIP(hipGetLastError());
    if (!poll()) {
        hipGraph_t gr = nullptr;
        hipGraphExec_t ge_ = nullptr;
        PFDR_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        try {
            for (int i = 0; i < kBatch; i++) level();
        } catch (...) {
            (void)hipStreamEndCapture(s, &gr);
            if (gr) (void)hipGraphDestroy(gr);
            throw;
        }
        PFDR_HIP(hipStreamEndCapture(s, &gr));
        const hipError_t e = hipGraphInstantiate(&ge_, gr, nullptr, nullptr, 0);
        (void)hipGraphDestroy(gr);
        PFDR_HIP(e);
        struct Exec {
            hipStream_t s;
            hipGraphExec_t g;
            ~Exec() { (void)hipStreamSynchronize(s); (void)hipGraphExecDestroy(g); }
        } ex{s, ge_};
        // a level adds at least one vertex until done: at most V batches
        for (long b = 0; b <= (long)Vn; b++) {
            PFDR_HIP(hipGraphLaunch(ge_, s));
            if (poll()) break;
        }
    }
    if (h->overflow) throw std::runtime_error("components: BFS overflow");
    if (h->hi != Vn) throw std::runtime_error("components: BFS did not reach every vertex");
}

int CpGraphBase::activate(const uint8_t *seg, int mem) {
    DevBuf<uint8_t> bs;
    const uint8_t *ds = seg;
    if (mem != PFDR_MEM_DEVICE) {
        bs.alloc(V);
        PFDR_HIP(hipMemcpyAsync(bs.p, seg, V, hipMemcpyHostToDevice, s));
        ds = bs.p;
    }
    if (!count.p) count.alloc(1);
    PFDR_HIP(hipMemsetAsync(count.p, 0, sizeof(int), s));
    if (E > 0) k_cp_activate<<<count_grid(E), kBlock, 0, s>>>(E, Eu.p, Ev.p, ds, active.p, count.p);
    PFDR_HIP(hipGetLastError());
    return d2h_scalar(count.p, s);
}

void CpGraphBase::sx_expand(int n, const uint8_t *seg, int mem) {
    if (!K) throw std::runtime_error("simplex: call pfdr_cpgraph_simplex_setup first");
    if (!Djv.p) throw std::runtime_error("simplex: compute the gradient first");
    if (n < 1 || n >= K) throw std::runtime_error("simplex: expansion n out of [1, K)");
    DevBuf<uint8_t> bs;
    const uint8_t *ds = seg;
    if (mem != PFDR_MEM_DEVICE) {
        bs.alloc(V);
        PFDR_HIP(hipMemcpyAsync(bs.p, seg, V, hipMemcpyHostToDevice, s));
        ds = bs.p;
    }
    k_sx_expand<<<grid_for(V), kBlock, 0, s>>>(V, n, ds, Djv.p);
    PFDR_HIP(hipGetLastError());
    PFDR_HIP(hipStreamSynchronize(s));
}

int CpGraphBase::sx_activate() {
    if (!Djv.p) throw std::runtime_error("simplex: compute the gradient first");
    if (!count.p) count.alloc(1);
    PFDR_HIP(hipMemsetAsync(count.p, 0, sizeof(int), s));
    if (E > 0) k_sx_activate<<<count_grid(E), kBlock, 0, s>>>(E, Eu.p, Ev.p, Djv.p, active.p, count.p);
    PFDR_HIP(hipGetLastError());
    return d2h_scalar(count.p, s);
}

int CpGraphBase::activate_duplex(const uint8_t *seg, int mem) {
    DevBuf<uint8_t> bs;
    const uint8_t *ds = seg;
    if (mem != PFDR_MEM_DEVICE) {
        bs.alloc(2 * (size_t)V);
        PFDR_HIP(hipMemcpyAsync(bs.p, seg, 2 * (size_t)V, hipMemcpyHostToDevice, s));
        ds = bs.p;
    }
    if (!count.p) count.alloc(1);
    PFDR_HIP(hipMemsetAsync(count.p, 0, sizeof(int), s));
    if (E > 0)
        k_cp_activate_duplex<<<count_grid(E), kBlock, 0, s>>>(V, E, Eu.p, Ev.p, ds, active.p, count.p);
    PFDR_HIP(hipGetLastError());
    return d2h_scalar(count.p, s);
}

template <typename real>
struct CpGraph : CpGraphBase {
    DevBuf<real> La, L1, rX, DfS, rLa, rL1, gw, ws;
    bool has_l1 = false;

    void set_values(const void *x, int mem) override {
        if (rV <= 0) throw std::runtime_error("set_values: no components");
        rX.alloc(rV);
        PFDR_HIP(hipMemcpyAsync(rX.p, x, sizeof(real) * rV, kind_in(mem), s));
        PFDR_HIP(hipStreamSynchronize(s));
    }

    void reduced_graph(double eps_d) override {
        const real eps = (real)eps_d;
        const int Vn = V;
        const int rbits = bits_for(rV);
        DevBuf<uint8_t> nonIso(rV);
        PFDR_HIP(hipMemsetAsync(nonIso.p, 0, rV, s));
        i1.alloc(Vn + 1);
        i2.alloc(Vn + 1);
        k_rg_scan<real, false><<<grid_for(Vn), kBlock, 0, s>>>(
            Vn, rbits, Vc.p, Cv.p, inc.ptr.p, inc.idx.p, Eu.p, Ev.p, active.p, La.p, i1.p,
            nonIso.p, nullptr, nullptr, nullptr);
        PFDR_HIP(hipMemsetAsync(i1.p + Vn, 0, sizeof(int), s));
        excl_scan(tmp, i1.p, i2.p, Vn + 1, s);
        const long M = d2h_scalar(i2.p + Vn, s);
        DevBuf<unsigned long long> key(M + 1), skey(M + 1);
        DevBuf<unsigned> pos(M + 1), spos(M + 1);
        DevBuf<int> cand_e(M + 1);
        if (M > 0) {
            k_rg_scan<real, true><<<grid_for(Vn), kBlock, 0, s>>>(
                Vn, rbits, Vc.p, Cv.p, inc.ptr.p, inc.idx.p, Eu.p, Ev.p, active.p, La.p, i2.p,
                nonIso.p, key.p, pos.p, cand_e.p);
            sort_pairs(tmp, key.p, skey.p, pos.p, spos.p, M, 2 * rbits, s);
        }
        // groups
        DevBuf<int> head(M + 1), gid(M + 1);
        int G = 0;
        if (M > 0) {
            k_rg_heads<<<grid_for(M), kBlock, 0, s>>>(M, skey.p, head.p);
            PFDR_HIP(hipMemsetAsync(head.p + M, 0, sizeof(int), s));
            excl_scan(tmp, head.p, gid.p, M + 1, s);
            G = d2h_scalar(gid.p + M, s);
        }
        DevBuf<int> goff(G + 1), gru(G + 1), grv(G + 1);
        DevBuf<unsigned> gfirst(G + 1);
        gw.alloc(G + 1);
        ws.alloc(M + 1);
        if (G > 0) {
            k_rg_groups<real><<<grid_for(M), kBlock, 0, s>>>(M, rbits, skey.p, spos.p, cand_e.p,
                                                             La.p, head.p, gid.p, goff.p, gru.p,
                                                             grv.p, gfirst.p, ws.p);
            // (M fits an int: at most 2E candidates)
            const int Mi = (int)M;
            PFDR_HIP(hipMemcpyAsync(goff.p + G, &Mi, sizeof(int), hipMemcpyHostToDevice, s));
            segsum<real>(G, goff.p, nullptr, ws.p, gw.p, longs, nlong, s);
        }
        // isolated components, non-isolated list
        DevBuf<int> fl(rV + 1), isoid(rV + 1), niid(rV + 1), NI(rV + 1);
        k_flag_to_int<<<grid_for(rV), kBlock, 0, s>>>(rV, nonIso.p, 1, fl.p);
        PFDR_HIP(hipMemsetAsync(fl.p + rV, 0, sizeof(int), s));
        excl_scan(tmp, fl.p, isoid.p, rV + 1, s);
        k_flag_to_int<<<grid_for(rV), kBlock, 0, s>>>(rV, nonIso.p, 0, fl.p);
        excl_scan(tmp, fl.p, niid.p, rV + 1, s);
        k_compact_ids<<<grid_for(rV), kBlock, 0, s>>>(rV, nonIso.p, niid.p, NI.p);
        const int nIso = d2h_scalar(isoid.p + rV, s);
        const int nNI = d2h_scalar(niid.p + rV, s);
        rE = G + nIso;
        DevBuf<unsigned long long> okey(rE + 1), oskey(rE + 1);
        DevBuf<int> oval(rE + 1), osval(rE + 1);
        k_rg_order_keys<<<grid_for(G + rV), kBlock, 0, s>>>(G, rV, gru.p, gfirst.p, nonIso.p,
                                                            isoid.p, okey.p, oval.p);
        if (rE > 0) sort_pairs(tmp, okey.p, oskey.p, oval.p, osval.p, rE, 32 + rbits, s);
        rEu.alloc(rE + 1);
        rEv.alloc(rE + 1);
        rLa.alloc(rE + 1);
        if (rE > 0)
            k_rg_write<real><<<grid_for(rE), kBlock, 0, s>>>(rE, nNI, osval.p, gru.p, grv.p, gw.p,
                                                             NI.p, eps, rEu.p, rEv.p, rLa.p);
        // l1 weights: component sums in Vc order (:611-613)
        if (has_l1) {
            rL1.alloc(rV);
            segsum<real>(rV, rVc.p, Vc.p, L1.p, rL1.p, longs, nlong, s);
        }
        PFDR_HIP(hipGetLastError());
        PFDR_HIP(hipStreamSynchronize(s));
    }

    void get_reduced(int *rEu_o, int *rEv_o, void *rLa_o, void *rL1_o, int mem) override {
        const auto k = kind_out(mem);
        if (rEu_o && rE) PFDR_HIP(hipMemcpyAsync(rEu_o, rEu.p, sizeof(int) * rE, k, s));
        if (rEv_o && rE) PFDR_HIP(hipMemcpyAsync(rEv_o, rEv.p, sizeof(int) * rE, k, s));
        if (rLa_o && rE) PFDR_HIP(hipMemcpyAsync(rLa_o, rLa.p, sizeof(real) * rE, k, s));
        if (rL1_o && has_l1 && rL1.p)
            PFDR_HIP(hipMemcpyAsync(rL1_o, rL1.p, sizeof(real) * rV, k, s));
        PFDR_HIP(hipStreamSynchronize(s));
    }

    int merge(double eps, double difTol) override {
        if (!rX.p) throw std::runtime_error("merge: set the component values first");
        if (!count.p) count.alloc(1);
        PFDR_HIP(hipMemsetAsync(count.p, 0, sizeof(int), s));
        if (E > 0)
            k_cp_merge<real><<<count_grid(E), kBlock, 0, s>>>(E, Eu.p, Ev.p, Cv.p, rX.p, (real)eps,
                                                            (real)difTol, active.p, count.p);
        PFDR_HIP(hipGetLastError());
        return d2h_scalar(count.p, s);
    }

    void gradient(int N, const void *A, const void *Y, const void *R, int mem) override {
        if (!rX.p) throw std::runtime_error("gradient: set the component values first");
        DfS.alloc(V);
        const size_t asz = N > 0 ? (size_t)N * V : N < 0 ? (size_t)V * V : (size_t)V;
        const size_t ysz = (size_t)V;
        DevBuf<real> bA, bY, bR;
        auto in = [&](DevBuf<real> &b, const void *h, size_t n) -> const real * {
            if (!h) return nullptr;
            if (mem == PFDR_MEM_DEVICE) return (const real *)h;
            b.alloc(n);
            PFDR_HIP(hipMemcpyAsync(b.p, h, sizeof(real) * n, hipMemcpyHostToDevice, s));
            return b.p;
        };
        const real *dA = in(bA, A, asz);
        const real *dY = in(bY, Y, N > 0 ? 0 : ysz);
        const real *dR = in(bR, R, N > 0 ? (size_t)N : 0);
        int mode = 0;
        if (N > 0) {
            if (!dA || !dR) throw std::runtime_error("gradient: N > 0 needs A and R");
            k_cp_grad_direct<real><<<(V + kWave - 1) / kWave, kWave, 0, s>>>(N, V, dA, dR, DfS.p);
            mode = 2;
        } else if (N < 0) {
            if (-N != V || !dA || !dY) throw std::runtime_error("gradient: N < 0 needs A^tA, A^tY");
            k_cp_grad_ata<real><<<grid_for(V), kBlock, 0, s>>>(V, rV, dA, dY, Vc.p, rVc.p, rX.p,
                                                               DfS.p);
            mode = 2;
        } else {
            if (!dY) throw std::runtime_error("gradient: Y required");
            mode = dA ? 1 : 0;
        }
        k_cp_grad<real><<<grid_for(V), kBlock, 0, s>>>(V, mode, dA, dY, inc.ptr.p, inc.idx.p, Eu.p,
                                                       Ev.p, active.p, La.p,
                                                       has_l1 ? L1.p : nullptr, Cv.p, rX.p, DfS.p);
        PFDR_HIP(hipGetLastError());
        PFDR_HIP(hipStreamSynchronize(s));
    }

    void get_dfs(void *out, int mem) override {
        if (!DfS.p) throw std::runtime_error("no gradient computed");
        PFDR_HIP(hipMemcpyAsync(out, DfS.p, sizeof(real) * V, kind_out(mem), s));
        PFDR_HIP(hipStreamSynchronize(s));
    }

    void capacities_bounds(int cut, double mn, double mx, void *tr, void *rc, int mem) override {
        capacities_impl(cut, 0, true, (real)mn, (real)mx, tr, rc, mem);
    }
    void capacities(int cut, int positivity, void *tr, void *rc, int mem) override {
        if (cut == 2 && !positivity && !has_l1)
            throw std::runtime_error("capacities: cut 2 without positivity needs La_l1");
        capacities_impl(cut, positivity, false, real(0), real(0), tr, rc, mem);
    }
    void capacities_impl(int cut, int positivity, bool bounds, real mn, real mx, void *tr,
                         void *rc, int mem) {
        if (!DfS.p) throw std::runtime_error("capacities: compute the gradient first");
        DevBuf<real> btr, brc;
        real *dtr = (real *)tr, *drc = (real *)rc;
        if (mem != PFDR_MEM_DEVICE) {
            btr.alloc(V);
            brc.alloc(E > 0 ? E : 1);
            dtr = btr.p;
            drc = brc.p;
        }
        if (tr && bounds)
            k_cp_trcap_bounds<real><<<grid_for(V), kBlock, 0, s>>>(V, cut, mn, mx, Cv.p, rX.p,
                                                                   DfS.p, dtr);
        else if (tr)
            k_cp_trcap<real><<<grid_for(V), kBlock, 0, s>>>(V, cut, positivity,
                                                            has_l1 ? L1.p : nullptr, Cv.p, rX.p,
                                                            DfS.p, dtr);
        if (rc && E > 0) k_cp_rcap<real><<<grid_for(E), kBlock, 0, s>>>(E, active.p, La.p, drc);
        PFDR_HIP(hipGetLastError());
        if (mem != PFDR_MEM_DEVICE) {  // the caller's arrays pinned for the DMA (HostPins)
            HostPins hp(s);
            if (tr) hp.copy(tr, dtr, sizeof(real) * V, hipMemcpyDeviceToHost);
            if (rc && E > 0) hp.copy(rc, drc, sizeof(real) * E, hipMemcpyDeviceToHost);
            hp.release();
        }
        PFDR_HIP(hipStreamSynchronize(s));
    }

    // ---- the duplex driver's two-layer cut
    void capacities_duplex(int positivity, void *tr, void *link, void *rc, int mem) override {
        if (!DfS.p) throw std::runtime_error("capacities_duplex: compute the gradient first");
        if (!has_l1 && !positivity)
            throw std::runtime_error("capacities_duplex: differentiable problem (one-layer cut)");
        DevBuf<real> btr, bln, brc;
        real *dtr = (real *)tr, *dln = (real *)link, *drc = (real *)rc;
        if (mem != PFDR_MEM_DEVICE) {
            btr.alloc(2 * (size_t)V);
            bln.alloc(V);
            brc.alloc(E > 0 ? E : 1);
            dtr = btr.p;
            dln = bln.p;
            drc = brc.p;
        }
        if (tr || link) {
            if (!tr) { btr.alloc(2 * (size_t)V); dtr = btr.p; }
            if (!link) { bln.alloc(V); dln = bln.p; }
            k_cp_trcap_duplex<real><<<grid_for(V), kBlock, 0, s>>>(
                V, positivity, has_l1 ? L1.p : nullptr, Cv.p, rX.p, DfS.p, dtr, dln);
        }
        if (rc && E > 0) k_cp_rcap<real><<<grid_for(E), kBlock, 0, s>>>(E, active.p, La.p, drc);
        PFDR_HIP(hipGetLastError());
        if (mem != PFDR_MEM_DEVICE) {
            if (tr)
                PFDR_HIP(hipMemcpyAsync(tr, dtr, sizeof(real) * 2 * V, hipMemcpyDeviceToHost, s));
            if (link) PFDR_HIP(hipMemcpyAsync(link, dln, sizeof(real) * V, hipMemcpyDeviceToHost, s));
            if (rc && E > 0)
                PFDR_HIP(hipMemcpyAsync(rc, drc, sizeof(real) * E, hipMemcpyDeviceToHost, s));
        }
        PFDR_HIP(hipStreamSynchronize(s));
    }

    // ---- the simplex driver
    real sal = real(0);
    DevBuf<real> Q, Qt, rP, DfSK, S;

    void sx_setup(int K_, double al, const void *q, int mem) override {
        if (K_ < 2 || !q) throw std::runtime_error("simplex_setup: K >= 2 and Q required");
        if (!(al >= 0.0 && al <= 1.0)) throw std::runtime_error("simplex_setup: al in [0, 1]");
        K = K_;
        sal = (real)al;
        const size_t n = (size_t)V * K;
        Q.alloc(n);
        Qt.alloc(n);
        PFDR_HIP(hipMemcpyAsync(Q.p, q, sizeof(real) * n, kind_in(mem), s));
        k_sx_transpose<real><<<grid_for((long)n), kBlock, 0, s>>>(V, K, Q.p, Qt.p);
        PFDR_HIP(hipGetLastError());
        rP.release();
        DfSK.release();
        Djv.release();
        PFDR_HIP(hipStreamSynchronize(s));
    }

    void need_k(const char *fn) const {
        if (!K) throw std::runtime_error(std::string(fn) + ": call pfdr_cpgraph_simplex_setup first");
    }

    // :733-766 (and initialize() :96-108): per label the ordered sums of Qt
    // over each component's vertices in Vc order, then the observations;
    // rP becomes the component values
    void sx_observations(void *rPo, void *rQo, void *rLafo, int mem) override {
        need_k("simplex_observations");
        S.alloc((size_t)rV * K);
        // every label in one launch pair: (component, label) segments side by side
        segsum<real>(rV, rVc.p, Vc.p, Qt.p, S.p, longs, nlong, s, K, (long)V);
        rP.alloc((size_t)rV * K);
        DevBuf<real> bQ((size_t)rV * K), bL(rV);
        const int linear = sal == real(0);
        k_sx_observations<real><<<grid_for(rV), kBlock, 0, s>>>(rV, K, linear, S.p, rVc.p, rP.p,
                                                                bQ.p, linear ? nullptr : bL.p);
        PFDR_HIP(hipGetLastError());
        const auto ko = kind_out(mem);
        if (rPo) PFDR_HIP(hipMemcpyAsync(rPo, rP.p, sizeof(real) * rV * K, ko, s));
        if (rQo) PFDR_HIP(hipMemcpyAsync(rQo, bQ.p, sizeof(real) * rV * K, ko, s));
        if (rLafo && !linear) PFDR_HIP(hipMemcpyAsync(rLafo, bL.p, sizeof(real) * rV, ko, s));
        PFDR_HIP(hipStreamSynchronize(s));
    }

    void sx_set_values(const void *x, int mem) override {
        need_k("simplex_set_values");
        rP.alloc((size_t)rV * K);
        PFDR_HIP(hipMemcpyAsync(rP.p, x, sizeof(real) * rV * K, kind_in(mem), s));
        PFDR_HIP(hipStreamSynchronize(s));
    }

    // :327-376 DfS[V*K]; :523-536 rDi, Djv = 0
    void sx_gradient(double eps, void *out, int *rDio, int mem) override {
        need_k("simplex_gradient");
        if (!rP.p) throw std::runtime_error("simplex_gradient: set the component values first");
        const size_t n = (size_t)V * K;
        DfSK.alloc(n);
        real alK = real(0), al1 = real(0), alKal1 = real(0);
        if (real(0) < sal && sal < real(1)) {  // :208-212
            alK = sal / (real)K;
            al1 = real(1) - sal;
            alKal1 = alK / al1;
        }
        const int loss = sal == real(0) ? 0 : sal == real(1) ? 1 : 2;
        k_sx_gradient<real><<<grid_for((long)n), kBlock, 0, s>>>(
            V, K, loss, alK, al1, alKal1, Q.p, inc.ptr.p, inc.idx.p, Eu.p, Ev.p, active.p, La.p,
            Cv.p, rP.p, (real)eps, DfSK.p);
        rDi.alloc(rV);
        k_sx_best<real><<<grid_for(rV), kBlock, 0, s>>>(rV, K, rP.p, rDi.p);
        Djv.alloc(V);
        PFDR_HIP(hipMemsetAsync(Djv.p, 0, sizeof(int) * V, s));
        PFDR_HIP(hipGetLastError());
        const auto ko = kind_out(mem);
        if (out) PFDR_HIP(hipMemcpyAsync(out, DfSK.p, sizeof(real) * n, ko, s));
        if (rDio) PFDR_HIP(hipMemcpyAsync(rDio, rDi.p, sizeof(int) * rV, ko, s));
        PFDR_HIP(hipStreamSynchronize(s));
    }

    void sx_capacities(int n, void *tr, void *rc, int mem) override {
        need_k("simplex_capacities");
        if (!DfSK.p || !Djv.p) throw std::runtime_error("simplex_capacities: compute the gradient first");
        if (n < 1 || n >= K) throw std::runtime_error("simplex_capacities: n out of [1, K)");
        DevBuf<real> btr, brc;
        real *dtr = (real *)tr, *drc = (real *)rc;
        if (mem != PFDR_MEM_DEVICE) {
            btr.alloc(V);
            brc.alloc(E > 0 ? E : 1);
            dtr = btr.p;
            drc = brc.p;
        }
        if (tr)
            k_sx_trcap<real><<<grid_for(V), kBlock, 0, s>>>(V, K, n, inc.ptr.p, inc.idx.p, Eu.p,
                                                            Ev.p, active.p, La.p, Cv.p, rDi.p,
                                                            Djv.p, DfSK.p, dtr);
        if (rc && E > 0)
            k_sx_rcap<real><<<grid_for(E), kBlock, 0, s>>>(E, Eu.p, Ev.p, active.p, La.p, Djv.p,
                                                           drc);
        PFDR_HIP(hipGetLastError());
        if (mem != PFDR_MEM_DEVICE) {  // the caller's arrays pinned for the DMA (HostPins)
            HostPins hp(s);
            if (tr) hp.copy(tr, dtr, sizeof(real) * V, hipMemcpyDeviceToHost);
            if (rc && E > 0) hp.copy(rc, drc, sizeof(real) * E, hipMemcpyDeviceToHost);
            hp.release();
        }
        PFDR_HIP(hipStreamSynchronize(s));
    }

    int sx_merge(double eps) override {
        need_k("simplex_merge");
        if (!rP.p) throw std::runtime_error("simplex_merge: set the component values first");
        if (!count.p) count.alloc(1);
        PFDR_HIP(hipMemsetAsync(count.p, 0, sizeof(int), s));
        if (E > 0)
            k_sx_merge<real><<<count_grid(E), kBlock, 0, s>>>(E, K, Eu.p, Ev.p, Cv.p, rP.p,
                                                            (real)eps, active.p, count.p);
        PFDR_HIP(hipGetLastError());
        return d2h_scalar(count.p, s);
    }
};

}  // namespace pfdr

struct pfdr_cpgraph {
    pfdr::CpGraphBase *g;
};

using pfdr::report_error;

#define CPG_TRY(fn, body)                                  \
    try {                                                  \
        pfdr::StreamScope sc_(h->g->s, h->g->dev);         \
        body;                                              \
    } catch (const pfdr::HipError &h) {                    \
        return report_error(fn, h);                        \
    } catch (const std::exception &ex) {                   \
        return report_error(fn, ex.what());                \
    }                                                      \
    return PFDR_OK;

template <typename real>
static pfdr::CpGraphBase *cpg_new(int V, int E, const int *Eu, const int *Ev, const void *La_d1,
                                  const void *La_l1, int mem) {
    using namespace pfdr;
    auto *g = new CpGraph<real>();
    std::unique_ptr<CpGraph<real>> hold(g);
    g->V = V;
    g->E = E;
    g->dtype = sizeof(real) == 4 ? PFDR_F32 : PFDR_F64;
    g->s = lib_stream();
    PFDR_HIP(hipGetDevice(&g->dev));
    const auto k = kind_in(mem);
    g->Eu.alloc(E > 0 ? E : 1);
    g->Ev.alloc(E > 0 ? E : 1);
    g->La.alloc(E > 0 ? E : 1);
    if (E > 0) {
        PFDR_HIP(hipMemcpyAsync(g->Eu.p, Eu, sizeof(int) * E, k, g->s));
        PFDR_HIP(hipMemcpyAsync(g->Ev.p, Ev, sizeof(int) * E, k, g->s));
        PFDR_HIP(hipMemcpyAsync(g->La.p, La_d1, sizeof(real) * E, k, g->s));
    }
    g->has_l1 = La_l1 != nullptr;
    if (La_l1) {
        g->L1.alloc(V);
        PFDR_HIP(hipMemcpyAsync(g->L1.p, La_l1, sizeof(real) * V, k, g->s));
    }
    build_incidence(g->Eu.p, g->Ev.p, V, E, g->inc, g->s);  // validates the endpoints
    g->active.alloc(E > 0 ? E : 1);
    PFDR_HIP(hipMemsetAsync(g->active.p, 0, E > 0 ? E : 1, g->s));
    // CP's initial state: one component, Vc = 0..V-1 (:181-187)
    g->rV = 1;
    g->Cv.alloc(V);
    g->Vc.alloc(V);
    g->rVc.alloc(V + 1);
    PFDR_HIP(hipMemsetAsync(g->Cv.p, 0, sizeof(int) * V, g->s));
    {
        std::vector<int> iota(V);
        for (int v = 0; v < V; v++) iota[v] = v;
        PFDR_HIP(hipMemcpyAsync(g->Vc.p, iota.data(), sizeof(int) * V, hipMemcpyHostToDevice, g->s));
        const int r[2] = {0, V};
        PFDR_HIP(hipMemcpyAsync(g->rVc.p, r, sizeof r, hipMemcpyHostToDevice, g->s));
        PFDR_HIP(hipStreamSynchronize(g->s));
    }
    hold.release();
    return g;
}

extern "C" int pfdr_cpgraph_create(pfdr_cpgraph **out, int dtype, int V, int E, const int *Eu,
                                   const int *Ev, const void *La_d1, const void *La_l1, int mem) {
    const char *fn = "pfdr_cpgraph_create";
    if (!out || V <= 0 || E < 0 || (E > 0 && (!Eu || !Ev || !La_d1)) ||
        (dtype != PFDR_F32 && dtype != PFDR_F64))
        return report_error(fn, "invalid arguments");
    if ((long)E * 2 >= (1L << 31)) return report_error(fn, "E must be < 2^30");
    *out = nullptr;
    try {
        pfdr::CpGraphBase *g = dtype == PFDR_F32
                                   ? cpg_new<float>(V, E, Eu, Ev, La_d1, La_l1, mem)
                                   : cpg_new<double>(V, E, Eu, Ev, La_d1, La_l1, mem);
        *out = new pfdr_cpgraph{g};
    } catch (const pfdr::HipError &h) {
        return report_error(fn, h);
    } catch (const std::exception &ex) {
        return report_error(fn, ex.what());
    }
    return PFDR_OK;
}

extern "C" void pfdr_cpgraph_destroy(pfdr_cpgraph *g) {
    if (!g) return;
    try {
        pfdr::StreamScope sc(g->g->s, g->g->dev);
        (void)hipStreamSynchronize(g->g->s);
        delete g->g;
    } catch (...) {
    }
    delete g;
}

extern "C" int pfdr_cpgraph_set_active(pfdr_cpgraph *h, const uint8_t *active, int mem) {
    if (!h || !active) return report_error("pfdr_cpgraph_set_active", "null argument");
    CPG_TRY("pfdr_cpgraph_set_active", {
        auto *g = h->g;
        if (g->E > 0)
            PFDR_HIP(hipMemcpyAsync(g->active.p, active, g->E, pfdr::kind_in(mem), g->s));
        PFDR_HIP(hipStreamSynchronize(g->s));
    })
}

extern "C" int pfdr_cpgraph_get_active(pfdr_cpgraph *h, uint8_t *active, int mem) {
    if (!h || !active) return report_error("pfdr_cpgraph_get_active", "null argument");
    CPG_TRY("pfdr_cpgraph_get_active", {
        auto *g = h->g;
        if (g->E > 0)
            PFDR_HIP(hipMemcpyAsync(active, g->active.p, g->E, pfdr::kind_out(mem), g->s));
        PFDR_HIP(hipStreamSynchronize(g->s));
    })
}

extern "C" int pfdr_cpgraph_set_components(pfdr_cpgraph *h, int rV, const int *Cv, const int *Vc,
                                           const int *rVc, int mem) {
    const char *fn = "pfdr_cpgraph_set_components";
    if (!h || !Cv || !Vc || !rVc || rV <= 0 || rV > h->g->V)
        return report_error(fn, "invalid arguments");
    CPG_TRY(fn, {
        auto *g = h->g;
        const auto k = pfdr::kind_in(mem);
        g->rV = rV;
        PFDR_HIP(hipMemcpyAsync(g->Cv.p, Cv, sizeof(int) * g->V, k, g->s));
        PFDR_HIP(hipMemcpyAsync(g->Vc.p, Vc, sizeof(int) * g->V, k, g->s));
        PFDR_HIP(hipMemcpyAsync(g->rVc.p, rVc, sizeof(int) * (rV + 1), k, g->s));
        PFDR_HIP(hipStreamSynchronize(g->s));
    })
}

extern "C" int pfdr_cpgraph_get_components(pfdr_cpgraph *h, int *rV, int *Cv, int *Vc, int *rVc,
                                           int mem) {
    if (!h) return report_error("pfdr_cpgraph_get_components", "null graph");
    CPG_TRY("pfdr_cpgraph_get_components", {
        auto *g = h->g;
        const auto k = pfdr::kind_out(mem);
        if (rV) *rV = g->rV;
        if (Cv) PFDR_HIP(hipMemcpyAsync(Cv, g->Cv.p, sizeof(int) * g->V, k, g->s));
        if (Vc) PFDR_HIP(hipMemcpyAsync(Vc, g->Vc.p, sizeof(int) * g->V, k, g->s));
        if (rVc) PFDR_HIP(hipMemcpyAsync(rVc, g->rVc.p, sizeof(int) * (g->rV + 1), k, g->s));
        PFDR_HIP(hipStreamSynchronize(g->s));
    })
}

extern "C" int pfdr_cpgraph_set_values(pfdr_cpgraph *h, const void *rX, int mem) {
    if (!h || !rX) return report_error("pfdr_cpgraph_set_values", "null argument");
    CPG_TRY("pfdr_cpgraph_set_values", h->g->set_values(rX, mem))
}

extern "C" int pfdr_cpgraph_components(pfdr_cpgraph *h, int *rV) {
    if (!h) return report_error("pfdr_cpgraph_components", "null graph");
    CPG_TRY("pfdr_cpgraph_components", {
        h->g->components();
        if (rV) *rV = h->g->rV;
    })
}

extern "C" int pfdr_cpgraph_reduced_graph(pfdr_cpgraph *h, double eps, int *rE) {
    if (!h) return report_error("pfdr_cpgraph_reduced_graph", "null graph");
    CPG_TRY("pfdr_cpgraph_reduced_graph", {
        h->g->reduced_graph(eps);
        if (rE) *rE = h->g->rE;
    })
}

extern "C" int pfdr_cpgraph_get_reduced(pfdr_cpgraph *h, int *rEu, int *rEv, void *rLa_d1,
                                        void *rLa_l1, int mem) {
    if (!h) return report_error("pfdr_cpgraph_get_reduced", "null graph");
    CPG_TRY("pfdr_cpgraph_get_reduced", h->g->get_reduced(rEu, rEv, rLa_d1, rLa_l1, mem))
}

extern "C" int pfdr_cpgraph_merge(pfdr_cpgraph *h, double eps, double difTol, int *deactivated) {
    if (!h) return report_error("pfdr_cpgraph_merge", "null graph");
    CPG_TRY("pfdr_cpgraph_merge", {
        const int n = h->g->merge(eps, difTol);
        if (deactivated) *deactivated = n;
    })
}

extern "C" int pfdr_cpgraph_gradient(pfdr_cpgraph *h, int N, const void *A, const void *Y,
                                     const void *R, int mem, void *DfS) {
    if (!h) return report_error("pfdr_cpgraph_gradient", "null graph");
    CPG_TRY("pfdr_cpgraph_gradient", {
        h->g->gradient(N, A, Y, R, mem);
        if (DfS) h->g->get_dfs(DfS, mem);
    })
}

extern "C" int pfdr_cpgraph_capacities(pfdr_cpgraph *h, int cut, int positivity, void *tr_cap,
                                       void *r_cap, int mem) {
    if (!h || cut < 0 || cut > 2) return report_error("pfdr_cpgraph_capacities", "invalid arguments");
    CPG_TRY("pfdr_cpgraph_capacities", h->g->capacities(cut, positivity, tr_cap, r_cap, mem))
}

extern "C" int pfdr_cpgraph_capacities_bounds(pfdr_cpgraph *h, int cut, double min, double max,
                                              void *tr_cap, void *r_cap, int mem) {
    if (!h || cut < 0 || cut > 2)
        return report_error("pfdr_cpgraph_capacities_bounds", "invalid arguments");
    CPG_TRY("pfdr_cpgraph_capacities_bounds",
            h->g->capacities_bounds(cut, min, max, tr_cap, r_cap, mem))
}

extern "C" int pfdr_cpgraph_activate(pfdr_cpgraph *h, const uint8_t *segment, int mem,
                                     int *activated) {
    if (!h || !segment) return report_error("pfdr_cpgraph_activate", "null argument");
    CPG_TRY("pfdr_cpgraph_activate", {
        const int n = h->g->activate(segment, mem);
        if (activated) *activated = n;
    })
}

// ------------------------------------------------- the simplex driver --
extern "C" int pfdr_cpgraph_simplex_setup(pfdr_cpgraph *h, int K, double al, const void *Q,
                                          int mem) {
    if (!h || !Q || K < 2) return report_error("pfdr_cpgraph_simplex_setup", "invalid arguments");
    CPG_TRY("pfdr_cpgraph_simplex_setup", h->g->sx_setup(K, al, Q, mem))
}

extern "C" int pfdr_cpgraph_simplex_observations(pfdr_cpgraph *h, void *rP, void *rQ,
                                                 void *rLa_f, int mem) {
    if (!h) return report_error("pfdr_cpgraph_simplex_observations", "null graph");
    CPG_TRY("pfdr_cpgraph_simplex_observations", h->g->sx_observations(rP, rQ, rLa_f, mem))
}

extern "C" int pfdr_cpgraph_simplex_set_values(pfdr_cpgraph *h, const void *rP, int mem) {
    if (!h || !rP) return report_error("pfdr_cpgraph_simplex_set_values", "null argument");
    CPG_TRY("pfdr_cpgraph_simplex_set_values", h->g->sx_set_values(rP, mem))
}

extern "C" int pfdr_cpgraph_simplex_gradient(pfdr_cpgraph *h, double eps, void *DfS, int *rDi,
                                             int mem) {
    if (!h) return report_error("pfdr_cpgraph_simplex_gradient", "null graph");
    CPG_TRY("pfdr_cpgraph_simplex_gradient", h->g->sx_gradient(eps, DfS, rDi, mem))
}

extern "C" int pfdr_cpgraph_simplex_capacities(pfdr_cpgraph *h, int n, void *tr_cap, void *r_cap,
                                               int mem) {
    if (!h) return report_error("pfdr_cpgraph_simplex_capacities", "null graph");
    CPG_TRY("pfdr_cpgraph_simplex_capacities", h->g->sx_capacities(n, tr_cap, r_cap, mem))
}

extern "C" int pfdr_cpgraph_simplex_expand(pfdr_cpgraph *h, int n, const uint8_t *segment,
                                           int mem) {
    if (!h || !segment) return report_error("pfdr_cpgraph_simplex_expand", "null argument");
    CPG_TRY("pfdr_cpgraph_simplex_expand", h->g->sx_expand(n, segment, mem))
}

extern "C" int pfdr_cpgraph_simplex_activate(pfdr_cpgraph *h, int *activated) {
    if (!h) return report_error("pfdr_cpgraph_simplex_activate", "null graph");
    CPG_TRY("pfdr_cpgraph_simplex_activate", {
        const int n = h->g->sx_activate();
        if (activated) *activated = n;
    })
}

extern "C" int pfdr_cpgraph_simplex_merge(pfdr_cpgraph *h, double eps, int *deactivated) {
    if (!h) return report_error("pfdr_cpgraph_simplex_merge", "null graph");
    CPG_TRY("pfdr_cpgraph_simplex_merge", {
        const int n = h->g->sx_merge(eps);
        if (deactivated) *deactivated = n;
    })
}

extern "C" int pfdr_cpgraph_simplex_labels(pfdr_cpgraph *h, int *Djv, int mem) {
    if (!h || !Djv) return report_error("pfdr_cpgraph_simplex_labels", "null argument");
    CPG_TRY("pfdr_cpgraph_simplex_labels", {
        auto *g = h->g;
        if (!g->Djv.p) throw std::runtime_error("simplex_labels: compute the gradient first");
        PFDR_HIP(hipMemcpyAsync(Djv, g->Djv.p, sizeof(int) * g->V, pfdr::kind_out(mem), g->s));
        PFDR_HIP(hipStreamSynchronize(g->s));
    })
}

// ---------------------------------------------------- the duplex driver --
extern "C" int pfdr_cpgraph_capacities_duplex(pfdr_cpgraph *h, int positivity, void *tr_cap,
                                              void *r_link, void *r_cap, int mem) {
    if (!h) return report_error("pfdr_cpgraph_capacities_duplex", "null graph");
    CPG_TRY("pfdr_cpgraph_capacities_duplex",
            h->g->capacities_duplex(positivity, tr_cap, r_link, r_cap, mem))
}

extern "C" int pfdr_cpgraph_activate_duplex(pfdr_cpgraph *h, const uint8_t *segment, int mem,
                                            int *activated) {
    if (!h || !segment) return report_error("pfdr_cpgraph_activate_duplex", "null argument");
    CPG_TRY("pfdr_cpgraph_activate_duplex", {
        const int n = h->g->activate_duplex(segment, mem);
        if (activated) *activated = n;
    })
}
