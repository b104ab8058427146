// Strictly sequential floating-point sum of NONNEGATIVE terms,
// s <- fl(s + a[0]), s <- fl(s + a[1]), ..., computed by a whole workgroup
// with the same rounding as the one-lane loop.
//
// Why it parallelises: with a[i] >= 0 the running sum never decreases, so
// it crosses each binade [2^e, 2^(e+1)) at most once.  While s stays in one
// binade every float it can take is a multiple of u = ulp(s), and
// fl(s + a) = s + u * r(a / u), where r rounds to an integer: down below a
// half, up above, and on an exact half to the even one of the two
// neighbours of s/u + a/u, which depends only on the PARITY of s/u.  A run
// of terms is therefore summarised by the pair (d0, d1) of integer
// increments it adds for an even / odd starting s/u; pairs compose
// associatively ((A.B)_p = A_p + B_(p + A_p mod 2)), so a workgroup scans a
// tile of terms in log steps.  The first term whose result would leave the
// binade (s/u + increment >= 2^p, or a term itself >= 2^(e+1)) is added
// with one ordinary floating-point addition, the binade and u are taken
// from the new s, and the scan resumes after that term: one restart per
// binade crossing (about log2(sum / first term) of them), each a tile.
//
// Used for the amplitude sum of the preconditioner, whose order is the
// reference's single-thread loop (src/PFDR_graph_quadratic_d1_l1.cpp:146-152).
#pragma once
#include "pfdr_dev.hpp"

namespace pfdr {

template <typename real> struct FpGrid;
template <> struct FpGrid<float> {
    static constexpr int p = 24, emin = -126;
    static constexpr float min_normal = 1.17549435082228750797e-38f;
};
template <> struct FpGrid<double> {
    static constexpr int p = 53, emin = -1022;
    static constexpr double min_normal = 2.2250738585072013831e-308;
};

// exponent of the spacing of the floats around s >= 0 (subnormals and 0 share
// the spacing of the smallest normal binade)
template <typename real>
__device__ __forceinline__ int grid_exp(real s) {
    const int e = (s >= FpGrid<real>::min_normal) ? ilogb(s) : FpGrid<real>::emin;
    return e - FpGrid<real>::p + 1;
}

// term a >= 0 on the grid 2^ue: floor(a / u) and how the remainder rounds
// (0 down, 1 up, 2 exact half, 3 the term alone reaches 2^p u)
template <typename real>
__device__ __forceinline__ void grid_term(real a, int ue, long long &fl, int &cls) {
    constexpr real top = real(1ll << FpGrid<real>::p);
    const real q = ldexp(a, -ue);  // exact (a scaled by a power of two), or
    if (!(q < top)) {              // underflowed far below one half
        fl = 0;
        cls = 3;
        return;
    }
    const real f = floor(q), r = q - f;
    fl = (long long)f;
    cls = r < real(0.5) ? 0 : (r > real(0.5) ? 1 : 2);
}

template <typename real>
__device__ __forceinline__ long long grid_inc(long long fl, int cls, long long parity) {
    constexpr long long cap = (1ll << FpGrid<real>::p) + 1;
    return cls == 3 ? cap : fl + (cls == 2 ? ((parity + fl) & 1) : cls);
}

// (d0, d1) summaries; increments saturate at 2^p + 1 (past that point the
// binade has been left and everything after the exit is discarded)
template <typename real>
__device__ __forceinline__ long long sat_add(long long a, long long b) {
    constexpr long long cap = (1ll << FpGrid<real>::p) + 1;
    const long long x = a + b;
    return x > cap ? cap : x;
}
template <typename real>
__device__ __forceinline__ void compose(long long a0, long long a1, long long &b0, long long &b1) {
    // (A then B) for start parity 0 and 1; result in (b0, b1)
    const long long n0 = sat_add<real>(a0, (a0 & 1) ? b1 : b0);
    const long long n1 = sat_add<real>(a1, ((1 + a1) & 1) ? b1 : b0);
    b0 = n0;
    b1 = n1;
}

constexpr int kMonoThreads = 512;
constexpr int kMonoCand = 3;  // binades summarised per tile (predicted, one below, one above)

template <typename real>
struct MonoTile {
    static constexpr int J = 64 / sizeof(real);             // terms per lane
    static constexpr long TILE = (long)kMonoThreads * J;     // terms per tile
};

constexpr int kMonoSerial = 256;  // terms added by one lane after each exit

// Shared state of a workgroup walking terms one tile at a time.
struct MonoShared {
    alignas(16) char ser[kMonoSerial * sizeof(double)];
    long long w0[kMonoThreads / kWave], w1[kMonoThreads / kWave];
    int exit_at;
    int k;
    long long S;
    double sd;  // the running sum's bits travel as a double (exact for both reals)
};

// the J terms of lane t of the tile at `b` (zeros outside [0, n))
template <typename real>
__device__ __forceinline__ void mono_load(real *x, const real *__restrict__ a, long n, long b,
                                          int t) {
    constexpr int J = MonoTile<real>::J, W = Vec<real>::kPer16B;
    using P = Pk<real, W>;
    const long i0 = b + (long)t * J;
    if (i0 + J <= n && ((reinterpret_cast<uintptr_t>(a + i0) & 15) == 0)) {
#pragma unroll
        for (int v = 0; v < J / W; v++) {
            const P pk = *reinterpret_cast<const P *>(a + i0 + v * W);
#pragma unroll
            for (int k = 0; k < W; k++) x[v * W + k] = pk.v[k];
        }
    } else {
#pragma unroll
        for (int j = 0; j < J; j++) x[j] = (i0 + j < n) ? a[i0 + j] : real(0);
    }
}

// lane summary (d0, d1) of J terms on the grid 2^ue
template <typename real>
__device__ __forceinline__ void mono_run(const real *x, int ue, long long &d0, long long &d1) {
    d0 = d1 = 0;
#pragma unroll
    for (int j = 0; j < MonoTile<real>::J; j++) {
        long long fl;
        int cls;
        grid_term(x[j], ue, fl, cls);
        d0 = sat_add<real>(d0, grid_inc<real>(fl, cls, d0));
        d1 = sat_add<real>(d1, grid_inc<real>(fl, cls, 1 + d1));
    }
}

// inclusive scan of summaries over the wave (earlier lanes first)
template <typename real>
__device__ __forceinline__ void mono_wave_scan(long long &i0, long long &i1, int lane) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const long long p0 = __shfl_up(i0, o, kWave), p1 = __shfl_up(i1, o, kWave);
        if (lane >= o) compose<real>(p0, p1, i0, i1);
    }
}

// s + a[lo] + ... + a[hi-1] by the whole workgroup, term by term semantics:
// scans tile after tile on the binade of s, adds the first term that leaves
// it with one floating-point addition, and resumes after that term.
template <typename real>
__device__ real mono_range(const real *__restrict__ a, long lo, long hi, real s, MonoShared &sh) {
    constexpr int NT = kMonoThreads, J = MonoTile<real>::J;
    constexpr long TILE = MonoTile<real>::TILE;
    constexpr long long TOP = 1ll << FpGrid<real>::p;
    const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
    // tiles are aligned to TILE (16-byte loads); terms before `start` are
    // masked to zero, which adds nothing
    long start = lo;
    real x[J], nx[J];
    bool have = false;  // nx holds the tile at `base`
    while (start < hi && s < Lim<real>::huge) {
        const int ue = grid_exp(s);
        long long S = (long long)ldexp(s, -ue);  // s / u, an integer below 2^p
        bool left = false;
        for (long base = start / TILE * TILE; base < hi; base += TILE) {
            if (have) {
#pragma unroll
                for (int j = 0; j < J; j++) x[j] = nx[j];
            } else {
                mono_load(x, a, hi, base, t);
            }
            const bool more = base + TILE < hi;
            if (more) mono_load(nx, a, hi, base + TILE, t);  // in flight during the scan
            have = more;
            if (start > base) {
#pragma unroll
                for (int j = 0; j < J; j++)
                    if (base + (long)t * J + j < start) x[j] = real(0);
            }
            long long r0, r1;
            mono_run(x, ue, r0, r1);
            long long i0 = r0, i1 = r1;
            mono_wave_scan<real>(i0, i1, lane);
            if (lane == kWave - 1) {
                sh.w0[w] = i0;
                sh.w1[w] = i1;
            }
            long long e0 = __shfl_up(i0, 1, kWave), e1 = __shfl_up(i1, 1, kWave);
            if (lane == 0) e0 = e1 = 0;
            __syncthreads();
            // prefix of the earlier waves (in order), then this lane's start
            long long q0 = 0, q1 = 0;
            for (int k = 0; k < w; k++) {
                long long b0 = sh.w0[k], b1 = sh.w1[k];
                compose<real>(q0, q1, b0, b1);
                q0 = b0;
                q1 = b1;
            }
            compose<real>(q0, q1, e0, e1);
            // this lane's exact starting count; only a lane whose run ends
            // outside the binade walks its terms to find the exit
            long long cur = sat_add<real>(S, (S & 1) ? e1 : e0), cex = 0;
            const long long end = sat_add<real>(cur, (cur & 1) ? r1 : r0);
            int mine = INT_MAX;
            real xex = real(0);
            if (end >= TOP) {
#pragma unroll
                for (int j = 0; j < J; j++) {
                    long long fl;
                    int cls;
                    grid_term(x[j], ue, fl, cls);  // recomputed: fewer live registers
                    const long long inc = grid_inc<real>(fl, cls, cur);
                    if (mine == INT_MAX && (cls == 3 || cur + inc >= TOP)) {
                        mine = t * J + j;
                        cex = cur;
                        xex = x[j];
                    }
                    cur = sat_add<real>(cur, inc);
                }
            }
            cur = end;
            if (mine != INT_MAX) atomicMin(&sh.exit_at, mine);
            __syncthreads();
            const int ex = sh.exit_at;
            if (ex == INT_MAX) {  // the whole tile stays in the binade
                if (t == NT - 1) sh.S = cur;
                __syncthreads();
                S = sh.S;
                __syncthreads();
                continue;
            }
            // the earliest exit term: one ordinary addition (s = cex * u exactly)
            if (mine == ex) sh.sd = (double)(ldexp((real)cex, ue) + xex);
            __syncthreads();
            s = (real)sh.sd;
            if (t == 0) sh.exit_at = INT_MAX;
            // exits cluster where the sum is young (it doubles every few
            // terms): the next kMonoSerial terms are added by one lane, from LDS
            start = base + ex + 1;
            const int m = (int)min((long)kMonoSerial, hi - start);
            real *buf = reinterpret_cast<real *>(sh.ser);
            for (int i = t; i < m; i += NT) buf[i] = a[start + i];
            __syncthreads();
            if (t == 0) sh.sd = (double)ordered_add(s, buf, m);
            __syncthreads();
            s = (real)sh.sd;
            start += m;
            have = false;
            left = true;
            __syncthreads();
            break;
        }
        if (!left) {
            s = ldexp((real)S, ue);
            break;
        }
    }
    return s;
}

template <typename real>
__device__ __forceinline__ void mono_count(int nparts, const int *__restrict__ cnt_part,
                                           long long *__restrict__ cnt_out, MonoShared &sh) {
    const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
    long long c = 0;
    for (int i = t; i < nparts; i += kMonoThreads) c += cnt_part[i];
    c = wave_sum(c);
    if (lane == 0) sh.w0[w] = c;
    __syncthreads();
    if (t == 0) {
        long long z = 0;
        for (int i = 0; i < kMonoThreads / kWave; i++) z += sh.w0[i];
        *cnt_out = z;
    }
    __syncthreads();
}

// Whole sum by one workgroup (small n): *sum_out = seed + a[0] + ... +
// a[n-1] in that order (seed nullptr: 0); also *cnt_out = the sum of
// cnt_part[0..nparts) when cnt_out is given.
template <typename real>
__global__ __launch_bounds__(kMonoThreads) void k_mono_sum(long n, const real *__restrict__ a,
                                                           const real *__restrict__ seed,
                                                           int nparts,
                                                           const int *__restrict__ cnt_part,
                                                           real *__restrict__ sum_out,
                                                           long long *__restrict__ cnt_out) {
    __shared__ MonoShared sh;
    if (cnt_out) mono_count<real>(nparts, cnt_part, cnt_out, sh);
    if (threadIdx.x == 0) sh.exit_at = INT_MAX;
    __syncthreads();
    const real s = mono_range(a, 0, n, seed ? *seed : real(0), sh);
    if (threadIdx.x == 0) *sum_out = s;
}

// ---- large n: the tiles are summarised in parallel on predicted binades,
// one workgroup then chains the summaries and scans term by term only the
// tiles where the sum leaves its binade or the prediction missed.
//
// Every kernel below runs gridDim.y independent sums at once (sum y over
// a + y * astride, its scratch at y times the one-sum offsets): the
// iterate evolution needs two per iteration (sum (X_ - X)^2 and sum X^2).
// `halt` (may be null): a nonzero flag there makes every kernel return at
// once (a halted chunk of captured iterations).
//
// 1. per-tile sums in f64 (only to predict the binade of the running sum)
template <typename real>
__global__ __launch_bounds__(256) void k_mono_tile_sums(long n, const real *__restrict__ a,
                                                        long astride, double *__restrict__ tsum,
                                                        const int *__restrict__ halt) {
    constexpr long TILE = MonoTile<real>::TILE;
    __shared__ double red[kBlock / kWave];
    if (halt && *halt) return;
    a += blockIdx.y * astride;
    tsum += (long)blockIdx.y * gridDim.x;
    const long b = (long)blockIdx.x * TILE;
    double z = 0.0;
    for (long i = b + threadIdx.x; i < min(b + TILE, n); i += 256) z += (double)a[i];
    z = block_sum(z, red);
    if (threadIdx.x == 0) tsum[blockIdx.x] = z;
}

// 2. exclusive prefix -> predicted grid exponent at each tile start.  The
//    running sum starts at seed[y * sstride] (nullptr: 0) or, for the part of
//    a sum held by rank `prank` of a partition (chain_mono_sum), at the f64
//    totals of the ranks before it, dpre[q * nsum + y] for q < prank.
template <typename real>
__global__ __launch_bounds__(1024) void k_mono_predict(int ntiles, const double *__restrict__ tsum,
                                                       const real *__restrict__ seed, int sstride,
                                                       int *__restrict__ ebase,
                                                       const int *__restrict__ halt,
                                                       const double *__restrict__ dpre = nullptr,
                                                       int prank = 0) {
    __shared__ double wsum[1024 / kWave];
    __shared__ double carry;
    if (halt && *halt) return;
    const int y = blockIdx.y;
    tsum += (long)y * ntiles;
    ebase += (long)y * ntiles;
    const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
    if (t == 0) {
        double c = seed ? (double)seed[y * sstride] : 0.0;
        if (dpre)
            for (int q = 0; q < prank; q++) c += dpre[q * gridDim.y + y];
        carry = c;
    }
    __syncthreads();
    for (int c0 = 0; c0 < ntiles; c0 += 1024) {
        const int j = c0 + t;
        double v = j < ntiles ? tsum[j] : 0.0, inc = v;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const double p = __shfl_up(inc, o, kWave);
            if (lane >= o) inc += p;
        }
        if (lane == kWave - 1) wsum[w] = inc;
        __syncthreads();
        double pre = carry;
        for (int k = 0; k < w; k++) pre += wsum[k];
        if (j < ntiles) ebase[j] = grid_exp((real)(pre + inc - v));
        __syncthreads();
        if (t == 1023) carry = pre + inc;
        __syncthreads();
    }
}

// f64 total of each sum's tiles (fixed order) at tot[y] (rank totals of a
// partitioned sum, see chain_mono_sum)
static __global__ __launch_bounds__(256) void k_mono_total(int ntiles, const double *__restrict__ tsum,
                                                    double *__restrict__ tot,
                                                    const int *__restrict__ halt) {
    __shared__ double red[kBlock / kWave];
    if (halt && *halt) return;
    tsum += (long)blockIdx.y * ntiles;
    double z = 0.0;
    for (int j = threadIdx.x; j < ntiles; j += 256) z += tsum[j];
    z = block_sum(z, red);
    if (threadIdx.x == 0) tot[blockIdx.y] = z;
}

// 3. summaries (d0, d1) of tile blockIdx.x on the grids 2^(ebase - 1 + c),
//    c = 0 .. kMonoCand - 1, from one load of the tile
template <typename real>
__global__ __launch_bounds__(kMonoThreads) void k_mono_summaries(long n, const real *__restrict__ a,
                                                                 long astride,
                                                                 const int *__restrict__ ebase,
                                                                 long long *__restrict__ summ,
                                                                 const int *__restrict__ halt) {
    constexpr int J = MonoTile<real>::J, NW = kMonoThreads / kWave;
    __shared__ long long w0[kMonoCand][NW], w1[kMonoCand][NW];
    if (halt && *halt) return;
    const long nt = gridDim.x;
    a += blockIdx.y * astride;
    ebase += (long)blockIdx.y * nt;
    summ += (long)blockIdx.y * nt * 2 * kMonoCand;
    const int tile = blockIdx.x;
    const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
    real x[J];
    mono_load(x, a, n, (long)tile * MonoTile<real>::TILE, t);
    const int e0 = ebase[tile] - 1;
#pragma unroll
    for (int c = 0; c < kMonoCand; c++) {
        long long i0, i1;
        mono_run(x, e0 + c, i0, i1);
        mono_wave_scan<real>(i0, i1, lane);
        if (lane == kWave - 1) {
            w0[c][w] = i0;
            w1[c][w] = i1;
        }
    }
    __syncthreads();
    if (t < kMonoCand) {
        long long q0 = 0, q1 = 0;
        for (int k = 0; k < NW; k++) {
            long long b0 = w0[t][k], b1 = w1[t][k];
            compose<real>(q0, q1, b0, b1);
            q0 = b0;
            q1 = b1;
        }
        summ[2 * ((long)tile * kMonoCand + t)] = q0;
        summ[2 * ((long)tile * kMonoCand + t) + 1] = q1;
    }
}

// 4. one workgroup per sum: wave 0 chains the summaries of 64 tiles at a
//    time on the current binade; the first tile that would leave it (or has
//    no summary for it) is scanned term by term by the workgroup (mono_range).
template <typename real>
__global__ __launch_bounds__(kMonoThreads) void k_mono_walk(long n, const real *__restrict__ a,
                                                            long astride, int ntiles,
                                                            const int *__restrict__ ebase,
                                                            const long long *__restrict__ summ,
                                                            const real *__restrict__ seed,
                                                            int sstride, int nparts,
                                                            const int *__restrict__ cnt_part,
                                                            real *__restrict__ sum_out,
                                                            long long *__restrict__ cnt_out,
                                                            const int *__restrict__ halt) {
    constexpr long TILE = MonoTile<real>::TILE;
    constexpr long long TOP = 1ll << FpGrid<real>::p, CAP = TOP + 1;
    __shared__ MonoShared sh;
    if (halt && *halt) return;
    a += blockIdx.y * astride;
    ebase += (long)blockIdx.y * ntiles;
    summ += (long)blockIdx.y * ntiles * 2 * kMonoCand;
    sum_out += blockIdx.y;
    const int t = threadIdx.x, lane = t & (kWave - 1);
    if (cnt_out && blockIdx.y == 0) mono_count<real>(nparts, cnt_part, cnt_out, sh);
    if (t == 0) sh.exit_at = INT_MAX;
    __syncthreads();
    real s = seed ? seed[blockIdx.y * sstride] : real(0);
    int j = 0;
    while (j < ntiles && s < Lim<real>::huge) {
        const int ue = grid_exp(s);
        long long S = (long long)ldexp(s, -ue);
        for (;;) {  // whole tiles on this binade
            if (t < kWave) {
                const int jj = j + lane;
                const int c = jj < ntiles ? ue - ebase[jj] + 1 : -1;
                long long i0 = CAP, i1 = CAP;  // no summary: stops the chain here
                if (c >= 0 && c < kMonoCand) {
                    i0 = summ[2 * ((long)jj * kMonoCand + c)];
                    i1 = summ[2 * ((long)jj * kMonoCand + c) + 1];
                }
                mono_wave_scan<real>(i0, i1, lane);
                const long long after = sat_add<real>(S, (S & 1) ? i1 : i0);
                const unsigned long long stop = __ballot(after >= TOP);
                const int k = stop ? __ffsll(stop) - 1 : kWave;
                if (lane == k - 1) sh.S = after;
                if (t == 0) {
                    sh.k = k;
                    if (k == 0) sh.S = S;
                }
            }
            __syncthreads();
            const int k = sh.k;
            S = sh.S;
            __syncthreads();
            j += k;
            if (k < kWave || j >= ntiles) break;
        }
        s = ldexp((real)S, ue);
        if (j >= ntiles) break;
        // tile j leaves the binade (or was not predicted): term by term
        s = mono_range(a, (long)j * TILE, min(n, (long)(j + 1) * TILE), s, sh);
        j++;
    }
    if (t == 0) *sum_out = s;
}

// nsum sums of n terms each, sum y at a + y * astride (device), seed
// (device, may be nullptr; the same for every sum) -> out[y] (device);
// cnt_out (may be nullptr) receives the sum of cnt_part[0..nparts).
// ws: scratch of mono_ws_bytes(n, nsum) bytes.  halt: see above.
template <typename real>
inline size_t mono_ws_bytes(long n, int nsum = 1) {
    const long nt = (n + MonoTile<real>::TILE - 1) / MonoTile<real>::TILE;
    return (size_t)nsum * nt * (sizeof(double) + sizeof(int) + 2 * kMonoCand * sizeof(long long)) +
           64;
}
template <typename real>
void mono_sum(long n, const real *a, const real *seed, int nparts, const int *cnt_part, real *out,
              long long *cnt_out, void *ws, hipStream_t s, int nsum = 1, long astride = 0,
              const int *halt = nullptr) {
    constexpr long TILE = MonoTile<real>::TILE;
    const long nt = (n + TILE - 1) / TILE;
    if (nt <= 4 && nsum == 1 && !halt) {
        k_mono_sum<real><<<1, kMonoThreads, 0, s>>>(n, a, seed, nparts, cnt_part, out, cnt_out);
        return;
    }
    long long *summ = static_cast<long long *>(ws);
    double *tsum = reinterpret_cast<double *>(summ + 2 * kMonoCand * nt * nsum);
    int *ebase = reinterpret_cast<int *>(tsum + nt * nsum);
    const dim3 gt((unsigned)nt, (unsigned)nsum), g1(1, (unsigned)nsum);
    k_mono_tile_sums<real><<<gt, 256, 0, s>>>(n, a, astride, tsum, halt);
    k_mono_predict<real><<<g1, 1024, 0, s>>>((int)nt, tsum, seed, 0, ebase, halt);
    k_mono_summaries<real><<<gt, kMonoThreads, 0, s>>>(n, a, astride, ebase, summ, halt);
    k_mono_walk<real><<<g1, kMonoThreads, 0, s>>>(n, a, astride, (int)nt, ebase, summ, seed, 0,
                                                  nparts, cnt_part, out, cnt_out, halt);
}

// The same sum by one lane (PFDR_SEQSUM=lane, and the A/B tests): all lanes
// stage chunks in LDS (double buffered), lane 0 adds them in order.  One
// dependent add per term (~3.4 ns), 34 ms for 10M terms.
template <typename real>
__global__ __launch_bounds__(256) void k_seq_sum(long V, const real *__restrict__ absval,
                                                 const real *__restrict__ seed,
                                                 int nparts, const int *__restrict__ cnt_part,
                                                 real *__restrict__ sum_out,
                                                 long long *__restrict__ cnt_out) {
    constexpr int CH = 4096;
    __shared__ alignas(16) real buf[2][CH];
    __shared__ long long red[kBlock / kWave];
    long long cnt = 0;
    for (int i = threadIdx.x; i < nparts; i += kBlock) cnt += cnt_part[i];
    cnt = block_sum(cnt, red);
    real s = seed ? *seed : real(0);
    int cur = 0;
    for (long j = threadIdx.x; j < min((long)CH, (long)V); j += kBlock) buf[0][j] = absval[j];
    __syncthreads();
    for (long c0 = 0; c0 < V; c0 += CH) {
        const long n = min((long)CH, (long)V - c0);
        const long nxt = c0 + CH;
        if (threadIdx.x == 0) {
            s = ordered_add(s, buf[cur], (int)n);
        } else if (threadIdx.x >= kWave && nxt < V) {
            // waves 1-3 stage the next chunk, 16 loads in flight per lane
            constexpr int B = 16, NL = kBlock - kWave;
            const int m = (int)min((long)CH, (long)V - nxt);
            for (int j0 = threadIdx.x - kWave; j0 < m; j0 += B * NL) {
                real x[B];
#pragma unroll
                for (int u = 0; u < B; u++) x[u] = absval[nxt + min(j0 + u * NL, m - 1)];
#pragma unroll
                for (int u = 0; u < B; u++)
                    if (j0 + u * NL < m) buf[cur ^ 1][j0 + u * NL] = x[u];
            }
        }
        __syncthreads();
        cur ^= 1;
    }
    if (threadIdx.x == 0) {
        *sum_out = s;
        *cnt_out = cnt;
    }
}

}  // namespace pfdr
