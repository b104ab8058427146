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
#include <type_traits>

#include "pfdr_dev.hpp"

namespace pfdr {

// Phase timers of the walk for tools/monoprof.hip (compiled out otherwise):
// lane 0 of sum 0 charges the wall-clock time since the previous tick to
// phase k and counts the phase.
#ifdef PFDR_MONO_PROFILE
__device__ unsigned long long g_mono_prof[32];
struct MonoProf {
    unsigned long long t[16], n[16], last;
    __device__ MonoProf() : last(wall_clock64()) {
        for (int k = 0; k < 16; k++) t[k] = n[k] = 0;
    }
    __device__ void tick(int k) {
        const unsigned long long now = wall_clock64();
        t[k] += now - last;
        n[k]++;
        last = now;
    }
    __device__ void out() const {
        if (threadIdx.x == 0 && blockIdx.y == 0)
            for (int k = 0; k < 16; k++) {
                g_mono_prof[k] = t[k];
                g_mono_prof[16 + k] = n[k];
            }
    }
};
#else
struct MonoProf {
    __device__ void tick(int) {}
    __device__ void out() const {}
};
#endif

template <typename real> struct FpGrid;
template <> struct FpGrid<float> {
    static constexpr int p = 24, emin = -126;
    static constexpr float min_normal = 1.17549435082228750797e-38f;
};
template <> struct FpGrid<double> {
    static constexpr int p = 53, emin = -1022;
    static constexpr double min_normal = 2.2250738585072013831e-308;
};

// integer counts on the grid of a binade: below 2^p + 1 per tile after
// saturation, so 32 bits hold them for f32 (half the ALU work of 64)
template <typename real>
using mcnt = typename std::conditional<sizeof(real) == 4, int, long long>::type;

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
__device__ __forceinline__ void grid_term(real a, int ue, mcnt<real> &fl, int &cls) {
    constexpr real top = real(1ll << FpGrid<real>::p);
    const real q = ldexp(a, -ue);  // exact (a scaled by a power of two), or
    if (!(q < top)) {              // underflowed far below one half
        fl = 0;
        cls = 3;
        return;
    }
    const real f = floor(q), r = q - f;
    fl = (mcnt<real>)f;
    cls = r < real(0.5) ? 0 : (r > real(0.5) ? 1 : 2);
}

template <typename real>
__device__ __forceinline__ mcnt<real> grid_inc(mcnt<real> fl, int cls, mcnt<real> parity) {
    constexpr mcnt<real> cap = (1ll << FpGrid<real>::p) + 1;
    return cls == 3 ? cap : fl + (cls == 2 ? ((parity + fl) & 1) : cls);
}

// (d0, d1) summaries; increments saturate at 2^p + 1 (past that point the
// binade has been left and everything after the exit is discarded)
template <typename real>
__device__ __forceinline__ mcnt<real> sat_add(mcnt<real> a, mcnt<real> b) {
    constexpr mcnt<real> cap = (1ll << FpGrid<real>::p) + 1;
    const mcnt<real> x = a + b;
    return x > cap ? cap : x;
}
template <typename real>
__device__ __forceinline__ void compose(mcnt<real> a0, mcnt<real> a1, mcnt<real> &b0,
                                        mcnt<real> &b1) {
    // (A then B) for start parity 0 and 1; result in (b0, b1)
    const mcnt<real> n0 = sat_add<real>(a0, (a0 & 1) ? b1 : b0);
    const mcnt<real> n1 = sat_add<real>(a1, ((1 + a1) & 1) ? b1 : b0);
    b0 = n0;
    b1 = n1;
}

constexpr int kMonoThreads = 512;
constexpr int kMonoCand = 3;  // binades summarised per tile (predicted, one below, one above)

template <typename real>
struct MonoTile {
    static constexpr int J = 64 / sizeof(real);             // terms per lane
    static constexpr long TILE = (long)kMonoThreads * J;     // terms per tile
    static constexpr int SUB = kWave * J;                   // terms per sub-tile (a wave's)
    static constexpr int NSUB = kMonoThreads / kWave;       // sub-tiles per tile
    static constexpr int FJ = SUB / kMonoThreads;           // terms per lane in a fine scan
};

constexpr int kMonoSerial = 256;     // terms added by one lane after each exit (mono_range)
constexpr int kMonoSerialFine = kWave;  // the same in the walk (fine_scan, serial_wave)

// Shared state of a workgroup walking terms one tile at a time.  The tile
// held in registers is also kept in LDS: the terms after an exit are added
// by one lane from there, and the scan resumes on the registers (one global
// load per tile, however many exits it holds).
struct MonoShared {
    static constexpr int NW = kMonoThreads / kWave;
    alignas(16) char tile[kMonoThreads * 64];
    long long w0[NW], w1[NW];                // wave totals (mono_range)
    long long fw0[2][NW], fw1[2][NW];        // wave totals of fine_scan, by parity
    long long cw0[NW], cw1[NW], lastS[NW];   // the walk's chain steps
    long long subs[2 * kMonoCand * NW];      // the staged tile's sub-tile summaries
    long long cexl[2];                       // fine_scan: the count before its exit, by parity
    int cnt[NW];
    int exit_at;
    int fexit[2];                            // fine_scan's exit, by parity
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
template <typename real, int N = MonoTile<real>::J>
__device__ __forceinline__ void mono_run(const real *x, int ue, mcnt<real> &d0, mcnt<real> &d1) {
    d0 = d1 = 0;
#pragma unroll
    for (int j = 0; j < N; j++) {
        mcnt<real> fl;
        int cls;
        grid_term(x[j], ue, fl, cls);
        d0 = sat_add<real>(d0, grid_inc<real>(fl, cls, d0));
        d1 = sat_add<real>(d1, grid_inc<real>(fl, cls, 1 + d1));
    }
}

// DPP moves (gfx9 encodings; a lane whose source is outside the pattern
// reads 0, the identity of compose): row_shr:n (lane i <- i - n within its
// row of 16), row_bcast:15 / :31 (the previous row's last lane to the rows
// of ROWS), wave_shr:1 (lane i <- i - 1)
constexpr int kDppRowShr = 0x110, kDppWaveShr1 = 0x138, kDppBcast15 = 0x142, kDppBcast31 = 0x143;
template <int CTRL, int ROWS, typename T>
__device__ __forceinline__ T dpp_mov(T v) {
    if constexpr (sizeof(T) == 4) {
        return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xf, false);
    } else {
        const int lo = __builtin_amdgcn_update_dpp(0, (int)(v & 0xffffffff), CTRL, ROWS, 0xf, false);
        const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), CTRL, ROWS, 0xf, false);
        return (T)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
    }
}
template <typename real, int CTRL, int ROWS>
__device__ __forceinline__ void scan_step(mcnt<real> &i0, mcnt<real> &i1) {
    mcnt<real> p0 = dpp_mov<CTRL, ROWS>(i0), p1 = dpp_mov<CTRL, ROWS>(i1);
    compose<real>(p0, p1, i0, i1);
}

// inclusive scan of summaries over the wave (earlier lanes first): rows of
// 16 by row_shr 1, 2, 4, 8, then the rows joined by the two broadcasts
template <typename real>
__device__ __forceinline__ void mono_wave_scan(mcnt<real> &i0, mcnt<real> &i1) {
    scan_step<real, kDppRowShr + 1, 0xf>(i0, i1);
    scan_step<real, kDppRowShr + 2, 0xf>(i0, i1);
    scan_step<real, kDppRowShr + 4, 0xf>(i0, i1);
    scan_step<real, kDppRowShr + 8, 0xf>(i0, i1);
    scan_step<real, kDppBcast15, 0xa>(i0, i1);
    scan_step<real, kDppBcast31, 0xc>(i0, i1);
}
// lane k's count (k uniform)
template <typename T>
__device__ __forceinline__ T read_lane(T v, int k) {
    if constexpr (sizeof(T) == 4) {
        return __builtin_amdgcn_readlane(v, k);
    } else {
        const unsigned lo = __builtin_amdgcn_readlane((int)(v & 0xffffffff), k);
        const unsigned hi = __builtin_amdgcn_readlane((int)(v >> 32), k);
        return (T)(((unsigned long long)hi << 32) | lo);
    }
}
// the summary of the lanes before this one (lane 0: the identity)
template <typename real>
__device__ __forceinline__ void mono_wave_excl(mcnt<real> i0, mcnt<real> i1, mcnt<real> &e0,
                                               mcnt<real> &e1) {
    e0 = dpp_mov<kDppWaveShr1, 0xf>(i0);
    e1 = dpp_mov<kDppWaveShr1, 0xf>(i1);
}

// s + q[0] + ... + q[m-1] for m <= kWave, every lane of the wave alike: one
// LDS read per lane, then the terms in order from the lanes (fully unrolled:
// the zeros past m add nothing to a sum of nonnegative terms)
template <typename real>
__device__ __forceinline__ real serial_wave(real s, const real *q, int m) {
    const int lane = threadIdx.x & (kWave - 1);
    const real v = lane < m ? q[lane] : real(0);
#pragma unroll
    for (int i = 0; i < kWave; i++) {
        if constexpr (sizeof(real) == 4) {
            s += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), i));
        } else {
            const long long b = __double_as_longlong(v);
            const unsigned lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), i);
            const unsigned hi = __builtin_amdgcn_readlane((int)(b >> 32), i);
            s += __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
        }
    }
    return s;
}

// s + q[0] + ... + q[m-1] by one lane from LDS (q of any alignment)
template <typename real>
__device__ __forceinline__ real serial_add(real s, const real *q, int m) {
    while (m > 0 && (reinterpret_cast<uintptr_t>(q) & 15)) {
        s += *q++;
        m--;
    }
    return ordered_add(s, q, m);
}

// s + a[lo] + ... + a[hi-1] by the whole workgroup, term by term semantics:
// scans tile after tile on the binade of s, adds the first term that leaves
// it with one floating-point addition, and resumes after that term.
template <typename real>
__device__ real mono_range(const real *__restrict__ a, long lo, long hi, real s, MonoShared &sh) {
    constexpr int J = MonoTile<real>::J, W = Vec<real>::kPer16B;
    constexpr long TILE = MonoTile<real>::TILE;
    constexpr mcnt<real> TOP = 1ll << FpGrid<real>::p;
    using P = Pk<real, W>;
    const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
    real *tb = reinterpret_cast<real *>(sh.tile);
    // tiles are aligned to TILE (16-byte loads); terms before `start` are
    // masked to zero, which adds nothing
    long start = lo, xb = -1;  // xb: the tile held in x and in sh.tile
    real x[J], nx[J];
    bool have = false;  // nx holds the tile at xb + TILE
    while (start < hi && s < Lim<real>::huge) {
        const int ue = grid_exp(s);
        mcnt<real> S = (mcnt<real>)ldexp(s, -ue);  // s / u, an integer below 2^p
        bool left = false;
        for (long base = start / TILE * TILE; base < hi; base += TILE) {
            if (base != xb) {
                if (have && base == xb + TILE) {
#pragma unroll
                    for (int j = 0; j < J; j++) x[j] = nx[j];
                } else {
                    mono_load(x, a, hi, base, t);
                }
                const bool more = base + TILE < hi;
                if (more) mono_load(nx, a, hi, base + TILE, t);  // in flight during the scan
                have = more;
                xb = base;
#pragma unroll
                for (int v = 0; v < J / W; v++) {
                    P pk;
#pragma unroll
                    for (int k = 0; k < W; k++) pk.v[k] = x[v * W + k];
                    *reinterpret_cast<P *>(tb + t * J + v * W) = pk;
                }
            }
            if (start > base) {
#pragma unroll
                for (int j = 0; j < J; j++)
                    if (base + (long)t * J + j < start) x[j] = real(0);
            }
            mcnt<real> r0, r1;
            mono_run(x, ue, r0, r1);
            mcnt<real> i0 = r0, i1 = r1;
            mono_wave_scan<real>(i0, i1);
            if (lane == kWave - 1) {
                sh.w0[w] = i0;
                sh.w1[w] = i1;
            }
            mcnt<real> e0, e1;
            mono_wave_excl<real>(i0, i1, e0, e1);
            __syncthreads();
            // prefix of the earlier waves (in order), then this lane's start
            mcnt<real> q0 = 0, q1 = 0;
            for (int k = 0; k < w; k++) {
                mcnt<real> b0 = sh.w0[k], b1 = sh.w1[k];
                compose<real>(q0, q1, b0, b1);
                q0 = b0;
                q1 = b1;
            }
            compose<real>(q0, q1, e0, e1);
            // this lane's exact starting count; only a lane whose run ends
            // outside the binade walks its terms to find the exit
            mcnt<real> cur = sat_add<real>(S, (S & 1) ? e1 : e0), cex = 0;
            const mcnt<real> end = sat_add<real>(cur, (cur & 1) ? r1 : r0);
            int mine = INT_MAX;
            real xex = real(0);
            if (cur < TOP && end >= TOP) {  // the one lane that leaves the binade
#pragma unroll
                for (int j = 0; j < J; j++) {
                    mcnt<real> fl;
                    int cls;
                    grid_term(x[j], ue, fl, cls);  // recomputed: fewer live registers
                    const mcnt<real> inc = grid_inc<real>(fl, cls, cur);
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
                if (t == kMonoThreads - 1) sh.S = cur;
                __syncthreads();
                S = sh.S;
                __syncthreads();
                continue;
            }
            // the earliest exit term: one ordinary addition (s = cex * u
            // exactly); exits cluster where the sum is young (it doubles
            // every few terms): the next kMonoSerial terms of the tile are
            // added by the same lane, from LDS
            start = base + ex + 1;
            if (mine == ex) {
                const int m = (int)min((long)kMonoSerial, min(hi, base + TILE) - start);
                sh.sd = (double)serial_add(ldexp((real)cex, ue) + xex, tb + ex + 1, m);
            }
            __syncthreads();
            s = (real)sh.sd;
            if (t == 0) sh.exit_at = INT_MAX;  // every lane has read it
            start += (int)min((long)kMonoSerial, min(hi, base + TILE) - start);
            left = true;
            break;
        }
        if (!left) {
            s = ldexp((real)S, ue);
            break;
        }
    }
    return s;
}

// lane t's J terms x into the LDS copy of the tile
template <typename real>
__device__ __forceinline__ void mono_stage(real *tb, const real *x, int t) {
    constexpr int J = MonoTile<real>::J, W = Vec<real>::kPer16B;
    using P = Pk<real, W>;
#pragma unroll
    for (int v = 0; v < J / W; v++) {
        P pk;
#pragma unroll
        for (int k = 0; k < W; k++) pk.v[k] = x[v * W + k];
        *reinterpret_cast<P *>(tb + t * J + v * W) = pk;
    }
}

// One pass of the workgroup over sub-tile `sub` of the tile staged in LDS
// (tb; positions relative to the tile, those before p masked, len terms in
// the tile) on the grid 2^ue from the count S.  No exit: S <- the count at
// the sub-tile's end, returns -1.  Otherwise the first term that leaves the
// binade is added with one floating-point addition and the next
// min(kMonoSerialFine, len - exit - 1) terms one by one (every lane alike,
// from LDS): returns the exit position, the running sum after those terms
// in s.  Every lane learns from the wave totals whether the sub-tile stays
// in the binade (the counts never decrease), so a pass without an exit
// costs one barrier; the LDS slots alternate with the parity `par` of the
// pass, so no barrier is needed to release them.
template <typename real>
__device__ int fine_scan(const real *tb, int sub, int p, int len, int ue, mcnt<real> &S, real &s,
                         MonoShared &sh, int &par, MonoProf &mp) {
    constexpr int FJ = MonoTile<real>::FJ, SUB = MonoTile<real>::SUB, NW = MonoShared::NW;
    constexpr mcnt<real> TOP = 1ll << FpGrid<real>::p;
    const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave, pr = par;
    par ^= 1;
    const int i0 = sub * SUB + t * FJ;
    real x[FJ];
#pragma unroll
    for (int j = 0; j < FJ; j++) x[j] = (i0 + j >= p) ? tb[i0 + j] : real(0);
    mcnt<real> r0, r1;
    mono_run<real, FJ>(x, ue, r0, r1);
    mcnt<real> c0 = r0, c1 = r1, e0, e1;
    mono_wave_scan<real>(c0, c1);
    if (lane == kWave - 1) {
        sh.fw0[pr][w] = c0;
        sh.fw1[pr][w] = c1;
    }
    mono_wave_excl<real>(c0, c1, e0, e1);
    mp.tick(5);
    __syncthreads();
    mp.tick(6);
    // the earlier waves' prefix and the sub-tile's total
    mcnt<real> v0[NW], v1[NW];
#pragma unroll
    for (int k = 0; k < NW; k++) {
        v0[k] = (mcnt<real>)sh.fw0[pr][k];
        v1[k] = (mcnt<real>)sh.fw1[pr][k];
    }
    mcnt<real> q0 = 0, q1 = 0, f0 = 0, f1 = 0;
#pragma unroll
    for (int k = 0; k < NW; k++) {
        if (k == w) {
            f0 = q0;
            f1 = q1;
        }
        mcnt<real> b0 = v0[k], b1 = v1[k];
        compose<real>(q0, q1, b0, b1);
        q0 = b0;
        q1 = b1;
    }
    const mcnt<real> tot = sat_add<real>(S, (S & 1) ? q1 : q0);
    mp.tick(7);
    if (tot < TOP) {
        S = tot;
        return -1;
    }
    compose<real>(f0, f1, e0, e1);
    mcnt<real> cur = sat_add<real>(S, (S & 1) ? e1 : e0);
    const mcnt<real> end = sat_add<real>(cur, (cur & 1) ? r1 : r0);
    // the counts never decrease: exactly one lane starts inside the binade
    // and ends outside it, and the exit is among its terms
    if (cur < TOP && end >= TOP) {
        int mine = INT_MAX;
        mcnt<real> cex = 0;
#pragma unroll
        for (int j = 0; j < FJ; j++) {
            mcnt<real> fl;
            int cls;
            grid_term(x[j], ue, fl, cls);
            const mcnt<real> inc = grid_inc<real>(fl, cls, cur);
            if (mine == INT_MAX && (cls == 3 || cur + inc >= TOP)) {
                mine = i0 + j;
                cex = cur;
            }
            cur = sat_add<real>(cur, inc);
        }
        sh.fexit[pr] = mine;
        sh.cexl[pr] = cex;
    }
    mp.tick(8);
    __syncthreads();
    mp.tick(9);
    const int ex = sh.fexit[pr];
    const real cex = (real)(mcnt<real>)sh.cexl[pr];
    s = serial_wave(ldexp(cex, ue) + tb[ex], tb + ex + 1, min(kMonoSerialFine, len - ex - 1));
    mp.tick(10);
    return ex;
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
//    totals of the ranks before it, dpre[q * nsum + y] for q < prank.  With
//    bpart, the tile sums are formed here from the block sums the producer
//    of the terms already has (bpart[nsum * b + y], kBlock terms per block b;
//    only a prediction, so their order and rounding do not matter) and step
//    1 is skipped.  One workgroup of kPredThreads per sum: small enough to be
//    dispatched between the sweeps' workgroups when it runs beside them.
constexpr int kPredThreads = 256;
template <typename real>
__global__ __launch_bounds__(kPredThreads) void k_mono_predict(
    int ntiles, const double *__restrict__ tsum, const real *__restrict__ seed, int sstride,
    int *__restrict__ ebase, const int *__restrict__ halt, const double *__restrict__ dpre = nullptr,
    int prank = 0, const real *__restrict__ bpart = nullptr, int nbpart = 0) {
    constexpr int BPT = MonoTile<real>::TILE / kBlock;
    __shared__ double wsum[kPredThreads / kWave];
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
    for (int c0 = 0; c0 < ntiles; c0 += kPredThreads) {
        const int j = c0 + t;
        double v = 0.0;
        if (j < ntiles && bpart) {
            const int b1 = min(nbpart, (j + 1) * BPT);
            for (int b = j * BPT; b < b1; b++) v += (double)bpart[(long)gridDim.y * b + y];
        } else if (j < ntiles) {
            v = tsum[j];
        }
        double inc = v;
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
        if (t == kPredThreads - 1) carry = pre + inc;
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
                                                                 long long *__restrict__ subs,
                                                                 const int *__restrict__ halt) {
    constexpr int J = MonoTile<real>::J, NW = kMonoThreads / kWave;
    __shared__ long long w0[kMonoCand][NW], w1[kMonoCand][NW];
    if (halt && *halt) return;
    const long nt = gridDim.x;
    a += blockIdx.y * astride;
    ebase += (long)blockIdx.y * nt;
    summ += (long)blockIdx.y * nt * 2 * kMonoCand;
    subs += (long)blockIdx.y * nt * 2 * kMonoCand * NW;
    const int tile = blockIdx.x;
    const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
    real x[J];
    mono_load(x, a, n, (long)tile * MonoTile<real>::TILE, t);
    const int e0 = ebase[tile] - 1;
#pragma unroll
    for (int c = 0; c < kMonoCand; c++) {
        mcnt<real> i0, i1;
        mono_run(x, e0 + c, i0, i1);
        mono_wave_scan<real>(i0, i1);
        if (lane == kWave - 1) {
            w0[c][w] = i0;
            w1[c][w] = i1;
            subs[2 * (((long)tile * kMonoCand + c) * NW + w)] = i0;  // sub-tile w
            subs[2 * (((long)tile * kMonoCand + c) * NW + w) + 1] = i1;
        }
    }
    __syncthreads();
    if (t < kMonoCand) {
        mcnt<real> q0 = 0, q1 = 0;
        for (int k = 0; k < NW; k++) {
            mcnt<real> b0 = w0[t][k], b1 = w1[t][k];
            compose<real>(q0, q1, b0, b1);
            q0 = b0;
            q1 = b1;
        }
        summ[2 * ((long)tile * kMonoCand + t)] = q0;
        summ[2 * ((long)tile * kMonoCand + t) + 1] = q1;
    }
}

// 4. one workgroup per sum: chains the summaries of kMonoThreads tiles at a
//    time on the current binade.  The first tile that would leave it (or has
//    no summary for it) is staged in LDS; its sub-tiles are chained on their
//    own summaries while the binade has one, and only the sub-tile that
//    leaves it is scanned term by term (fine_scan), 1/NSUB of the tile per
//    pass.
template <typename real>
__global__ __launch_bounds__(kMonoThreads) void k_mono_walk(long n, const real *__restrict__ a,
                                                            long astride, int ntiles,
                                                            const int *__restrict__ ebase,
                                                            const long long *__restrict__ summ,
                                                            const long long *__restrict__ subs,
                                                            const real *__restrict__ seed,
                                                            int sstride, int nparts,
                                                            const int *__restrict__ cnt_part,
                                                            real *__restrict__ sum_out,
                                                            long long *__restrict__ cnt_out,
                                                            const int *__restrict__ halt) {
    constexpr long TILE = MonoTile<real>::TILE;
    constexpr int J = MonoTile<real>::J, SUB = MonoTile<real>::SUB, NSUB = MonoTile<real>::NSUB;
    constexpr mcnt<real> TOP = 1ll << FpGrid<real>::p, CAP = TOP + 1;
    __shared__ MonoShared sh;
    if (halt && *halt) return;
    a += blockIdx.y * astride;
    ebase += (long)blockIdx.y * ntiles;
    summ += (long)blockIdx.y * ntiles * 2 * kMonoCand;
    subs += (long)blockIdx.y * ntiles * 2 * kMonoCand * NSUB;
    sum_out += blockIdx.y;
    real *tb = reinterpret_cast<real *>(sh.tile);
    const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
    MonoProf mp;
    if (cnt_out && blockIdx.y == 0) mono_count<real>(nparts, cnt_part, cnt_out, sh);
    __syncthreads();
    real s = seed ? seed[blockIdx.y * sstride] : real(0);
    int j = 0, par = 0;
    // the next chain step's tile (j + t): its predicted binade and its
    // summaries on every candidate, loaded ahead (during the previous
    // crossing tile's scans)
    int pe = 0;
    long long sc[2 * kMonoCand];
    auto fetch = [&](int base) {
        const int jj = base + t;
        if (jj < ntiles) {
            pe = ebase[jj];
#pragma unroll
            for (int q = 0; q < 2 * kMonoCand; q++) sc[q] = summ[2 * (long)jj * kMonoCand + q];
        }
    };
    fetch(0);
    while (j < ntiles && s < Lim<real>::huge) {
        const int ue = grid_exp(s);
        mcnt<real> S = (mcnt<real>)ldexp(s, -ue);
        for (;;) {  // whole tiles on this binade, kMonoThreads at a time
            const int c = j + t < ntiles ? ue - pe + 1 : -1;
            mcnt<real> i0 = CAP, i1 = CAP;  // no summary: stops the chain here
#pragma unroll
            for (int q = 0; q < kMonoCand; q++)
                if (c == q) {
                    i0 = (mcnt<real>)sc[2 * q];
                    i1 = (mcnt<real>)sc[2 * q + 1];
                }
            mono_wave_scan<real>(i0, i1);
            if (lane == kWave - 1) {
                sh.cw0[w] = i0;
                sh.cw1[w] = i1;
            }
            __syncthreads();
            mcnt<real> q0 = 0, q1 = 0;
#pragma unroll
            for (int k = 0; k < MonoShared::NW; k++) {
                mcnt<real> b0 = (mcnt<real>)sh.cw0[k], b1 = (mcnt<real>)sh.cw1[k];
                if (k < w) {
                    compose<real>(q0, q1, b0, b1);
                    q0 = b0;
                    q1 = b1;
                }
            }
            compose<real>(q0, q1, i0, i1);
            // the counts never decrease along the chain, so the tiles that
            // stay in the binade are a prefix: count them, keep the last
            const mcnt<real> after = sat_add<real>(S, (S & 1) ? i1 : i0);
            const int ng = __popcll(__ballot(after < TOP));
            if (lane == 0) sh.cnt[w] = ng;
            if (ng > 0 && lane == ng - 1) sh.lastS[w] = after;
            __syncthreads();
            int k = 0;
#pragma unroll
            for (int q = 0; q < MonoShared::NW; q++) k += sh.cnt[q];
            if (k > 0) S = (mcnt<real>)sh.lastS[(k - 1) / kWave];
            j += k;
            fetch(k < kMonoThreads ? j + 1 : j);  // after the crossing tile / the next step
            mp.tick(0);
            if (k < kMonoThreads || j >= ntiles) break;
        }
        s = ldexp((real)S, ue);
        if (j >= ntiles) break;
        // tile j leaves the binade (or was not predicted): staged in LDS with
        // its sub-tile summaries on every candidate binade
        {
            real x[J];
            mono_load(x, a, n, (long)j * TILE, t);
            if (t < 2 * kMonoCand * NSUB) sh.subs[t] = subs[2 * (long)j * kMonoCand * NSUB + t];
            mono_stage(tb, x, t);
        }
        const int len = (int)min(TILE, n - (long)j * TILE), eb = ebase[j];
        __syncthreads();
        mp.tick(1);
        int p = 0;
        while (p < len && s < Lim<real>::huge) {
            const int u2 = grid_exp(s), c = u2 - eb + 1;
            mcnt<real> S2 = (mcnt<real>)ldexp(s, -u2);
            if (p % SUB == 0 && c >= 0 && c < kMonoCand) {
                // whole sub-tiles on their summaries (every wave alike)
                const int sb = p / SUB;
                mcnt<real> i0 = CAP, i1 = CAP;
                if (lane < NSUB - sb) {
                    i0 = (mcnt<real>)sh.subs[2 * (c * NSUB + sb + lane)];
                    i1 = (mcnt<real>)sh.subs[2 * (c * NSUB + sb + lane) + 1];
                }
                mono_wave_scan<real>(i0, i1);
                const mcnt<real> after = sat_add<real>(S2, (S2 & 1) ? i1 : i0);
                const int k = __popcll(__ballot(after < TOP));
                mp.tick(2);
                if (k > 0) {
                    S2 = read_lane(after, k - 1);
                    s = ldexp((real)S2, u2);
                    p += k * SUB;
                    if (p >= len) break;
                }
            }
            real se = s;
            const int ex = fine_scan<real>(tb, p / SUB, p, len, u2, S2, se, sh, par, mp);
            mp.tick(3);
            if (ex < 0) {
                s = ldexp((real)S2, u2);
                p = (p / SUB + 1) * SUB;
            } else {
                s = se;
                p = ex + 1 + min(kMonoSerialFine, len - ex - 1);
            }
        }
        j++;
    }
    if (t == 0) *sum_out = s;
    mp.tick(4);
    mp.out();
}

// nsum sums of n terms each, sum y at a + y * astride (device), seed
// (device, may be nullptr; the same for every sum) -> out[y] (device);
// cnt_out (may be nullptr) receives the sum of cnt_part[0..nparts).
// ws: scratch of mono_ws_bytes(n, nsum) bytes.  halt: see above.
template <typename real>
inline size_t mono_ws_bytes(long n, int nsum = 1) {
    const long nt = (n + MonoTile<real>::TILE - 1) / MonoTile<real>::TILE;
    return (size_t)nsum * nt *
               (sizeof(double) + sizeof(int) +
                2 * kMonoCand * (1 + MonoTile<real>::NSUB) * sizeof(long long)) +
           64;
}
// the scratch's parts: tile and sub-tile summaries, f64 tile sums, binades
template <typename real>
struct MonoWs {
    long long *summ, *subs;
    double *tsum;
    int *ebase;
    MonoWs(void *ws, long nt, int nsum) {
        summ = static_cast<long long *>(ws);
        subs = summ + 2 * kMonoCand * nt * nsum;
        tsum = reinterpret_cast<double *>(subs + 2 * kMonoCand * MonoTile<real>::NSUB * nt * nsum);
        ebase = reinterpret_cast<int *>(tsum + nt * nsum);
    }
};
// bpart (may be nullptr): block sums of the terms, see k_mono_predict
template <typename real>
void mono_sum(long n, const real *a, const real *seed, int nparts, const int *cnt_part, real *out,
              long long *cnt_out, void *ws, hipStream_t s, int nsum = 1, long astride = 0,
              const int *halt = nullptr, const real *bpart = nullptr, int nbpart = 0) {
    constexpr long TILE = MonoTile<real>::TILE;
    const long nt = (n + TILE - 1) / TILE;
    if (nt <= 4 && nsum == 1 && !halt) {
        k_mono_sum<real><<<1, kMonoThreads, 0, s>>>(n, a, seed, nparts, cnt_part, out, cnt_out);
        return;
    }
    const MonoWs<real> w(ws, nt, nsum);
    const dim3 gt((unsigned)nt, (unsigned)nsum), g1(1, (unsigned)nsum);
    if (!bpart) k_mono_tile_sums<real><<<gt, 256, 0, s>>>(n, a, astride, w.tsum, halt);
    k_mono_predict<real><<<g1, kPredThreads, 0, s>>>((int)nt, w.tsum, seed, 0, w.ebase, halt,
                                                     nullptr, 0, bpart, nbpart);
    k_mono_summaries<real><<<gt, kMonoThreads, 0, s>>>(n, a, astride, w.ebase, w.summ, w.subs,
                                                       halt);
    k_mono_walk<real><<<g1, kMonoThreads, 0, s>>>(n, a, astride, (int)nt, w.ebase, w.summ, w.subs,
                                                  seed, 0, nparts, cnt_part, out, cnt_out, halt);
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
