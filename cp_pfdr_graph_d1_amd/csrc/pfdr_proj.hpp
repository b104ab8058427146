// Wave-parallel metric simplex projection, bit-exact with the reference's
// sequential active-set sweep (src/proj_simplex_metric.cpp:41-80).
//
// The reference walks the D coordinates of a column in order, keeping a
// running threshold la and metric sum s that change only where a coordinate
// enters (first pass, :48-57) or leaves (later passes, :60-72) the active
// set.  Between two such events every coordinate is compared with the SAME
// threshold, so the next event is simply the first coordinate, after the
// previous one, that satisfies the test against the current threshold: a
// ballot over the lanes that hold the next coordinates finds it, its (x, m)
// are broadcast, and every lane of the column applies the reference's update
// (s += m; la += m (x - la) / s, or s -= m; la += m (la - x) / s) to the same
// operands, so la and s carry the reference's rounding exactly.  The walk
// costs one ballot per event instead of one step per coordinate.
//
// A column is held by a SEGMENT of G lanes (G = 4 .. 64; 64 / G columns per
// wave when D <= 32) with coordinate d = j G + t at lane t of the segment,
// either in J registers per lane (D <= 64 J) or, for any D, in memory (one
// wave per column, 64 coordinates per chunk, the active flags as one byte per
// coordinate in scratch: the reference's own I[] of alloca(D), :38).
#pragma once

#include "pfdr_dev.hpp"

namespace pfdr {

template <typename T>
__device__ __forceinline__ T lane_read(T v, int l) {  // l wave-uniform
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
    } else {
        const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
        const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
        return __builtin_bit_cast(T, ((unsigned long long)hi << 32) | lo);
    }
}

// G lanes of a wave holding one column; lane t = sl of the segment at `base`
template <int G>
struct Seg {
    static_assert(G >= 2 && G <= 64 && (G & (G - 1)) == 0, "segment of 2..64 lanes");
    int sl, base;
    __device__ __forceinline__ Seg() {
        const int lane = (int)(threadIdx.x & (kWave - 1));
        sl = lane & (G - 1);
        base = lane - sl;
    }
    // the segment's lanes whose predicate holds (bit t = lane t of the segment)
    __device__ __forceinline__ unsigned long long bits(bool p) const {
        const unsigned long long b = __ballot(p);
        if constexpr (G == 64) return b;
        else return (b >> base) & ((1ull << G) - 1);
    }
    // value of lane l of this segment; executed by every lane of the wave
    template <typename T>
    __device__ __forceinline__ T bcast(T v, int l) const {
        if constexpr (G == 64) return lane_read(v, l);
        else return __shfl(v, base + l, kWave);
    }
    static __device__ __forceinline__ bool any(bool p) {
        if constexpr (G == 64) return p;  // segment-uniform = wave-uniform
        else return __ballot(p) != 0ull;
    }
};

__device__ __forceinline__ unsigned long long from_lane(int pos) {
    return pos >= 64 ? 0ull : (~0ull << pos);
}

// First pass over one chunk of G coordinates (ref :48-57): x already divided
// by its metric; coordinates before segment lane `pos` are skipped (pos = 1
// for the chunk holding d = 0).  Returns whether this lane's coordinate
// entered the active set.
template <typename real, int G>
__device__ __forceinline__ bool chunk_enter(const Seg<G> &sg, real x, real m, bool valid, int pos,
                                            real &la, real &s) {
    bool act = false;
    for (;;) {
        const unsigned long long c = sg.bits(valid && x > la) & from_lane(pos);
        if (!Seg<G>::any(c != 0ull)) break;
        const int l = c ? __ffsll((long long)c) - 1 : 0;
        const real xd = sg.bcast(x, l), md = sg.bcast(m, l);
        if (c) {
            if (sg.sl == l) act = true;
            s += md;
            la += md * (xd - la) / s;
            pos = l + 1;
        }
    }
    return act;
}

// One later pass over a chunk (ref :62-71): active coordinates below the
// threshold leave, in order.  Returns whether any left (segment-uniform).
template <typename real, int G>
__device__ __forceinline__ bool chunk_leave(const Seg<G> &sg, real x, real m, bool &act, real &la,
                                            real &s) {
    bool changed = false;
    int pos = 0;
    for (;;) {
        const unsigned long long c = sg.bits(act && x < la) & from_lane(pos);
        if (!Seg<G>::any(c != 0ull)) break;
        const int l = c ? __ffsll((long long)c) - 1 : 0;
        const real xd = sg.bcast(x, l), md = sg.bcast(m, l);
        if (c) {
            if (sg.sl == l) act = false;
            s -= md;
            la += md * (la - xd) / s;
            pos = l + 1;
            changed = true;
        }
    }
    return changed;
}

// Projection of one column held in registers: coordinate j G + sl in x[j],
// its metric in m[j] (lanes past D hold anything); a = the target sum.
// Every lane of the wave calls it (segments past the last column with D = 0).
template <typename real, int G, int J>
__device__ __forceinline__ void proj_segment(const Seg<G> &sg, real (&x)[J], const real (&m)[J],
                                             int D, real a) {
    // ref :43-46 (the threshold from the raw first coordinate)
    const real x0 = sg.bcast(x[0], 0), m0 = sg.bcast(m[0], 0);
    real la = (x0 - a) / m0;
    real s = m0;
    bool valid[J];
    unsigned act = 0u;
#pragma unroll
    for (int j = 0; j < J; j++) {
        valid[j] = j * G + sg.sl < D;
        if (valid[j]) x[j] = x[j] / m[j];
    }
#pragma unroll
    for (int j = 0; j < J; j++)
        if (chunk_enter<real, G>(sg, x[j], m[j], valid[j], j == 0 ? 1 : 0, la, s)) act |= 1u << j;
    if (sg.sl == 0 && D > 0) act |= 1u;  // I[0] = TRUE
    bool more = true;
    while (Seg<G>::any(more)) {  // segments already stable find nothing again
        bool ch = false;
#pragma unroll
        for (int j = 0; j < J; j++) {
            bool aj = (act >> j) & 1u;
            if (chunk_leave<real, G>(sg, x[j], m[j], aj, la, s)) {
                ch = true;
                act = aj ? (act | (1u << j)) : (act & ~(1u << j));
            }
        }
        more = ch;
    }
#pragma unroll
    for (int j = 0; j < J; j++)  // ref :74-80
        if (valid[j]) x[j] = ((act >> j) & 1u) ? (x[j] - la) * m[j] : real(0);
}

// Projection of one column in memory (any D), one whole wave: x in place,
// m its metric, I one byte per coordinate.  Lane t only ever touches the
// coordinates d = t mod 64 of x and I (own writes read back in program
// order); x[0] reaches the other lanes by a register broadcast.  Every lane
// of the wave calls it.
template <typename real>
__device__ void proj_wave_mem(real *x, const real *m, int D, real a, unsigned char *I) {
    const Seg<64> sg;
    const int nch = (D + 63) >> 6;
    const real m0 = m[0];
    // x[0] through lane 0 (the caller may have just written it from lane 0)
    const real x0 = lane_read(sg.sl == 0 ? x[0] : real(0), 0);
    real la = (x0 - a) / m0;
    real s = m0;
    for (int c = 0; c < nch; c++) {
        const int d = (c << 6) + sg.sl;
        const bool valid = d < D;
        real xd = real(0), md = real(1);
        if (valid) {
            md = m[d];
            xd = x[d] / md;
            x[d] = xd;
        }
        bool act = chunk_enter<real, 64>(sg, xd, md, valid, c == 0 ? 1 : 0, la, s);
        if (d == 0) act = true;
        if (valid) I[d] = act ? 1 : 0;
    }
    bool more = true;
    while (more) {
        more = false;
        for (int c = 0; c < nch; c++) {
            const int d = (c << 6) + sg.sl;
            const bool valid = d < D;
            real xd = real(0), md = real(1);
            bool act = false;
            if (valid) {
                xd = x[d];
                md = m[d];
                act = I[d] != 0;
            }
            if (chunk_leave<real, 64>(sg, xd, md, act, la, s)) {
                more = true;
                if (valid) I[d] = act ? 1 : 0;
            }
        }
    }
    for (int c = 0; c < nch; c++) {
        const int d = (c << 6) + sg.sl;
        if (d < D) x[d] = I[d] ? (x[d] - la) * m[d] : real(0);
    }
}

// First index of the largest coordinate, as the reference's scan
// `if (x[k] > mx)` from mx = x[0] (src/PFDR_graph_loss_d1_simplex.cpp:447-466,
// :656-676): NaN never wins, equal values keep the smaller index, and a NaN
// x[0] keeps index 0.  (v, i): this lane's candidate (i = INT_MAX: none).
template <typename real>
__device__ __forceinline__ void argmax_take(real x, int k, real &v, int &i) {
    if (x == x && (i == 0x7fffffff || x > v)) { v = x; i = k; }
}
template <typename real>
__device__ __forceinline__ int wave_argmax(real v, int i, bool x0_nan) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const real ov = __shfl_xor(v, o, kWave);
        const int oi = __shfl_xor(i, o, kWave);
        if (oi != 0x7fffffff && (i == 0x7fffffff || ov > v || (ov == v && oi < i))) { v = ov; i = oi; }
    }
    return (x0_nan || i == 0x7fffffff) ? 0 : i;
}

}  // namespace pfdr
