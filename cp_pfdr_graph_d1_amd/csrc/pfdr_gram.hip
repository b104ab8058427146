// Gram matrices on the matrix cores and the operator norm of a dense matrix
// (the CP reduced-problem builder).
//
// Reference: src/operator_norm_matrix.cpp:87-212 — the squared operator norm
// ||A||^2 by the power method on A^tA (or AA^t), from nbInit random starts,
// after an optional explicit symmetrisation (:112-165).  CP calls it on every
// reduced problem with a dense A (src/CP_PFDR_graph_quadratic_d1_l1.cpp:792,
// :822), and forms the reduced Gram rA^t rA the same way (:688-702).
//
// MI355X design:
//   * k_gram: G = L^t R for L = R = A (one matrix, two tiles), exact-f32
//     MFMA (v_mfma_f32_32x32x2_f32) or f64 MFMA (v_mfma_f64_16x16x4_f64);
//     256-thread blocks of 4 waves, a 2x2 grid of MFMA tiles per wave, K
//     staged through LDS in BK slices; only the upper block triangle is
//     computed, the epilogue mirrors it; the contraction is split into
//     chunks (deterministic second pass) so that a 1024-wide Gram over two
//     million columns still fills the 256 CUs.
//   * f32 on the bf16 matrix cores (k_gram_b): each element split exactly
//     into three bf16 pieces, six piece products per f32 product, f32
//     accumulation -- f32 accuracy at up to 2.7x the f32 MFMA rate per flop
//     (PFDR_GRAM_SPLIT=0: the exact-f32 tile k_gram_v).
//   * the power method runs all starts at once: X is S-by-B, one apply is
//     a skinny product (HBM-bound: each pass streams the matrix once for
//     all B starts); each start keeps the reference's stopping rule
//     (a - b)/b < nTol and result b.
//   * symmetrise when the Gram's matrix-core time beats itMax * nbInit
//     streaming passes over A on this GPU (the reference's rule counts CPU
//     flops, :112).
// Starts are deterministic (splitmix64), not time-seeded as in the
// reference (:187): the estimate is reproducible.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "pfdr_graph.hpp"
#include "pfdr_quadratic_kernels.hpp"
#include "pfdr_session.hpp"

namespace pfdr {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <typename real>
struct Mfma;
template <>
struct Mfma<float> {
    static constexpr int T = 32, KS = 2, NR = 16, BT = 128, BK = 32;
    typedef f32x16 acc_t;
    __device__ static acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    }
    // C/D map of the 32x32 shapes
    __device__ static int row(int lane, int r) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }
    __device__ static int col(int lane, int) { return lane & 31; }
};
template <>
struct Mfma<double> {
    static constexpr int T = 16, KS = 4, NR = 4, BT = 64, BK = 16;
    typedef f64x4 acc_t;
    __device__ static acc_t mma(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // f64 16x16x4 has its own C/D map (cdna_hip_programming.md §3)
    __device__ static int row(int lane, int r) { return (lane >> 4) + 4 * r; }
    __device__ static int col(int lane, int) { return lane & 15; }
};

enum GramLayout : int {
    GRAM_TN = 0,  // G = A^t A: A is K-by-P column-major (contraction index contiguous)
    GRAM_NT = 1   // G = A A^t: A is P-by-K column-major (output index contiguous)
};

// element (i, k) of the operand: TN A[k + i*ld], NT A[i + k*ld]
template <typename real, int LAYOUT>
__device__ __forceinline__ real gram_elem(const real *A, long ld, long i, long k) {
    return LAYOUT == GRAM_TN ? A[k + i * ld] : A[i + k * ld];
}

// Block -> (tile bi <= bj of the upper block triangle, contraction chunk z).
// The dispatcher deals blocks round-robin over the 8 XCDs (block b on XCD
// b % 8), so XCD x gets the chunks z = x, x + 8, ... with all their tiles
// together: every XCD has the same share of the work, and the operand
// panels of a chunk are fetched into that XCD's L2 for all the tiles that
// share them.  (A 3-D (bi, bj, z) grid put every tile of block row bi on
// XCD bi: XCD 0 had 8 tiles per chunk, XCD 7 one.)  With fewer than 8
// chunks (large P: A^tA of a wide A), XCD x gets the x-th eighth of the
// tiles of every chunk instead (consecutive tiles share their row panel);
// dealing chunks to XCDs there left 7 of the 8 XCDs idle.
__host__ __device__ __forceinline__ long gram_slots(int nb, long nchunk) {
    const long ntiles = (long)nb * (nb + 1) / 2;
    return nchunk % 8 == 0 ? nchunk * ntiles : 8 * ((ntiles + 7) / 8) * nchunk;
}
__device__ __forceinline__ bool gram_block(int nb, int nchunk, int &bi, int &bj, int &z) {
    const int ntiles = nb * (nb + 1) / 2;
    const int b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    int t;
    if (nchunk % 8 == 0) {
        z = (slot / ntiles) * 8 + xcd;
        t = slot - (slot / ntiles) * ntiles;
    } else {
        const int per = (ntiles + 7) / 8;
        z = slot / per;
        t = xcd * per + (slot - z * per);
        if (t >= ntiles) return false;
    }
    if (z >= nchunk) return false;
    bi = 0;
    while (t >= nb - bi) { t -= nb - bi; bi++; }
    bj = bi + t;
    return true;
}

// One block = one BT x BT tile (bi <= bj) of the chunk [k0, k1) of the
// contraction; output partial G (P x P, column-major) of this chunk.
template <typename real, int LAYOUT>
__global__ __launch_bounds__(256) void k_gram(int P, long K, const real *__restrict__ A, long ld,
                                            long kchunk, int nchunk, real *__restrict__ Gpart) {
    using M = Mfma<real>;
    constexpr int BT = M::BT, BK = M::BK, T = M::T, WT = BT / 2, NT = WT / T;
    int bi, bj, z;
    if (!gram_block((P + BT - 1) / BT, nchunk, bi, bj, z)) return;
    const long k0 = (long)z * kchunk;
    const long k1 = min(K, k0 + kchunk);
    real *G = Gpart + (size_t)z * P * P;
    __shared__ real Ls[BK][BT + 1], Rs[BK][BT + 1];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wi = w & 1, wj = w >> 1;
    typename M::acc_t acc[NT][NT];
#pragma unroll
    for (int a = 0; a < NT; a++)
#pragma unroll
        for (int b = 0; b < NT; b++)
#pragma unroll
            for (int r = 0; r < M::NR; r++) acc[a][b][r] = real(0);
    const long i0 = (long)bi * BT, j0 = (long)bj * BT;
    for (long kb = k0; kb < k1; kb += BK) {
        // stage the two BT x BK operand tiles as [k][i]
        for (int e = t; e < BT * BK; e += 256) {
            int i, k;
            if (LAYOUT == GRAM_TN) { i = e / BK; k = e - i * BK; }   // k fastest: coalesced columns
            else { k = e / BT; i = e - k * BT; }                     // i fastest
            const long kk = kb + k;
            const bool kin = kk < k1;
            Ls[k][i] = (kin && i0 + i < P) ? gram_elem<real, LAYOUT>(A, ld, i0 + i, kk) : real(0);
            Rs[k][i] = (kin && j0 + i < P) ? gram_elem<real, LAYOUT>(A, ld, j0 + i, kk) : real(0);
        }
        __syncthreads();
#pragma unroll 4
        for (int ks = 0; ks < BK; ks += M::KS) {
            const int kr = ks + lane / T, c = lane % T;
            real a[NT], b[NT];
#pragma unroll
            for (int q = 0; q < NT; q++) {
                a[q] = Ls[kr][wi * WT + q * T + c];
                b[q] = Rs[kr][wj * WT + q * T + c];
            }
#pragma unroll
            for (int x = 0; x < NT; x++)
#pragma unroll
                for (int y = 0; y < NT; y++) acc[x][y] = M::mma(a[x], b[y], acc[x][y]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int x = 0; x < NT; x++)
#pragma unroll
        for (int y = 0; y < NT; y++)
#pragma unroll
            for (int r = 0; r < M::NR; r++) {
                const long i = i0 + wi * WT + x * T + M::row(lane, r);
                const long j = j0 + wj * WT + y * T + M::col(lane, r);
                if (i < P && j < P) {
                    G[i + j * P] = acc[x][y][r];
                    if (bi != bj) G[j + i * P] = acc[x][y][r];
                }
            }
}

// The same tile with 16-byte operand loads and a register prefetch of the
// next K slice while the matrix cores work on the current one (needs
// ld % (16 / sizeof(real)) == 0 and a 16-byte aligned A).  WG waves per
// block: 4 -> a 2x2 grid of MFMA tiles per wave; 2 -> 4x2 per wave (each
// k step reads 4 + 2 operand fragments for 8 MFMAs instead of 2 + 2 for
// 4, and a wave does twice the MFMAs per K slice and barrier).  Measured
// (r4t, rocprofv3 MfmaUtil on C3's A A^t): 4x2 tiles need 324-352 VGPRs,
// one wave per SIMD, 94 TF/s / MfmaUtil 63 % against 113 TF/s / 81 % for
// 2x2 -- so 2x2 it is.
constexpr int kGramWaves = 4;
template <typename real, int LAYOUT, int WG = kGramWaves>
__global__ __launch_bounds__(64 * WG) void k_gram_v(int P, long K, const real *__restrict__ A,
                                                   long ld, long kchunk, int nchunk,
                                                   real *__restrict__ Gpart) {
    using M = Mfma<real>;
    constexpr int NTH = 64 * WG, WI = WG == 4 ? 2 : 1;     // waves along i (2 along j)
    constexpr int BT = M::BT, BK = M::BK, T = M::T, TI = BT / WI, TJ = BT / 2;
    constexpr int NX = TI / T, NY = TJ / T;               // MFMA tiles per wave
    constexpr int VW = 16 / sizeof(real);                 // reals per 16-byte load
    constexpr int NL = BT * BK / (NTH * VW);              // vector loads per operand per lane
    int bi, bj, z;
    if (!gram_block((P + BT - 1) / BT, nchunk, bi, bj, z)) return;
    const long k0 = (long)z * kchunk;
    const long k1 = min(K, k0 + kchunk);
    real *G = Gpart + (size_t)z * P * P;
    // row pad: NT stores 16-byte vectors (pad VW keeps them aligned); TN
    // stores the K-contiguous loads transposed, one real at a time, and a
    // pad of VW put a wave's (i, k) slots on 16 of the 32 banks (4-way
    // conflicts, 12 % of the cycles in SQ_LDS_BANK_CONFLICT on A^tA, r3q):
    // a pad of 1 spreads them (f32)
    constexpr int PADC = (LAYOUT == GRAM_TN && sizeof(real) == 4) ? 1 : VW;
    __shared__ alignas(16) real Ls[BK][BT + PADC], Rs[BK][BT + PADC];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wi = w % WI, wj = w / WI;
    const long i0 = (long)bi * BT, j0 = (long)bj * BT;
    typename M::acc_t acc[NX][NY];
#pragma unroll
    for (int a = 0; a < NX; a++)
#pragma unroll
        for (int b = 0; b < NY; b++)
#pragma unroll
            for (int r = 0; r < M::NR; r++) acc[a][b][r] = real(0);
    // lane's vector slots: NT layout (i, k) = (4 consecutive i, one k);
    // TN layout (i, k) = (one i, VW consecutive k)
    Pk<real, VW> lr[NL], rr[NL];
    auto load = [&](long kb) {
#pragma unroll
        for (int q = 0; q < NL; q++) {
            const int f = t + NTH * q;
            int i, k;
            if (LAYOUT == GRAM_NT) { k = f / (BT / VW); i = (f - k * (BT / VW)) * VW; }
            else { i = f / (BK / VW); k = (f - i * (BK / VW)) * VW; }
            const long kk = kb + k;
            for (int side = 0; side < 2; side++) {
                const long base = side ? j0 : i0;
                Pk<real, VW> &o = side ? rr[q] : lr[q];
                const bool full = LAYOUT == GRAM_NT ? (kk < k1 && base + i + VW <= P)
                                                    : (kk + VW <= k1 && base + i < P);
                if (full) {
                    o = LAYOUT == GRAM_NT ? ldv<real, VW>(A + (base + i) + kk * ld)
                                          : ldv<real, VW>(A + kk + (base + i) * ld);
                } else {
#pragma unroll
                    for (int u = 0; u < VW; u++) {
                        const long ii = LAYOUT == GRAM_NT ? base + i + u : base + i;
                        const long ku = LAYOUT == GRAM_NT ? kk : kk + u;
                        o.v[u] = (ii < P && ku < k1) ? gram_elem<real, LAYOUT>(A, ld, ii, ku)
                                                     : real(0);
                    }
                }
            }
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int q = 0; q < NL; q++) {
            const int f = t + NTH * q;
            if (LAYOUT == GRAM_NT) {
                const int k = f / (BT / VW), i = (f - k * (BT / VW)) * VW;
                stv<real, VW>(&Ls[k][i], lr[q]);
                stv<real, VW>(&Rs[k][i], rr[q]);
            } else {
                const int i = f / (BK / VW), k = (f - i * (BK / VW)) * VW;
#pragma unroll
                for (int u = 0; u < VW; u++) { Ls[k + u][i] = lr[q].v[u]; Rs[k + u][i] = rr[q].v[u]; }
            }
        }
    };
    if (k0 < k1) load(k0);
    for (long kb = k0; kb < k1; kb += BK) {
        store();
        __syncthreads();
        if (kb + BK < k1) load(kb + BK);  // in flight during the MFMAs below
#pragma unroll 4
        for (int ks = 0; ks < BK; ks += M::KS) {
            const int kr = ks + lane / T, c = lane % T;
            real a[NX], b[NY];
#pragma unroll
            for (int q = 0; q < NX; q++) a[q] = Ls[kr][wi * TI + q * T + c];
#pragma unroll
            for (int q = 0; q < NY; q++) b[q] = Rs[kr][wj * TJ + q * T + c];
#pragma unroll
            for (int x = 0; x < NX; x++)
#pragma unroll
                for (int y = 0; y < NY; y++) acc[x][y] = M::mma(a[x], b[y], acc[x][y]);
        }
        __syncthreads();
    }
    // epilogue through LDS: each wave writes its T x T MFMA tiles as whole
    // column segments of G (T contiguous reals per column) and, off the
    // diagonal, the mirror tile the same way (the accumulator map puts
    // consecutive lanes on consecutive COLUMNS: storing it directly made one
    // of the two writes a stride-P scatter, which dominated for large P)
    __shared__ real Os[WG][T][T + 1];
    real(*O)[T + 1] = Os[w];
    constexpr int JS = 64 / T;
    const int li = lane % T, lj = lane / T;
#pragma unroll
    for (int x = 0; x < NX; x++)
#pragma unroll
        for (int y = 0; y < NY; y++) {
            const long ib = i0 + wi * TI + x * T, jb = j0 + wj * TJ + y * T;
#pragma unroll
            for (int r = 0; r < M::NR; r++) O[M::row(lane, r)][M::col(lane, r)] = acc[x][y][r];
            __syncthreads();
            for (int j = lj; j < T; j += JS)
                if (ib + li < P && jb + j < P) G[(ib + li) + (jb + j) * P] = O[li][j];
            if (bi != bj)
                for (int i = lj; i < T; i += JS)
                    if (jb + li < P && ib + i < P) G[(jb + li) + (ib + i) * P] = O[i][li];
            __syncthreads();
        }
}


// f32 Gram on the bf16 matrix cores, f32-accurate: every element is split
// exactly into three bf16 pieces, x = h + m + l (h = x truncated to 8
// significant bits, m = x - h rounded to 8, l = x - h - m: no bits lost), and
// a product x y is formed from the six pieces whose weight reaches 2^-16 of
// it (hh, hm, mh, hl, lh, mm) on v_mfma_f32_32x32x16_bf16, accumulated in
// f32; the pieces left out (ml, lm, ll) weigh about 2^-23 of each product
// (up to ~2^-22 when the truncated leading piece leaves m near its bound;
// tests/test_gram_split_cpu.py checks <= 2^-21), at the f32 rounding of the
// sum.  A NaN in a tile (an overflow split into pieces of both signs, or an
// infinite element) sends the whole Gram to the exact-f32 tile (gram()).  Six bf16 MFMAs of 16 k do the work of
// eight f32 ones of 2 k at a sixteenth of the rate per flop: 2.7x the f32
// matrix-core throughput.  Same blocks, tiles and chunks
// as k_gram_v; the staging splits each element once, into three bf16
// planes [row][k] (rows of BK + 8: 16-byte fragment reads conflict-free).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ unsigned short bf16_rne(float x) {
    unsigned u = __builtin_bit_cast(unsigned, x);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}
// the leading piece: x's top 16 bits (truncation never overflows to inf,
// and x - h is exact with at most 16 significant bits)
__device__ __forceinline__ unsigned short bf16_trunc(float x) {
    return (unsigned short)(__builtin_bit_cast(unsigned, x) >> 16);
}
__device__ __forceinline__ float bf16_val(unsigned short h) {
    return __builtin_bit_cast(float, (unsigned)h << 16);
}
template <int LAYOUT, int BK, bool VEC>
__device__ __forceinline__ void gram_b_body(int P, long K, const float *__restrict__ A, long ld,
                                            long kchunk, int nchunk, float *__restrict__ Gpart,
                                            int *__restrict__ nanflag) {
    using M = Mfma<float>;
    constexpr int BT = 128, T = 32, RS = BK + 8, NK = BK / 2;
    constexpr int RW = 2, KQ = BK / (2 * RW);  // NT staging: RW rows of KQ k per lane
    // piece planes: [row][k] (rows of RS) -- or, for NT staged from row
    // loads, [k][row] (rows of RK = 160: the 4 k rows a transposed read
    // gathers sit 80 dwords apart, on distinct banks) read back with
    // ds_read_b64_tr_b16: a wave's staging writes are then 256 contiguous
    // bytes, where [row][k] put them 48 B apart on a quarter of the banks
    // (SQ_LDS_BANK_CONFLICT 2.6e9 cycles on C3, r6q)
    constexpr bool KI = LAYOUT == GRAM_NT && VEC;
    constexpr int RK = 160;
    constexpr int PL = KI ? BK * RK : BT * RS;
    static_assert(BK == 16 || BK == 32, "slices of one or two 16-k MFMA steps");
    int bi, bj, z;
    if (!gram_block((P + BT - 1) / BT, nchunk, bi, bj, z)) return;
    const long k0 = (long)z * kchunk;
    const long k1 = min(K, k0 + kchunk);
    float *G = Gpart + (size_t)z * P * P;
    // [side][piece][row][RS] bf16; the epilogue's tiles reuse it
    __shared__ alignas(16) unsigned short sm[2 * 3 * PL];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wi = w & 1, wj = w >> 1;
    const long i0 = (long)bi * BT, j0 = (long)bj * BT;
    M::acc_t acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int r = 0; r < M::NR; r++) acc[a][b][r] = 0.f;
    // staging: lane t holds row ri of both sides, k = kg NK ... kg NK + NK - 1
    const int ri = t & (BT - 1), kg = t >> 7;
    float st[2][NK];
    const int ld32 = (int)ld;  // (gram() checks 16 ld + 128 < 2^31)
    auto load = [&](long kb) {
        const long kk = kb + kg * NK;
#pragma unroll
        for (int side = 0; side < 2; side++) {
            const long rb0 = side ? j0 : i0, row = rb0 + ri;
            const bool rin = row < P;
            if (LAYOUT == GRAM_NT && VEC) {
                // rows RW rp ... RW rp + RW - 1 (one RW-wide load per k), k =
                // kq ... kq + KQ - 1: st[side][RW q + r] = (row RW rp + r, k
                // kq + q); a wave-uniform base and 32-bit lane offsets,
                // out-of-range elements from a clamped address, zeroed
                const float *base = A + rb0 + kb * ld;
                const int rp = t % (BT / RW), kq = (t / (BT / RW)) * KQ;
                const int kl = (int)(k1 - kb) - 1;  // last k of the chunk, from kb
                const bool whole = rb0 + BT <= P && kb + BK <= k1;  // block-uniform
#pragma unroll
                for (int q = 0; q < KQ; q++) {
                    const int kc = min(kq + q, kl);
                    if (whole || (rb0 + RW * rp + RW - 1 < P && kq + q <= kl)) {
                        const Pk<float, RW> v = ldv<float, RW>(base + RW * rp + kc * ld32);
#pragma unroll
                        for (int r = 0; r < RW; r++) st[side][RW * q + r] = v.v[r];
                    } else {
#pragma unroll
                        for (int r = 0; r < RW; r++)
                            st[side][RW * q + r] = (rb0 + RW * rp + r < P && kq + q <= kl)
                                                       ? base[RW * rp + r + kc * ld32] : 0.f;
                    }
                }
            } else if (LAYOUT == GRAM_NT) {
                const float *base = A + rb0 + kb * ld;
                const int rc = (int)min(row, (long)P - 1) - (int)rb0;
                const int kl = (int)(k1 - kb) - 1;
#pragma unroll
                for (int q = 0; q < NK; q++) {
                    const int kq = kg * NK + q;
                    const float v = base[rc + min(kq, kl) * ld32];
                    st[side][q] = (rin && kq <= kl) ? v : 0.f;
                }
            } else if (VEC && rin && kk + NK <= k1) {
#pragma unroll
                for (int q = 0; q < NK / 4; q++) {
                    const Pk<float, 4> v = ldv<float, 4>(A + kk + 4 * q + row * ld);
#pragma unroll
                    for (int u = 0; u < 4; u++) st[side][4 * q + u] = v.v[u];
                }
            } else {
#pragma unroll
                for (int q = 0; q < NK; q++)
                    st[side][q] = (rin && kk + q < k1) ? gram_elem<float, LAYOUT>(A, ld, row, kk + q) : 0.f;
            }
        }
    };
    auto store = [&]() {
        if (KI) {  // rows 2 rp, 2 rp + 1 at each of the lane's KQ k: 4 B per piece
            typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
            const int rp = t % (BT / RW), kq = (t / (BT / RW)) * KQ;
#pragma unroll
            for (int side = 0; side < 2; side++)
#pragma unroll
                for (int q = 0; q < KQ; q++) {
                    u16x2 ph, pm, pl;
#pragma unroll
                    for (int r = 0; r < 2; r++) {
                        const float x = st[side][2 * q + r];
                        const unsigned short h = bf16_trunc(x);
                        const float r1 = x - bf16_val(h);
                        const unsigned short m = bf16_rne(r1);
                        ph[r] = h;
                        pm[r] = m;
                        pl[r] = bf16_rne(r1 - bf16_val(m));
                    }
                    unsigned short *d = sm + side * 3 * PL + (kq + q) * RK + 2 * rp;
                    *reinterpret_cast<u16x2 *>(d) = ph;
                    *reinterpret_cast<u16x2 *>(d + PL) = pm;
                    *reinterpret_cast<u16x2 *>(d + 2 * PL) = pl;
                }
            return;
        }
#pragma unroll
        for (int side = 0; side < 2; side++)
#pragma unroll
            for (int c = 0; c < NK / 8; c++) {
                u16x8 ph, pm, pl;
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const float x = st[side][8 * c + u];
                    const unsigned short h = bf16_trunc(x);
                    const float r1 = x - bf16_val(h);
                    const unsigned short m = bf16_rne(r1);
                    ph[u] = h;
                    pm[u] = m;
                    pl[u] = bf16_rne(r1 - bf16_val(m));
                }
                unsigned short *d = sm + side * 3 * PL + ri * RS + kg * NK + 8 * c;
                *reinterpret_cast<u16x8 *>(d) = ph;
                *reinterpret_cast<u16x8 *>(d + PL) = pm;
                *reinterpret_cast<u16x8 *>(d + 2 * PL) = pl;
            }
    };
    // the 32x32x16 operand of rows tb ... tb + 31: lane l holds row tb + (l
    // & 31), k = 16 ks + 8 (l >> 5) ... + 7
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    auto frag = [&](int side, int piece, int tb, int ks) {
        const unsigned short *pl = sm + (side * 3 + piece) * PL;
        if constexpr (KI) {
            // two transposed reads of 4 k rows each: in lane group g = l >>
            // 4, lane 4 q + p names k row 16 ks + 8 (g >> 1) + q (+ 4) at
            // columns tb + 16 (g & 1) + 4 p ...; lane i of the group gets
            // column tb + 16 (g & 1) + i of the 4 rows
            const int g = lane >> 4, li = lane & 15;
            const unsigned short *a = pl + (16 * ks + 8 * (g >> 1) + (li >> 2)) * RK + tb +
                                      16 * (g & 1) + 4 * (li & 3);
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)a);
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a + 4 * RK));
            return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        } else {
            return *reinterpret_cast<const bf16x8 *>(pl + (tb + (lane & 31)) * RS + 16 * ks +
                                                     8 * (lane >> 5));
        }
    };
    const int ra = wi * 64, rb = wj * 64;
    if (k0 < k1) load(k0);
    for (long kb = k0; kb < k1; kb += BK) {
        store();
        __syncthreads();
        if (kb + BK < k1) load(kb + BK);  // in flight during the MFMAs below
#pragma unroll
        for (int ks = 0; ks < BK / 16; ks++) {
            bf16x8 ah[2], bh[2], am[2], bm[2];
#pragma unroll
            for (int q = 0; q < 2; q++) {
                ah[q] = frag(0, 0, ra + 32 * q, ks);
                bh[q] = frag(1, 0, rb + 32 * q, ks);
            }
#pragma unroll
            for (int x = 0; x < 2; x++)
#pragma unroll
                for (int y = 0; y < 2; y++)
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[x], bh[y], acc[x][y], 0, 0, 0);
#pragma unroll
            for (int q = 0; q < 2; q++) {
                am[q] = frag(0, 1, ra + 32 * q, ks);
                bm[q] = frag(1, 1, rb + 32 * q, ks);
            }
#pragma unroll
            for (int x = 0; x < 2; x++)
#pragma unroll
                for (int y = 0; y < 2; y++) {
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[x], bm[y], acc[x][y], 0, 0, 0);
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[x], bh[y], acc[x][y], 0, 0, 0);
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[x], bm[y], acc[x][y], 0, 0, 0);
                }
#pragma unroll
            for (int q = 0; q < 2; q++) {
                am[q] = frag(0, 2, ra + 32 * q, ks);  // the l pieces
                bm[q] = frag(1, 2, rb + 32 * q, ks);
            }
#pragma unroll
            for (int x = 0; x < 2; x++)
#pragma unroll
                for (int y = 0; y < 2; y++) {
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[x], bm[y], acc[x][y], 0, 0, 0);
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[x], bh[y], acc[x][y], 0, 0, 0);
                }
        }
        __syncthreads();
    }
    // epilogue as k_gram_v's, its tiles in the staging array
    float(*O)[T + 1] = reinterpret_cast<float(*)[T + 1]>(reinterpret_cast<float *>(sm) + w * T * (T + 1));
    const int li = lane % T, lj = lane / T;
    // a NaN here where no input was NaN is an overflow the split turned into
    // inf - inf (pieces of both signs, or an infinite element split as
    // h = inf, m = NaN): gram() then recomputes G on the exact-f32 tile,
    // whose inf the reference's f32 sums give (one lane's vector store)
    bool bad = false;
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 2; y++)
#pragma unroll
            for (int r = 0; r < M::NR; r++) bad |= acc[x][y][r] != acc[x][y][r];
    if (bad) nanflag[0] = 1;
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 2; y++) {
            const long ib = i0 + wi * 64 + x * T, jb = j0 + wj * 64 + y * T;
#pragma unroll
            for (int r = 0; r < M::NR; r++) O[M::row(lane, r)][M::col(lane, r)] = acc[x][y][r];
            __syncthreads();
            // the pieces' cross products (hm, mh) are added in row-column
            // order, so G(i, j) and G(j, i) of a diagonal block may round
            // apart: there the upper triangle is written and mirrored
            const bool diag = bi == bj;
            for (int j = lj; j < T; j += 2)
                if (ib + li < P && jb + j < P && (!diag || ib + li <= jb + j))
                    G[(ib + li) + (jb + j) * P] = O[li][j];
            for (int i = lj; i < T; i += 2)
                if (jb + li < P && ib + i < P && (!diag || ib + i < jb + li))
                    G[(jb + li) + (ib + i) * P] = O[i][li];
            __syncthreads();
        }
}

// four blocks per CU (LDS 36 KB, <= 128 registers; loading two slices
// ahead needs three waves per SIMD and measured slower: C3 26.7 vs 21.6 ms)
template <int LAYOUT, int BK, bool VEC>  // (NT from 16-byte four-row loads: C3 28.4 ms)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_gram_b(
    int P, long K, const float *__restrict__ A, long ld, long kchunk, int nchunk,
    float *__restrict__ Gpart, int *__restrict__ nanflag) {
    gram_b_body<LAYOUT, BK, VEC>(P, K, A, ld, kchunk, nchunk, Gpart, nanflag);
}

// G = sum of the chunk partials, in chunk order
template <typename real>
__global__ void k_gram_sum(long PP, int nchunk, const real *__restrict__ part,
                           real *__restrict__ G) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= PP) return;
    real s = part[i];
    for (int c = 1; c < nchunk; c++) s += part[(size_t)c * PP + i];
    G[i] = s;
}

// G (P x P) of A: which = 0 -> A^t A (A is K x P, ld >= K), 1 -> A A^t (A is
// P x K, ld >= P).  Device pointers; G may not alias A.
template <typename real>
void gram(int which, int P, long K, const real *A, long ld, real *G, hipStream_t s) {
    using M = Mfma<real>;
    if (P <= 0) return;
    // 16-byte operand loads when the layout allows (k_gram_v), else k_gram
    const bool vec = (ld % (16 / sizeof(real))) == 0 && ((uintptr_t)A % 16) == 0;
    const int BT = M::BT, BK = M::BK;
    // f32 on the bf16 matrix cores (k_gram_b; paired on one box: c3_ata's
    // A^t A 9.1 vs 11.0 ms, C3's A A^t 19.7 vs 21.1 ms); PFDR_GRAM_SPLIT=0
    // keeps the exact-f32 tile (k_gram_v)
    static const bool split_on = [] {
        const char *e = getenv("PFDR_GRAM_SPLIT");
        return !(e && e[0] == '0');
    }();
    const bool split = sizeof(real) == 4 && split_on && 16 * ld + 128 < 0x7fffffffL;
    // blocks to aim for: the split tile's shorter blocks want more of them
    // (C3: 128 chunks 19.2-19.4 ms against 64 chunks' 19.9-20.0, r6n)
    const long target = split ? 4096 : 2048;
    const int nb = (P + BT - 1) / BT;
    const long tiles = (long)nb * (nb + 1) / 2;
    long nchunk = std::max(1L, std::min((target + tiles - 1) / tiles, (K + 4 * BK - 1) / (4 * BK)));
    if (nchunk > 8) nchunk = (nchunk + 7) / 8 * 8;  // the same number of chunks on every XCD
    long kchunk = (K + nchunk - 1) / nchunk;
    kchunk = ((kchunk + BK - 1) / BK) * BK;
    nchunk = K > 0 ? (K + kchunk - 1) / kchunk : 1;
    if (nchunk > 65535) throw std::runtime_error("gram: contraction too long");
    const size_t PP = (size_t)P * P;
    DevBuf<real> part;
    real *out = G;
    if (nchunk > 1) { part.alloc(PP * nchunk); out = part.p; }
    if (K == 0) { PFDR_HIP(hipMemsetAsync(G, 0, PP * sizeof(real), s)); return; }
    const long nblk = gram_slots(nb, nchunk);  // see gram_block
    if (nblk > 0x7fffffffL) throw std::runtime_error("gram: grid too large");
    const dim3 grid((unsigned)nblk);
    if (split) {
        const float *Af = reinterpret_cast<const float *>(A);
        float *of = reinterpret_cast<float *>(out);
        DevBuf<int> nanflag(1);
        PFDR_HIP(hipMemsetAsync(nanflag.p, 0, sizeof(int), s));
        constexpr int BKS = 16;  // (BK = 32: 61 KB of LDS, two blocks per CU, slower)
        if (which == 0) {
            if (vec) k_gram_b<GRAM_TN, BKS, true><<<grid, 256, 0, s>>>(P, K, Af, ld, kchunk, (int)nchunk, of, nanflag.p);
            else k_gram_b<GRAM_TN, BKS, false><<<grid, 256, 0, s>>>(P, K, Af, ld, kchunk, (int)nchunk, of, nanflag.p);
        } else {
            if (vec) k_gram_b<GRAM_NT, BKS, true><<<grid, 256, 0, s>>>(P, K, Af, ld, kchunk, (int)nchunk, of, nanflag.p);
            else k_gram_b<GRAM_NT, BKS, false><<<grid, 256, 0, s>>>(P, K, Af, ld, kchunk, (int)nchunk, of, nanflag.p);
        }
        PFDR_HIP(hipGetLastError());
        int h = 0;
        PFDR_HIP(hipMemcpyAsync(&h, nanflag.p, sizeof(int), hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
        if (h) {  // an overflow (or a non-finite input): the exact-f32 tile's semantics
            if (vec && which == 0)
                k_gram_v<real, GRAM_TN><<<grid, 64 * kGramWaves, 0, s>>>(P, K, A, ld, kchunk,
                                                                        (int)nchunk, out);
            else if (vec)
                k_gram_v<real, GRAM_NT><<<grid, 64 * kGramWaves, 0, s>>>(P, K, A, ld, kchunk,
                                                                        (int)nchunk, out);
            else if (which == 0)
                k_gram<real, GRAM_TN><<<grid, 256, 0, s>>>(P, K, A, ld, kchunk, (int)nchunk, out);
            else
                k_gram<real, GRAM_NT><<<grid, 256, 0, s>>>(P, K, A, ld, kchunk, (int)nchunk, out);
        }
    } else if (vec) {
        if (which == 0)
            k_gram_v<real, GRAM_TN><<<grid, 64 * kGramWaves, 0, s>>>(P, K, A, ld, kchunk,
                                                                    (int)nchunk, out);
        else
            k_gram_v<real, GRAM_NT><<<grid, 64 * kGramWaves, 0, s>>>(P, K, A, ld, kchunk,
                                                                    (int)nchunk, out);
    } else {
        if (which == 0) k_gram<real, GRAM_TN><<<grid, 256, 0, s>>>(P, K, A, ld, kchunk, (int)nchunk, out);
        else k_gram<real, GRAM_NT><<<grid, 256, 0, s>>>(P, K, A, ld, kchunk, (int)nchunk, out);
    }
    PFDR_HIP(hipGetLastError());
    if (nchunk > 1) {
        k_gram_sum<real><<<grid_for((long)PP), kBlock, 0, s>>>((long)PP, (int)nchunk, part.p, G);
        PFDR_HIP(hipGetLastError());
        PFDR_HIP(hipStreamSynchronize(s));  // part is freed on return
    }
}

// ------------------------------------------------------- power method --
// Y (rows x B) = Mat (rows x K, column-major, ld) * X (K x B): one lane per
// row, the B columns of X broadcast from LDS, the matrix streamed once.
template <typename real, int B>
__global__ __launch_bounds__(256) void k_apply_rows(int rows, long K, const real *__restrict__ Mat,
                                                  long ld, const real *__restrict__ X,
                                                  real *__restrict__ Y, int kchunk,
                                                  real *__restrict__ part) {
    __shared__ real xs[64][B];
    const long r = (long)blockIdx.x * 256 + threadIdx.x;
    const long kb0 = (long)blockIdx.y * kchunk, kb1 = min(K, kb0 + kchunk);
    real acc[B];
#pragma unroll
    for (int c = 0; c < B; c++) acc[c] = real(0);
    for (long k0 = kb0; k0 < kb1; k0 += 64) {
        const int nk = (int)min(64L, kb1 - k0);
        for (int e = threadIdx.x; e < 64 * B; e += 256) {
            const int k = e / B, c = e - k * B;
            xs[k][c] = k < nk ? X[(k0 + k) + (long)c * K] : real(0);
        }
        __syncthreads();
        if (r < rows) {
            for (int k = 0; k < nk; k++) {
                const real m = Mat[r + (k0 + k) * ld];
#pragma unroll
                for (int c = 0; c < B; c++) acc[c] += m * xs[k][c];
            }
        }
        __syncthreads();
    }
    if (r < rows) {
        real *out = gridDim.y > 1 ? part + (size_t)blockIdx.y * rows * B : Y;
#pragma unroll
        for (int c = 0; c < B; c++) out[r + (long)c * rows] = acc[c];
    }
}

template <typename real>
__global__ void k_sum_parts(long n, int np, const real *__restrict__ part, real *__restrict__ Y) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    real s = part[i];
    for (int c = 1; c < np; c++) s += part[(size_t)c * n + i];
    Y[i] = s;
}

// Y (cols x B) = Mat^t X: Mat is rows x cols column-major; one wave per column
template <typename real, int B>
__global__ __launch_bounds__(256) void k_apply_cols(int rows, long cols, const real *__restrict__ Mat,
                                                  long ld, const real *__restrict__ X,
                                                  real *__restrict__ Y) {
    const int lane = threadIdx.x & 63;
    const long j = ((long)blockIdx.x * 256 + threadIdx.x) >> 6;
    if (j >= cols) return;
    const real *m = Mat + j * ld;
    real acc[B];
#pragma unroll
    for (int c = 0; c < B; c++) acc[c] = real(0);
    for (int i = lane; i < rows; i += 64) {
        const real v = m[i];
#pragma unroll
        for (int c = 0; c < B; c++) acc[c] += v * X[i + (long)c * rows];
    }
#pragma unroll
    for (int c = 0; c < B; c++) {
        const real s = wave_sum(acc[c]);
        if (lane == 0) Y[j + c * cols] = s;
    }
}

// starting vectors: U[-1, 1) from splitmix64 (deterministic)
template <typename real>
__global__ void k_power_init(long n, int B, real *X) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * B) return;
    unsigned long long z = (unsigned long long)i * 0xD1B54A32D192ED03ull + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    X[i] = (real)((double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0);
}

// per-column norms of X (n x B): one block per column
template <typename real>
__global__ __launch_bounds__(256) void k_col_norms(long n, const real *__restrict__ X,
                                                 real *__restrict__ nrm) {
    __shared__ real red[kBlock / kWave];
    const real *x = X + (long)blockIdx.x * n;
    real s = real(0);
    for (long i = threadIdx.x; i < n; i += 256) s += x[i] * x[i];
    s = block_sum(s, red);
    if (threadIdx.x == 0) nrm[blockIdx.x] = std::sqrt(s);
}

// X[:, c] /= b[c]
template <typename real>
__global__ void k_col_scale(long n, int B, real *X, const real *__restrict__ b) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * B) return;
    X[i] /= b[i / n];
}

// the reference's per-start stopping rule (:201-205): a = new norm, b = old;
// state[c]: 0 running, 1 stopped; res[c] holds b
template <typename real>
__global__ void k_power_step(int B, const real *__restrict__ a, real *b, int *state, real nTol,
                             int *running) {
    const int c = threadIdx.x;
    if (c >= B) return;
    if (state[c]) return;
    if ((a[c] - b[c]) / b[c] < nTol) { state[c] = 1; return; }
    b[c] = a[c];
    atomicAdd(running, 1);
}

template <typename real>
static void apply_rows(int B, int rows, long K, const real *Mat, long ld, const real *X, real *Y,
                       hipStream_t s) {
    // split the contraction so that short-and-wide products fill the GPU
    const int rb = (rows + 255) / 256;
    int np = (int)std::max(1L, std::min(512L / rb, (K + 1023) / 1024));
    const int kchunk = (int)((K + np - 1) / np);
    np = (int)((K + kchunk - 1) / kchunk);
    DevBuf<real> part;
    if (np > 1) part.alloc((size_t)np * rows * B);
    dim3 g(rb, np);
#define PFDR_APPLY(BB) k_apply_rows<real, BB><<<g, 256, 0, s>>>(rows, K, Mat, ld, X, Y, kchunk, part.p)
    if (B == 16) PFDR_APPLY(16);
    else if (B == 32) PFDR_APPLY(32);
    else PFDR_APPLY(64);
#undef PFDR_APPLY
    PFDR_HIP(hipGetLastError());
    if (np > 1) {
        k_sum_parts<real><<<grid_for((long)rows * B), kBlock, 0, s>>>((long)rows * B, np, part.p, Y);
        PFDR_HIP(hipGetLastError());
        PFDR_HIP(hipStreamSynchronize(s));
    }
}

template <typename real>
static void apply_cols(int B, int rows, long cols, const real *Mat, long ld, const real *X, real *Y,
                       hipStream_t s) {
    const int g = grid_for(cols * 64);
    if (B == 16) k_apply_cols<real, 16><<<g, 256, 0, s>>>(rows, cols, Mat, ld, X, Y);
    else if (B == 32) k_apply_cols<real, 32><<<g, 256, 0, s>>>(rows, cols, Mat, ld, X, Y);
    else k_apply_cols<real, 64><<<g, 256, 0, s>>>(rows, cols, Mat, ld, X, Y);
    PFDR_HIP(hipGetLastError());
}

// squared operator norm of A (M x N column-major, device), or of the
// symmetric S x S matrix A when M or N is 0 (ref :95-103)
template <typename real>
real operator_norm_device(int M, int N, const real *A, real nTol, int itMax, int nbInit,
                          int verbose, hipStream_t s, double *gram_ms) {
    if (gram_ms) *gram_ms = 0.0;
    const int P = std::min(M, N);
    int S;
    const real *Mat = A;
    DevBuf<real> G;
    bool sym = false;
    if (P == 0) {
        S = std::max(M, N);
        sym = true;
    } else {
        S = N;
        // matrix-core Gram (2 M N P flops at ~1e14/s) vs itMax * nbInit
        // streaming pass pairs over A (2 M N * sizeof(real) bytes at ~5e12/s)
        const double t_gram = 2.0 * M * N * (double)P / 1e14;
        const double t_pass = 2.0 * M * N * sizeof(real) / 5e12 * itMax * std::max(1, nbInit / 64 + 1);
        if (t_gram < t_pass) {
            sym = true;
            S = P;
            G.alloc((size_t)P * P);
            hipEvent_t e0, e1;
            if (gram_ms) {
                PFDR_HIP(hipEventCreate(&e0));
                PFDR_HIP(hipEventCreate(&e1));
                PFDR_HIP(hipEventRecord(e0, s));
            }
            if (P == M) gram<real>(1, P, N, A, M, G.p, s);  // A A^t
            else gram<real>(0, P, M, A, M, G.p, s);         // A^t A
            if (gram_ms) {
                float ms = 0.f;
                PFDR_HIP(hipEventRecord(e1, s));
                PFDR_HIP(hipEventSynchronize(e1));
                PFDR_HIP(hipEventElapsedTime(&ms, e0, e1));
                *gram_ms = ms;
                (void)hipEventDestroy(e0);
                (void)hipEventDestroy(e1);
            }
            Mat = G.p;
        }
    }
    if (verbose) {
        printf("compute matrix operator norm on %d initializations (%s)... ", nbInit,
               sym ? "symmetrized" : "direct");
        fflush(stdout);
    }
    const int n = S;               // length of the iterated vectors
    const int B = nbInit <= 16 ? 16 : nbInit <= 32 ? 32 : 64;
    real best = real(0);
    for (int done = 0; done < std::max(nbInit, 1); done += B) {
        DevBuf<real> X((size_t)n * B), Y((size_t)n * B), T(sym ? 0 : (size_t)M * B), a(B), b(B);
        DevBuf<int> state(B), running(1);
        PFDR_HIP(hipMemsetAsync(state.p, 0, B * sizeof(int), s));
        k_power_init<real><<<grid_for((long)n * B), kBlock, 0, s>>>(n, B, X.p);
        auto apply = [&](real *in, real *out) {  // out = Mat^t Mat in (or Mat in)
            if (sym) {
                apply_rows<real>(B, n, n, Mat, n, in, out, s);
            } else {
                apply_rows<real>(B, M, N, A, M, in, T.p, s);       // A X
                apply_cols<real>(B, M, N, A, M, T.p, out, s);      // A^t (A X)
            }
        };
        // b = ||X||; X /= b; X = A^tA X; b = ||X|| (ref :193-196)
        k_col_norms<real><<<B, 256, 0, s>>>(n, X.p, b.p);
        k_col_scale<real><<<grid_for((long)n * B), kBlock, 0, s>>>(n, B, X.p, b.p);
        apply(X.p, Y.p);
        k_col_norms<real><<<B, 256, 0, s>>>(n, Y.p, b.p);
        std::swap(X.p, Y.p);
        PinnedSmall pin(s);  // returned on every exit path
        int *hrun = static_cast<int *>(pin.p);
        for (int it = 0; it < itMax; it++) {
            k_col_scale<real><<<grid_for((long)n * B), kBlock, 0, s>>>(n, B, X.p, b.p);
            apply(X.p, Y.p);
            k_col_norms<real><<<B, 256, 0, s>>>(n, Y.p, a.p);
            PFDR_HIP(hipMemsetAsync(running.p, 0, sizeof(int), s));
            k_power_step<real><<<1, 64, 0, s>>>(B, a.p, b.p, state.p, nTol, running.p);
            PFDR_HIP(hipGetLastError());
            std::swap(X.p, Y.p);
            PFDR_HIP(hipMemcpyAsync(hrun, running.p, sizeof(int), hipMemcpyDeviceToHost, s));
            PFDR_HIP(hipStreamSynchronize(s));
            if (*hrun == 0) break;
        }
        std::vector<real> hb(B);
        PFDR_HIP(hipMemcpyAsync(hb.data(), b.p, B * sizeof(real), hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
        const int use = std::min(B, std::max(nbInit, 1) - done);
        for (int c = 0; c < use; c++)
            if (hb[c] > best) best = hb[c];  // NaN-free starts only (ref :208)
    }
    if (verbose) { printf("done.\n"); fflush(stdout); }
    return best;
}

template <typename real>
static int opnorm_host(const char *fn, int M, int N, const real *A, int mem, real nTol, int itMax,
                       int nbInit, int verbose, real *norm2, double *gram_ms) {
    if (M < 0 || N < 0 || (M == 0 && N == 0) || !A || !norm2)
        return report_error(fn, "invalid arguments");
    try {
        hipStream_t s = lib_stream();
        const int P = std::min(M, N);
        const size_t n = P == 0 ? (size_t)std::max(M, N) * std::max(M, N) : (size_t)M * N;
        const real *dA = A;
        DevBuf<real> buf;
        if (mem != PFDR_MEM_DEVICE) {
            buf.alloc(n);
            PFDR_HIP(hipMemcpyAsync(buf.p, A, n * sizeof(real), hipMemcpyHostToDevice, s));
            dA = buf.p;
        }
        *norm2 = operator_norm_device<real>(M, N, dA, nTol, itMax, nbInit, verbose, s, gram_ms);
    } catch (const HipError &h) {
        return report_error(fn, h);
    } catch (const std::exception &ex) {
        return report_error(fn, ex.what());
    }
    return PFDR_OK;
}

template <typename real>
static int gram_host(const char *fn, int which, int M, int N, const real *A, int mem, real *G,
                     double *ms) {
    if (M < 0 || N < 0 || !A || !G || (which != 0 && which != 1))
        return report_error(fn, "invalid arguments");
    try {
        hipStream_t s = lib_stream();
        const int P = which == 0 ? N : M;
        const long K = which == 0 ? M : N;
        const size_t n = (size_t)M * N, PP = (size_t)P * P;
        const real *dA = A;
        real *dG = G;
        DevBuf<real> bA, bG;
        if (mem != PFDR_MEM_DEVICE) {
            bA.alloc(n);
            bG.alloc(PP);
            PFDR_HIP(hipMemcpyAsync(bA.p, A, n * sizeof(real), hipMemcpyHostToDevice, s));
            dA = bA.p;
            dG = bG.p;
        }
        hipEvent_t e0, e1;
        PFDR_HIP(hipEventCreate(&e0));
        PFDR_HIP(hipEventCreate(&e1));
        PFDR_HIP(hipEventRecord(e0, s));
        gram<real>(which, P, K, dA, M, dG, s);
        PFDR_HIP(hipEventRecord(e1, s));
        PFDR_HIP(hipEventSynchronize(e1));
        float t = 0.f;
        PFDR_HIP(hipEventElapsedTime(&t, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        if (ms) *ms = t;
        if (mem != PFDR_MEM_DEVICE)
            PFDR_HIP(hipMemcpyAsync(G, dG, PP * sizeof(real), hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
    } catch (const HipError &h) {
        return report_error(fn, h);
    } catch (const std::exception &ex) {
        return report_error(fn, ex.what());
    }
    return PFDR_OK;
}

template void gram<float>(int, int, long, const float *, long, float *, hipStream_t);
template void gram<double>(int, int, long, const double *, long, double *, hipStream_t);
template float operator_norm_device<float>(int, int, const float *, float, int, int, int,
                                           hipStream_t, double *);
template double operator_norm_device<double>(int, int, const double *, double, int, int, int,
                                             hipStream_t, double *);

}  // namespace pfdr

extern "C" int pfdr_gram_f32(int which, int M, int N, const float *A, int mem, float *G,
                             double *ms) {
    return pfdr::gram_host<float>("pfdr_gram_f32", which, M, N, A, mem, G, ms);
}
extern "C" int pfdr_gram_f64(int which, int M, int N, const double *A, int mem, double *G,
                             double *ms) {
    return pfdr::gram_host<double>("pfdr_gram_f64", which, M, N, A, mem, G, ms);
}
extern "C" int pfdr_operator_norm_f32(int M, int N, const float *A, int mem, float nTol,
                                      int itMax, int nbInit, int verbose, float *norm2,
                                      double *gram_ms) {
    return pfdr::opnorm_host<float>("pfdr_operator_norm_f32", M, N, A, mem, nTol, itMax, nbInit,
                                    verbose, norm2, gram_ms);
}
extern "C" int pfdr_operator_norm_f64(int M, int N, const double *A, int mem, double nTol,
                                      int itMax, int nbInit, int verbose, double *norm2,
                                      double *gram_ms) {
    return pfdr::opnorm_host<double>("pfdr_operator_norm_f64", M, N, A, mem, nTol, itMax, nbInit,
                                     verbose, norm2, gram_ms);
}
