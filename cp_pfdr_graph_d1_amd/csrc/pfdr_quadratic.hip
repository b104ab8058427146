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
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>

#include "pfdr_graph.hpp"
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
struct alignas(sizeof(T) * N) Pk { T v[N]; };

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

// Ordered sum over the incidence slots of the block's vertices.  The slots
// of the block's contiguous vertex range are gathered cooperatively (all
// lanes busy whatever the degrees, coalesced index reads, GB = 16 index
// loads then 16 value gathers in flight per lane) into LDS chunks, then each
// lane adds its own vertex's slots in CSR order.
// Slot value source (MODE): AVG_WZ: wz[slot] written by the edge sweep;
// AVG_GATHER: W2[slot] * Z2[slot] formed here (the reference's Wu*Zu);
// AVG_SCATTER: the edge sweep stored W*Z straight at its CSR position, so the
// row segment is read as one coalesced stream (no index).
// AVG_SPLIT: as AVG_WZ with the contributions stored side-major,
// wz[side * E + e], so the u-side run of a vertex is contiguous.
enum AvgMode : int { AVG_WZ = 0, AVG_GATHER = 1, AVG_SCATTER = 2, AVG_SPLIT = 3 };
constexpr int GB = 16;
template <typename real, int CAP, int MODE = AVG_WZ>
__device__ __forceinline__ real gather_sum(int V, int v0,
                                           const int *__restrict__ ptr,
                                           const unsigned *__restrict__ idx,
                                           const real *__restrict__ wz,
                                           real *lds,
                                           const real *__restrict__ z2 = nullptr,
                                           long E = 0) {
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
            real w[GB];
            if (MODE == AVG_SCATTER) {
#pragma unroll
                for (int u = 0; u < GB; u++) {
                    const int j = b + u * kBlock + tid;
                    w[u] = (j < n) ? wz[c0 + j] : real(0);
                }
            } else {
                unsigned id[GB];
#pragma unroll
                for (int u = 0; u < GB; u++) {
                    const int j = b + u * kBlock + tid;
                    id[u] = (j < n) ? idx[c0 + j] : 0u;
                }
#pragma unroll
                for (int u = 0; u < GB; u++) {
                    const int j = b + u * kBlock + tid;
                    if (MODE == AVG_GATHER) w[u] = (j < n) ? wz[id[u]] * z2[id[u]] : real(0);
                    else if (MODE == AVG_SPLIT)
                        w[u] = (j < n) ? wz[(long)(id[u] & 1u) * E + (id[u] >> 1)] : real(0);
                    else w[u] = (j < n) ? wz[id[u]] : real(0);
                }
            }
#pragma unroll
            for (int u = 0; u < GB; u++) {
                const int j = b + u * kBlock + tid;
                if (j < n) lds[j] = w[u];
            }
        }
        __syncthreads();
        const long a = max(my0, c0), e = min(my1, c0 + (long)n);
        for (long j = a; j < e; j++) s += lds[j - c0];
        __syncthreads();
    }
    return s;
}

template <typename real> struct GatherCap;
template <> struct GatherCap<float> { static constexpr int v = 4096; };
template <> struct GatherCap<double> { static constexpr int v = 4096; };

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

// Z_u = X[Eu], Z_v = X[Ev]   (ref :320-324); half-edge layout Z2[2e + side]
template <typename real>
__global__ void k_z_init(long E, const int *__restrict__ Eu,
                         const int *__restrict__ Ev,
                         const R2<real> *__restrict__ xp,
                         real *__restrict__ Z2) {
    long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    Z2[2 * e] = xp[Eu[e]].x;
    Z2[2 * e + 1] = xp[Ev[e]].x;
}

// diagonal of A^t A for the identity / diagonal / A^tA modes (ref :101-122)
template <typename real>
__global__ void k_diag(int V, int mode, const real *__restrict__ A,
                       real *__restrict__ diag) {
    int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    real d = real(1);
    if (mode == A_DIAG) d = A[v];
    else if (mode == A_ATA) d = A[(size_t)(V + 1) * v];
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

// One wave64 per column: 16-byte loads of the column (and of w, which
// every wave re-reads from L2), wave-shuffle reduction, fused epilogue.
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
    real acc = real(0);
    if ((a.len % VW) == 0) {
        const int nv = a.len / VW;
        for (int i = lane; i < nv; i += 64) {
            Pk<real, VW> x = ldv<real, VW>(c + (size_t)i * VW);
            Pk<real, VW> y = ldv<real, VW>(w + (size_t)i * VW);
#pragma unroll
            for (int j = 0; j < VW; j++) acc += x.v[j] * y.v[j];
        }
    } else {
        for (int i = lane; i < a.len; i += 64) acc += c[i] * w[i];
    }
    acc = wave_sum(acc);
    if (lane != 0) return;
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

// R partials: part[b][n] = sum_{v in block b} A[n + N v] X[v]
// (column-major A streamed once, 16-byte loads, 4 columns in flight)
template <typename real>
__global__ __launch_bounds__(256) void k_rows_partial(
    int N, int V, const real *__restrict__ A, const R2<real> *__restrict__ xp,
    int cpb, real *__restrict__ part, const Ctrl<real> *ctrl, int gate) {
    if (gated(ctrl, gate)) return;
    const int b = blockIdx.x;
    const int v0 = b * cpb, v1 = min(v0 + cpb, V);
    constexpr int VW = Vec<real>::kPer16B;
    if ((N % VW) == 0) {
        for (int n0 = threadIdx.x * VW; n0 < N; n0 += kBlock * VW) {
            real acc[VW];
#pragma unroll
            for (int j = 0; j < VW; j++) acc[j] = real(0);
            int v = v0;
            for (; v + 4 <= v1; v += 4) {
                Pk<real, VW> c[4];
                real x[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    c[q] = ldv<real, VW>(A + (size_t)N * (v + q) + n0);
                    x[q] = xp[v + q].x;
                }
#pragma unroll
                for (int q = 0; q < 4; q++)
#pragma unroll
                    for (int j = 0; j < VW; j++) acc[j] += c[q].v[j] * x[q];
            }
            for (; v < v1; v++) {
                Pk<real, VW> c = ldv<real, VW>(A + (size_t)N * v + n0);
                real x = xp[v].x;
#pragma unroll
                for (int j = 0; j < VW; j++) acc[j] += c.v[j] * x;
            }
#pragma unroll
            for (int j = 0; j < VW; j++) part[(size_t)b * N + n0 + j] = acc[j];
        }
    } else {
        for (int n = threadIdx.x; n < N; n += kBlock) {
            real acc = real(0);
            for (int v = v0; v < v1; v++) acc += A[(size_t)N * v + n] * xp[v].x;
            part[(size_t)b * N + n] = acc;
        }
    }
}

// R[n] = Y[n] - sum_b part[b][n]   (ref :356-367)
template <typename real>
__global__ void k_rows_finish(int N, int nb, const real *__restrict__ part,
                              const real *__restrict__ Y,
                              real *__restrict__ R, const Ctrl<real> *ctrl,
                              int gate) {
    if (gated(ctrl, gate)) return;
    int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    real s = real(0);
    int b = 0;
    for (; b + 8 <= nb; b += 8) {
        real t[8];
#pragma unroll
        for (int q = 0; q < 8; q++) t[q] = part[(size_t)(b + q) * N + n];
#pragma unroll
        for (int q = 0; q < 8; q++) s += t[q];
    }
    for (; b < nb; b++) s += part[(size_t)b * N + n];
    R[n] = Y[n] - s;
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

// c = n / sum|a| (first call) or sum|a| / n (reconditioning), with the sum
// accumulated strictly sequentially in increasing v — the reference's
// single-thread order — so the metric rounds exactly as the reference's.
// One workgroup: all lanes stage chunks in LDS, lane 0 adds them in order.
template <typename real>
__global__ __launch_bounds__(256) void k_seq_c(int V,
                                               const real *__restrict__ absval,
                                               int nparts,
                                               const int *__restrict__ cnt_part,
                                               int init, Ctrl<real> *ctrl) {
    constexpr int CH = 4096;
    __shared__ real buf[2][CH];
    __shared__ int red[kBlock / kWave];
    int cnt = 0;
    for (int i = threadIdx.x; i < nparts; i += kBlock) cnt += cnt_part[i];
    cnt = block_sum(cnt, red);
    real s = real(0);
    int cur = 0;
    // prologue: stage chunk 0
    for (long j = threadIdx.x; j < min((long)CH, (long)V); j += kBlock) buf[0][j] = absval[j];
    __syncthreads();
    for (long c0 = 0; c0 < V; c0 += CH) {
        const long n = min((long)CH, (long)V - c0);
        const long nxt = c0 + CH;
        if (threadIdx.x == 0) {
            const real *b = buf[cur];
            for (long j = 0; j < n; j++) s += b[j];
        } else if (nxt < V) {
            const long m = min((long)CH, (long)V - nxt);
            for (long j = threadIdx.x - 1; j < m; j += kBlock - 1) buf[cur ^ 1][j] = absval[nxt + j];
        }
        __syncthreads();
        cur ^= 1;
    }
    if (threadIdx.x == 0) {
        const real n = (real)cnt;
        ctrl->c = init ? n / s : s / n;
        ctrl->cnt = cnt;
    }
}

// d1 splitting weights (ref :156-192) into both half-edges W2[2e + side].
// On reconditioning, first turn the auxiliary variables into subgradients
// with the OLD weights and metric (ref :89-99).
template <typename real>
__global__ void k_d1_weights(long E, const int *__restrict__ Eu,
                             const int *__restrict__ Ev,
                             const real *__restrict__ La_d1,
                             const Ctrl<real> *__restrict__ ctrl, int init,
                             real condMin, const R2<real> *__restrict__ xp,
                             real *__restrict__ W2,
                             const real *__restrict__ Ga,
                             const real *__restrict__ grad,
                             real *__restrict__ Z2) {
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
        Z2[2 * e] = (W2[2 * e] / gu) * (xu - gu * grad[u] - Z2[2 * e]);
        Z2[2 * e + 1] = (W2[2 * e + 1] / gv) * (xv - gv * grad[v] - Z2[2 * e + 1]);
        real a = xu, b = xv, d = a - b;
        if (a < real(0)) a = -a;
        if (b < real(0)) b = -b;
        if (d < real(0)) d = -d;
        if (a < b) a = b;
        if (a < c) a = c;
        a *= condMin;
        if (d < a) d = a;
        w = La_d1[e] / d;
    }
    W2[2 * e] = w;
    W2[2 * e + 1] = w;
}

// metric of every vertex (ref :193-239 and :262-264)
template <typename real>
__global__ __launch_bounds__(256) void k_precond_vertex(
    int V, const int *__restrict__ ptr, const unsigned *__restrict__ idx,
    const real *__restrict__ W2, const real *__restrict__ diag,
    const real *__restrict__ La_l1, const R2<real> *__restrict__ xp,
    const Ctrl<real> *__restrict__ ctrl, int init, real condMin, real cap,
    const real *__restrict__ Ldiag, real *__restrict__ Ga,
    real *__restrict__ invAux, real *__restrict__ Th_l1) {
    __shared__ real lds[GatherCap<real>::v];
    const int v0 = blockIdx.x * kBlock;
    const real s = gather_sum<real, GatherCap<real>::v>(V, v0, ptr, idx, W2, lds);
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

// normalised splitting weights, prox weights and thresholds
// (ref :196-203, :241-261)
template <typename real>
__global__ void k_precond_edge2(long E, const int *__restrict__ Eu,
                                const int *__restrict__ Ev,
                                const real *__restrict__ invAux,
                                const real *__restrict__ Ga,
                                const real *__restrict__ La_d1,
                                real *__restrict__ W2,
                                real *__restrict__ Wd1u,
                                real *__restrict__ Wd1v,
                                real *__restrict__ Th, int recond,
                                const R2<real> *__restrict__ xp,
                                const real *__restrict__ grad,
                                real *__restrict__ Z2) {
    long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int u = Eu[e], v = Ev[e];
    const real wu = W2[2 * e] * invAux[u];
    const real wv = W2[2 * e + 1] * invAux[v];
    W2[2 * e] = wu;
    W2[2 * e + 1] = wv;
    const real gu = Ga[u], gv = Ga[v];
    if (recond) {
        Z2[2 * e] = xp[u].x - gu * (grad[u] + Z2[2 * e] / wu);
        Z2[2 * e + 1] = xp[v].x - gv * (grad[v] + Z2[2 * e + 1] / wv);
    }
    const real a = wu / gu, b = wv / gv, s = a + b;
    Th[e] = La_d1[e] * s / (a * b);
    Wd1u[e] = a / s;
    Wd1v[e] = b / s;
}

// CSR position of every slot: pos2[idx[j]] = j
__global__ void k_slot_positions(long n, const unsigned *__restrict__ idx,
                                 unsigned *__restrict__ pos2) {
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) pos2[idx[j]] = (unsigned)j;
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

// DR contributions W*Z: AVG_WZ writes them at wz[2e + side], AVG_SCATTER at
// their CSR position wz[pos2[2e + side]], AVG_GATHER leaves them to the
// vertex sweep
template <typename real, int MODE>
__global__ __launch_bounds__(256) void k_edge_sweep(
    long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
    const R2<real> *__restrict__ xp, real *__restrict__ Z2,
    const real *__restrict__ Wd1u, const real *__restrict__ Wd1v,
    const real *__restrict__ Th, const real *__restrict__ W2,
    real *__restrict__ wz, const unsigned *__restrict__ pos2, real rho,
    const Ctrl<real> *ctrl, int nb, int xcd) {
    constexpr bool WZ = MODE != AVG_GATHER;
    if (ctrl && ctrl->halt) return;
    constexpr int EPT = Vec<real>::kPer16B;
    const int blk = xcd_block(blockIdx.x, nb, xcd);
    if (blk >= nb) return;
    const long e0 = ((long)blk * blockDim.x + threadIdx.x) * EPT;
    if (e0 >= E) return;
    if (e0 + EPT <= E) {
        const Pk<int, EPT> iu = ldv<int, EPT>(Eu + e0);
        const Pk<int, EPT> iv = ldv<int, EPT>(Ev + e0);
        R2<real> pu[EPT], pv[EPT];
#pragma unroll
        for (int j = 0; j < EPT; j++) { pu[j] = xp[iu.v[j]]; pv[j] = xp[iv.v[j]]; }
        Pk<real, 2 * EPT> z = ldv<real, 2 * EPT>(Z2 + 2 * e0);
        const Pk<real, EPT> a = ldv<real, EPT>(Wd1u + e0);
        const Pk<real, EPT> b = ldv<real, EPT>(Wd1v + e0);
        const Pk<real, EPT> t = ldv<real, EPT>(Th + e0);
#pragma unroll
        for (int j = 0; j < EPT; j++)
            edge_update<real>(pu[j], pv[j], z.v[2 * j], z.v[2 * j + 1], a.v[j], b.v[j],
                              t.v[j], rho);
        stv<real, 2 * EPT>(Z2 + 2 * e0, z);
        if (WZ) {
            const Pk<real, 2 * EPT> w = ldv<real, 2 * EPT>(W2 + 2 * e0);
            Pk<real, 2 * EPT> out;
#pragma unroll
            for (int j = 0; j < 2 * EPT; j++) out.v[j] = w.v[j] * z.v[j];
            if (MODE == AVG_SCATTER) {
                const Pk<unsigned, 2 * EPT> p = ldv<unsigned, 2 * EPT>(pos2 + 2 * e0);
#pragma unroll
                for (int j = 0; j < 2 * EPT; j++) wz[p.v[j]] = out.v[j];
            } else if (MODE == AVG_SPLIT) {
                Pk<real, EPT> ou, ov;
#pragma unroll
                for (int j = 0; j < EPT; j++) { ou.v[j] = out.v[2 * j]; ov.v[j] = out.v[2 * j + 1]; }
                stv<real, EPT>(wz + e0, ou);
                stv<real, EPT>(wz + E + e0, ov);
            } else {
                stv<real, 2 * EPT>(wz + 2 * e0, out);
            }
        }
    } else {
        for (long e = e0; e < E; e++) {
            const R2<real> pu = xp[Eu[e]], pv = xp[Ev[e]];
            real zu = Z2[2 * e], zv = Z2[2 * e + 1];
            edge_update<real>(pu, pv, zu, zv, Wd1u[e], Wd1v[e], Th[e], rho);
            Z2[2 * e] = zu;
            Z2[2 * e + 1] = zv;
            if (WZ) {
                long iu = (MODE == AVG_SCATTER) ? (long)pos2[2 * e] : 2 * e;
                long iv = (MODE == AVG_SCATTER) ? (long)pos2[2 * e + 1] : 2 * e + 1;
                if (MODE == AVG_SPLIT) { iu = e; iv = E + e; }
                wz[iu] = W2[2 * e] * zu;
                wz[iv] = W2[2 * e + 1] * zv;
            }
        }
    }
}

template <typename real>
struct VArgs {
    int V;
    int nb, xcd;            // logical blocks, XCD-aware order
    long E;
    const int *ptr;
    const unsigned *idx;
    const real *wz;         // W*Z per slot (WZ) or W2 (products formed here)
    const real *z2;         // Z2 when the products are formed here
    R2<real> *xp;
    const real *Y, *A, *Ga, *Th_l1;
    int prox, positivity;
    real lo, hi;
    int fwd;        // 0: keep P (dense modes), 1: identity, 2: diagonal A
    int track;      // iterate-evolution partials
    real *part;     // 2 per block
    const Ctrl<real> *ctrl;
};

// DR average (ordered), prox on the iterate, evolution partials, next
// forward step (ref :491-529 then :355-464 of the next iteration)
template <typename real, int MODE>
__global__ __launch_bounds__(256) void k_vertex_sweep(VArgs<real> a) {
    if (a.ctrl && a.ctrl->halt) return;
    __shared__ real lds[GatherCap<real>::v];
    __shared__ real red[2][kBlock / kWave];
    const int blk = xcd_block(blockIdx.x, a.nb, a.xcd);
    if (blk >= a.nb) return;
    const int v0 = blk * kBlock;
    const int v = v0 + threadIdx.x;
    // per-vertex operands first: their latency hides under the gather
    R2<real> q{};
    real th = real(0), yv = real(0), gv = real(0), av = real(0);
    if (v < a.V) {
        q = a.xp[v];
        if (a.prox == PROX_L1) th = a.Th_l1[v];
        if (a.fwd) { yv = a.Y[v]; gv = a.Ga[v]; }
        if (a.fwd == 2) av = a.A[v];
    }
    real x = gather_sum<real, GatherCap<real>::v, MODE>(a.V, v0, a.ptr, a.idx, a.wz, lds, a.z2, a.E);
    real num = real(0), den = real(0);
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
        }
        q.x = x;
        if (a.fwd) {
            real p = (a.fwd == 2) ? av * x : x;
            p -= yv;
            q.y = real(2) * x - gv * p;
        }
        a.xp[v] = q;
    }
    if (a.track) {
        num = block_sum(num, red[0]);
        den = block_sum(den, red[1]);
        if (threadIdx.x == 0) {
            a.part[2 * blk] = num;
            a.part[2 * blk + 1] = den;
        }
    }
}

// iterate evolution and loop control (ref :514-529, :424-429, :447-460)
template <typename real>
__global__ __launch_bounds__(256) void k_finalize(int nparts,
                                                  const real *__restrict__ part,
                                                  Ctrl<real> *ctrl,
                                                  real *__restrict__ Dif,
                                                  int track) {
    __shared__ real red[2][kBlock / kWave];
    if (ctrl->halt) return;
    real num = real(0), den = real(0);
    if (track) {
        for (int i = threadIdx.x; i < nparts; i += kBlock) {
            num += part[2 * i];
            den += part[2 * i + 1];
        }
        num = block_sum(num, red[0]);
        den = block_sum(den, red[1]);
    }
    if (threadIdx.x != 0) return;
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

template <typename real>
__global__ __launch_bounds__(256) void k_obj_finalize(
    const real *__restrict__ part, int nbv, int nbe, int nbn, int direct,
    int has_l1, Ctrl<real> *ctrl, real *__restrict__ Obj) {
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
    if (threadIdx.x != 0) return;
    real o = direct ? real(0.5) * dat : dat;
    o += tv;
    if (has_l1) o += l1;
    const int it = ctrl ? ctrl->it : 0;
    Obj[it] = o;
    if (ctrl) ctrl->obj_it = it;
}

// ====================================================================== //
//                               session                                   //
// ====================================================================== //

template <typename real>
static void copy_in(DevBuf<real> &d, const void *src, size_t n, int mem,
                    hipStream_t s) {
    if (!src || !n) { d.release(); return; }
    d.alloc(n);
    PFDR_HIP(hipMemcpyAsync(d.p, src, n * sizeof(real),
                            mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToDevice
                                                   : hipMemcpyHostToDevice,
                            s));
}

template <typename real>
class QuadSession final : public SessionBase {
  public:
    explicit QuadSession(const pfdr_problem *p);
    int run(int iters) override;
    void result(void *X_host, int *it, void *Obj_host, void *Dif_host) override;
    void *device_x() override;

  private:
    // problem
    int flavour_;  // 0 l1, 1 bounds
    int V_, N_, mode_, itMax_, verbose_;
    long E_;
    real rho_, condMin_, difTol_, difRcd2_, cap_;
    int prox_, positivity_;
    real lo_, hi_;
    bool Ldiag_;
    bool rec_obj_, rec_dif_, track_;
    // device state
    DevBuf<int> Eu_, Ev_;
    DevBuf<real> La_d1_, La_l1_, Y_, A_, L_;
    DevBuf<R2<real>> xp_;
    DevBuf<real> diag_, Ga_, invAux_, Th_l1_, absval_, grad_, pre_, xout_;
    DevBuf<real> Z2_, W2_, Wd1u_, Wd1v_, Th_, wz_;
    int avg_ = AVG_SPLIT;  // how the DR contributions reach the vertex sweep
    int xcd_e_ = 0, xcd_v_ = 1;  // XCD-aware block order (edge / vertex sweep)
    DevBuf<unsigned> pos2_;
    DevBuf<real> R_, Rpart_, vpart_, opart_, Obj_, Dif_;
    DevBuf<int> cnt_part_;
    DevBuf<Ctrl<real>> ctrl_;
    Incidence inc_;
    Ctrl<real> *hctrl_ = nullptr;  // pinned mirror
    int nbv_, nbe_, nbn_, rows_nb_, rows_cpb_;
    int it_ = 0;
    bool stopped_ = false;
    int chunk_ = 32;
    int next_print_ = 0;

    void precondition(bool init);
    void gemv_rows(int gate);
    void forward_dense(int gate);
    void gradient();
    void objective();
    void body();
    void push_ctrl();
    void pull_ctrl();
    void print_progress();

  public:
    ~QuadSession() override {
        if (hctrl_) (void)hipHostFree(hctrl_);
    }
};

template <typename real>
QuadSession<real>::QuadSession(const pfdr_problem *p) {
    if (p->V <= 0 || p->E < 0) throw std::runtime_error("V must be > 0 and E >= 0");
    if (!p->X || !p->Y || !p->Eu || !p->Ev || !p->La_d1)
        throw std::runtime_error("X, Y, Eu, Ev and La_d1 are required");
    if (p->nranks > 1)
        throw std::runtime_error("distributed quadratic sessions go through "
                                 "pfdr_dist_* (see DESIGN.md)");
    PFDR_HIP(hipGetDevice(&device));
    stream = lib_stream();
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
    if (mode_ == A_ATA && (!p->A || -N_ != V_))
        throw std::runtime_error("N < 0 requires A = A^tA of size V-by-V and N = -V");
    rho_ = (real)p->rho;
    condMin_ = (real)p->condMin;
    difTol_ = (real)p->difTol;
    const real difRcd = (real)p->difRcd;
    difRcd2_ = difRcd * difRcd;
    rec_obj_ = p->record_obj != 0;
    rec_dif_ = p->record_dif != 0;
    track_ = (difTol_ > real(0)) || (difRcd > real(0)) || rec_dif_;
    Ldiag_ = (p->Ltype == PFDR_LIPSCHITZ_DIAG) && p->L;
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

    const int mem = p->mem;
    const size_t V = V_, E = E_;
    const auto kind = mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    Eu_.alloc(E ? E : 1);
    Ev_.alloc(E ? E : 1);
    if (E) {
        PFDR_HIP(hipMemcpyAsync(Eu_.p, p->Eu, E * sizeof(int), kind, s));
        PFDR_HIP(hipMemcpyAsync(Ev_.p, p->Ev, E * sizeof(int), kind, s));
    }
    copy_in(La_d1_, p->La_d1, E, mem, s);
    if (flavour_ == 0) copy_in(La_l1_, p->La_l1, V, mem, s);
    copy_in(Y_, p->Y, mode_ == A_DIRECT ? (size_t)N_ : V, mem, s);
    size_t asz = mode_ == A_DIRECT ? (size_t)N_ * V : mode_ == A_ATA ? V * V : mode_ == A_DIAG ? V : 0;
    copy_in(A_, p->A, asz, mem, s);
    // scalar cap of the metric (ref :225-229); computed in `real` like the reference
    real cap = real(1.9) * (real(2) - rho_);
    if (p->L && !Ldiag_) {
        real L0;
        PFDR_HIP(hipMemcpyAsync(&L0, p->L, sizeof(real),
                                mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToHost : hipMemcpyHostToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
        cap /= L0;
    }
    cap_ = cap;
    if (Ldiag_) copy_in(L_, p->L, V, mem, s);

    // iterate (X, P) pairs
    {
        DevBuf<real> X0;
        copy_in(X0, p->X, V, mem, s);
        xp_.alloc(V);
        k_xp_init<real><<<grid_for(V), kBlock, 0, s>>>(V_, X0.p, xp_.p);
        PFDR_HIP(hipGetLastError());
        PFDR_HIP(hipStreamSynchronize(s));
    }
    // edge state and per-vertex metric
    {
        // tuning knobs for A/B runs: PFDR_AVERAGE = scatter | wz | gather,
        // PFDR_XCD = <edge><vertex> bits, e.g. "01" (default)
        const char *m = getenv("PFDR_AVERAGE");
        if (m && strcmp(m, "wz") == 0) avg_ = AVG_WZ;
        else if (m && strcmp(m, "split") == 0) avg_ = AVG_SPLIT;
        else if (m && strcmp(m, "scatter") == 0) avg_ = AVG_SCATTER;
        else if (m && strcmp(m, "gather") == 0) avg_ = AVG_GATHER;
        const char *x = getenv("PFDR_XCD");
        if (x && strlen(x) == 2) { xcd_e_ = x[0] == '1'; xcd_v_ = x[1] == '1'; }
    }
    Z2_.alloc(E ? 2 * E : 1);
    W2_.alloc(E ? 2 * E : 1);
    Wd1u_.alloc(E ? E : 1); Wd1v_.alloc(E ? E : 1); Th_.alloc(E ? E : 1);
    if (avg_ != AVG_GATHER) wz_.alloc(E ? 2 * E : 1);
    diag_.alloc(V); Ga_.alloc(V); invAux_.alloc(V); absval_.alloc(V);
    if (flavour_ == 0 && p->La_l1) Th_l1_.alloc(V);
    nbv_ = grid_for(V);
    nbe_ = grid_for(E);
    nbn_ = mode_ == A_DIRECT ? grid_for(N_) : 0;
    cnt_part_.alloc(nbv_);
    vpart_.alloc(2 * (size_t)nbv_);
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
    if (mode_ == A_ATA) pre_.alloc(V);

    // control block
    ctrl_.alloc(1);
    PFDR_HIP(hipHostMalloc(&hctrl_, sizeof(Ctrl<real>), hipHostMallocDefault));
    std::memset(hctrl_, 0, sizeof(Ctrl<real>));
    const real difTol2 = difTol_ * difTol_;
    hctrl_->it = 0;
    hctrl_->obj_it = -1;
    hctrl_->itMax = itMax_;
    hctrl_->dif = difTol2 > difRcd2_ ? difTol2 : difRcd2_;  // ref :342
    hctrl_->difTol = difTol2;
    hctrl_->difRcd = difRcd2_;
    // eps (ref :285-292)
    hctrl_->eps = (real(0) < difTol_ && difTol_ < Lim<real>::eps) ? difTol_ : Lim<real>::eps;
    push_ctrl();

    // graph: ordered incidence CSR (+ the CSR position of every slot)
    build_incidence(Eu_.p, Ev_.p, V_, E_, inc_, s);
    if (avg_ == AVG_SCATTER && E_) {
        pos2_.alloc(2 * E);
        k_slot_positions<<<grid_for(2 * E_), kBlock, 0, s>>>(2 * E_, inc_.idx.p, pos2_.p);
        PFDR_HIP(hipGetLastError());
    }
    // diagonal of A^tA
    if (mode_ == A_DIRECT) {
        ColArgs<real> ca{};
        ca.A = A_.p; ca.ncols = V_; ca.len = N_; ca.out = diag_.p;
        k_col_dot<real, EPI_SELF><<<grid_for((long)V_ * 64), kBlock, 0, s>>>(ca);
    } else {
        k_diag<real><<<grid_for(V), kBlock, 0, s>>>(V_, mode_, A_.p, diag_.p);
    }
    PFDR_HIP(hipGetLastError());
    // Z = X at both ends, first preconditioning, first forward step
    if (E_) k_z_init<real><<<grid_for(E), kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, xp_.p, Z2_.p);
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
    stopped_ = (itMax_ <= 0);

    device_bytes = 0;
    auto acc = [&](size_t b) { device_bytes += (int64_t)b; };
    acc(Eu_.n * 4 + Ev_.n * 4);
    for (DevBuf<real> *b : {&La_d1_, &La_l1_, &Y_, &A_, &L_, &diag_, &Ga_, &invAux_, &Th_l1_, &absval_,
                            &pre_, &Z2_, &W2_, &Wd1u_, &Wd1v_, &Th_, &wz_, &R_, &Rpart_,
                            &vpart_, &opart_, &Obj_, &Dif_})
        acc(b->n * sizeof(real));
    acc(xp_.n * sizeof(R2<real>) + inc_.ptr.n * 4 + inc_.idx.n * 4 + pos2_.n * 4);
}

template <typename real>
void QuadSession<real>::push_ctrl() {
    PFDR_HIP(hipMemcpyAsync(ctrl_.p, hctrl_, sizeof(Ctrl<real>), hipMemcpyHostToDevice, stream));
}
template <typename real>
void QuadSession<real>::pull_ctrl() {
    PFDR_HIP(hipMemcpyAsync(hctrl_, ctrl_.p, sizeof(Ctrl<real>), hipMemcpyDeviceToHost, stream));
    PFDR_HIP(hipStreamSynchronize(stream));
}

// R = Y - A X (direct mode), gated
template <typename real>
void QuadSession<real>::gemv_rows(int gate) {
    hipStream_t s = stream;
    ProfScope ps(prof, "gemv_rows", s);
    k_rows_partial<real><<<rows_nb_, kBlock, 0, s>>>(N_, V_, A_.p, xp_.p, rows_cpb_, Rpart_.p,
                                                    gate ? ctrl_.p : nullptr, gate);
    k_rows_finish<real><<<grid_for(N_), kBlock, 0, s>>>(N_, rows_nb_, Rpart_.p, Y_.p, R_.p,
                                                       gate ? ctrl_.p : nullptr, gate);
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
        k_col_dot<real, EPI_FWD_DIRECT><<<grid_for((long)V_ * 64), kBlock, 0, s>>>(ca);
    } else {
        ca.len = V_;
        // A^tA X needs every X: read them from a compact copy
        xout_.alloc(xp_.n);
        k_x_extract<real><<<grid_for(V_), kBlock, 0, s>>>(V_, xp_.p, xout_.p);
        ca.w = xout_.p;
        ProfScope ps(prof, "symv", s);
        k_col_dot<real, EPI_FWD_ATA><<<grid_for((long)V_ * 64), kBlock, 0, s>>>(ca);
    }
    PFDR_HIP(hipGetLastError());
}

// gradient of the smooth part at the current X into grad_ (reconditioning)
template <typename real>
void QuadSession<real>::gradient() {
    hipStream_t s = stream;
    grad_.alloc(V_);
    if (mode_ == A_IDENT || mode_ == A_DIAG) {
        k_grad_vertex<real><<<grid_for(V_), kBlock, 0, s>>>(V_, mode_, A_.p, Y_.p, xp_.p, grad_.p);
    } else {
        ColArgs<real> ca{};
        ca.A = A_.p; ca.ncols = V_; ca.out = grad_.p; ca.Y = Y_.p;
        if (mode_ == A_DIRECT) {
            gemv_rows(GATE_NONE);
            ca.len = N_; ca.w = R_.p;
            k_col_dot<real, EPI_GRAD_DIRECT><<<grid_for((long)V_ * 64), kBlock, 0, s>>>(ca);
        } else {
            ca.len = V_;
            xout_.alloc(xp_.n);
            k_x_extract<real><<<grid_for(V_), kBlock, 0, s>>>(V_, xp_.p, xout_.p);
            ca.w = xout_.p;
            k_col_dot<real, EPI_GRAD_ATA><<<grid_for((long)V_ * 64), kBlock, 0, s>>>(ca);
        }
    }
    PFDR_HIP(hipGetLastError());
}

// ref :57-268 (l1) / bounds :58-242
template <typename real>
void QuadSession<real>::precondition(bool init) {
    hipStream_t s = stream;
    const size_t V = V_;
    ProfScope ps(prof, init ? "precondition" : "recondition", s);
    // amplitude scale c
    if (init && mode_ == A_DIRECT) {
        ColArgs<real> ca{};
        ca.A = A_.p; ca.ncols = V_; ca.len = N_; ca.w = Y_.p; ca.out = pre_.p; ca.div = diag_.p;
        k_col_dot<real, EPI_DIV><<<grid_for((long)V_ * 64), kBlock, 0, s>>>(ca);
    }
    k_amp<real><<<nbv_, kBlock, 0, s>>>(V_, init ? (mode_ == A_DIRECT ? 1 : 0) : 2, Y_.p, diag_.p,
                                        pre_.p, xp_.p, absval_.p, cnt_part_.p);
    k_seq_c<real><<<1, kBlock, 0, s>>>(V_, absval_.p, nbv_, cnt_part_.p, init ? 1 : 0, ctrl_.p);
    PFDR_HIP(hipGetLastError());
    if (!init) gradient();
    if (E_) {
        k_d1_weights<real><<<nbe_, kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, La_d1_.p, ctrl_.p, init ? 1 : 0,
                                                   condMin_, xp_.p, W2_.p, Ga_.p,
                                                   grad_.p, Z2_.p);
    }
    k_precond_vertex<real><<<nbv_, kBlock, 0, s>>>(V_, inc_.ptr.p, inc_.idx.p, W2_.p, diag_.p,
                                                   La_l1_.p, xp_.p, ctrl_.p, init ? 1 : 0, condMin_,
                                                   cap_, Ldiag_ ? L_.p : nullptr, Ga_.p,
                                                   invAux_.p, Th_l1_.p);
    if (E_) {
        k_precond_edge2<real><<<nbe_, kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, invAux_.p, Ga_.p, La_d1_.p,
                                                      W2_.p, Wd1u_.p, Wd1v_.p, Th_.p,
                                                      init ? 0 : 1, xp_.p, grad_.p, Z2_.p);
    }
    PFDR_HIP(hipGetLastError());
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
    if (mode_ == A_ATA) {
        ColArgs<real> ca{};
        ca.A = A_.p; ca.ncols = V_; ca.len = V_; ca.out = pre_.p;
        ca.ctrl = c; ca.gate = GATE_OBJ;
        xout_.alloc(xp_.n);
        k_x_extract<real><<<grid_for(V_), kBlock, 0, s>>>(V_, xp_.p, xout_.p);
        ca.w = xout_.p;
        k_col_dot<real, EPI_STORE><<<grid_for((long)V_ * 64), kBlock, 0, s>>>(ca);
        papp = pre_.p;
    }
    k_obj_vertex<real><<<nbv_, kBlock, 0, s>>>(V_, mode_, xp_.p, A_.p, papp, Y_.p,
                                               flavour_ == 0 ? La_l1_.p : nullptr, opart_.p, nbv_, c);
    if (E_) k_obj_edge<real><<<nbe_, kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, xp_.p, La_d1_.p, opart_.p + 2 * nbv_, c);
    if (mode_ == A_DIRECT)
        k_obj_rsq<real><<<nbn_, kBlock, 0, s>>>(N_, R_.p, opart_.p + 2 * nbv_ + nbe_, c);
    k_obj_finalize<real><<<1, kBlock, 0, s>>>(opart_.p, nbv_, E_ ? nbe_ : 0, nbn_, mode_ == A_DIRECT,
                                              flavour_ == 0 && La_l1_.p != nullptr, ctrl_.p, Obj_.p);
    PFDR_HIP(hipGetLastError());
}

template <typename real>
void QuadSession<real>::body() {
    hipStream_t s = stream;
    const bool gated = track_ || rec_obj_;
    const Ctrl<real> *c = gated ? ctrl_.p : nullptr;
    constexpr int EPT = Vec<real>::kPer16B;
    if (E_) {
        ProfScope ps(prof, "edge_sweep", s);
        const int nb = grid_for(E_, EPT), g = xcd_grid(nb, xcd_e_);
#define PFDR_EDGE(M) k_edge_sweep<real, M><<<g, kBlock, 0, s>>>(E_, Eu_.p, Ev_.p, xp_.p, Z2_.p, \
            Wd1u_.p, Wd1v_.p, Th_.p, W2_.p, wz_.p, pos2_.p, rho_, c, nb, xcd_e_)
        if (avg_ == AVG_SCATTER) PFDR_EDGE(AVG_SCATTER);
        else if (avg_ == AVG_WZ) PFDR_EDGE(AVG_WZ);
        else if (avg_ == AVG_SPLIT) PFDR_EDGE(AVG_SPLIT);
        else PFDR_EDGE(AVG_GATHER);
#undef PFDR_EDGE
    }
    {
        VArgs<real> a{};
        a.V = V_; a.ptr = inc_.ptr.p; a.idx = inc_.idx.p; a.xp = xp_.p;
        a.wz = avg_ == AVG_GATHER ? W2_.p : wz_.p;
        a.z2 = avg_ == AVG_GATHER ? Z2_.p : nullptr;
        a.Y = Y_.p; a.A = A_.p; a.Ga = Ga_.p; a.Th_l1 = Th_l1_.p;
        a.prox = prox_; a.positivity = positivity_; a.lo = lo_; a.hi = hi_;
        a.fwd = mode_ == A_IDENT ? 1 : (mode_ == A_DIAG ? 2 : 0);
        a.track = track_ ? 1 : 0; a.part = vpart_.p; a.ctrl = c;
        a.nb = nbv_; a.xcd = xcd_v_;
        const int g = xcd_grid(nbv_, xcd_v_);
        ProfScope ps(prof, "vertex_sweep", s);
        a.E = E_;
        if (avg_ == AVG_SCATTER) k_vertex_sweep<real, AVG_SCATTER><<<g, kBlock, 0, s>>>(a);
        else if (avg_ == AVG_WZ) k_vertex_sweep<real, AVG_WZ><<<g, kBlock, 0, s>>>(a);
        else if (avg_ == AVG_SPLIT) k_vertex_sweep<real, AVG_SPLIT><<<g, kBlock, 0, s>>>(a);
        else k_vertex_sweep<real, AVG_GATHER><<<g, kBlock, 0, s>>>(a);
    }
    if (gated) {
        k_finalize<real><<<1, kBlock, 0, s>>>(nbv_, vpart_.p, ctrl_.p, rec_dif_ ? Dif_.p : nullptr,
                                              track_ ? 1 : 0);
    }
    PFDR_HIP(hipGetLastError());
    if (mode_ == A_DIRECT || mode_ == A_ATA) forward_dense(gated ? GATE_ACTIVE : GATE_NONE);
    if (rec_obj_) objective();
}

template <typename real>
void QuadSession<real>::print_progress() {
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
    while (!stopped_ && it_ < target) {
        const int n = std::min(target - it_, chunk_);
        for (int i = 0; i < n; i++) body();
        if (gated) {
            pull_ctrl();
            it_ = hctrl_->it;
            if (hctrl_->stop) {
                stopped_ = true;
            } else if (hctrl_->recond) {
                if (verbose_) { print_progress(); printf("Reconditioning... "); fflush(stdout); }
                precondition(false);
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
    PFDR_HIP(hipStreamSynchronize(stream));
    if (prof.on) prof.resolve();
    return it_;
}

template <typename real>
void *QuadSession<real>::device_x() {
    xout_.alloc(xp_.n);
    k_x_extract<real><<<grid_for(V_), kBlock, 0, stream>>>(V_, xp_.p, xout_.p);
    PFDR_HIP(hipGetLastError());
    PFDR_HIP(hipStreamSynchronize(stream));
    return xout_.p;
}

template <typename real>
void QuadSession<real>::result(void *X_host, int *it, void *Obj_host, void *Dif_host) {
    hipStream_t s = stream;
    if (X_host) {
        void *dx = device_x();
        PFDR_HIP(hipMemcpyAsync(X_host, dx, sizeof(real) * V_, hipMemcpyDeviceToHost, s));
    }
    if (it) *it = it_;
    if (Obj_host && rec_obj_)
        PFDR_HIP(hipMemcpyAsync(Obj_host, Obj_.p, sizeof(real) * (it_ + 1), hipMemcpyDeviceToHost, s));
    if (Dif_host && rec_dif_ && it_ > 0)
        PFDR_HIP(hipMemcpyAsync(Dif_host, Dif_.p, sizeof(real) * it_, hipMemcpyDeviceToHost, s));
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
    p.dtype = sizeof(real) == 4 ? PFDR_F32 : PFDR_F64;
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
        if (verbose) { printf("Initializing constants and variables... "); fflush(stdout); }
        std::unique_ptr<QuadSession<real>> s(new QuadSession<real>(&p));
        if (verbose) { printf("done.\nPreconditioned forward-Douglas-Rachford algorithm\n"); fflush(stdout); }
        s->run(itMax);
        int its = 0;
        s->result(X, &its, Obj, Dif);
        if (it) *it = its;
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
