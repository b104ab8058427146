// MI355X PFDR solver for
//     F(p) = f(p; q) + sum_{e,k} la_e |p_uk - p_vk| + i_simplex(p)
// (linear, quadratic or smoothed Kullback-Leibler loss), the algorithm of
// reference src/PFDR_graph_loss_d1_simplex.cpp:372-715, and the metric
// simplex projection of src/proj_simplex_metric.cpp:18-83.
//
//   per iteration:
//     k_sx_edge_sweep   : K-wide TV prox on every (edge, label) + relaxed Z
//                         update                              ref :589-634
//     k_sx_vertex_sweep : (K <= 64) ordered per-(vertex, label) DR average
//                         over the incidence CSR, W*Z formed from Z (the
//                         reference parallelises it over labels only,
//                         :636-648), per-vertex metric simplex projection,
//                         evolution partials (l1 or label changes) and the
//                         NEXT explicit step FP          ref :651-691, :567-587
//     k_sx_vertex_wide  : (K > 64) the same, one wave per vertex: coalesced
//                         K-runs, sums in registers, the projection on the
//                         whole wave (pfdr_proj.hpp); K > 1024 in memory
//     k_sx_finalize     : stop / recondition flags (when tracked)
// Layouts: P, Q, Ga, GaQ are K-by-V (index v*K + k) as in the reference; the
// explicit step FP lives next to P in (P, FP) pairs PF[v*K + k] and the
// splitting-weight factors in (Ga, 1/Aux) pairs GI[v*K + k], so the edge
// sweep (bound by its texture-address work, not by bytes) gathers each end
// with one 16-byte access per operand pair; edge state is K-by-E; the
// preconditioner's weight sums run over wz[side][e][k].
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>

#include "pfdr_graph.hpp"
#include "pfdr_halo.hpp"
#include "pfdr_monosum.hpp"
#include "pfdr_proj.hpp"
#include "pfdr_session.hpp"
#include "pfdr_sort.hpp"

namespace pfdr {

enum Loss : int { LOSS_LINEAR = 0, LOSS_QUAD = 1, LOSS_KL = 2 };

template <typename real>
struct SxConst {
    int K;
    int loss;
    real alK, al1, alKal1;
};

template <typename real> using SxR2 = typename Vec<real>::v2;

// Splitting weights as factors (ref :199-239): Wu[e*K+k] = a * Aux[u]^-1,
// a = La_d1[e] at the first conditioning, La_d1[e] / d at a
// reconditioning.  Only a (A1, one real per (e, k), after a
// reconditioning) and the per-(v, k) (Ga, 1/Aux) pairs (GI, Ga before its
// normalisation by the vertex maximum, ref :360-369) are kept; every
// product a * invAux is the reference's own operation.
template <typename real>
__device__ __forceinline__ real sx_a(long i, long e, const real *__restrict__ A1,
                                     const real *__restrict__ La_d1) {
    return A1 ? A1[i] : La_d1[e];
}

// prox weights and threshold (ref :287-306), operation for operation
template <typename real>
__device__ __forceinline__ void sx_prox_ab(real a, real b, real la, real &du, real &dv, real &th) {
    const real s = a + b;
    th = la * s / (a * b);
    du = a / s;
    dv = b / s;
}
template <typename real>
__device__ __forceinline__ void sx_prox_weights(real wu, real wv, real gu, real gv, real la,
                                                real &du, real &dv, real &th) {
    sx_prox_ab(wu / gu, wv / gv, la, du, dv, th);
}

// ------------------------------------------------ metric projection ----
// The metric simplex projection's sweep (ref src/proj_simplex_metric.cpp:41-80)
// down a column of LDS (stride `st` between coordinates),
// split for the group vertex sweep (k_sx_vertex_group): the coordinates
// arrive already divided by their metric (x[d] / m[d], the reference's own
// division, done by the item lanes) with the raw x[0] beside them, the
// active set goes to bytes I[d * st], and the final threshold is returned --
// the item lanes then form (x - la) m or 0 in parallel (ref :74-80).  The
// walk itself is the reference's sequence of comparisons and updates
// (ref :43-72), the next coordinate's loads issued before the current one's
// arithmetic.
template <typename real>
__device__ real proj_simplex_walk(const real *x, const real *m, unsigned char *I, int D, int st,
                                  real x0, real a) {
    const real m0 = m[0];
    real la = (x0 - a) / m0;
    real s = m0;
    I[0] = 1;
    real xn = D > 1 ? x[st] : real(0), mn = D > 1 ? m[st] : real(1);
    for (int d = 1; d < D; d++) {  // first pass (ref :48-57)
        const real xd = xn, md = mn;
        if (d + 1 < D) { xn = x[(d + 1) * st]; mn = m[(d + 1) * st]; }
        unsigned char in = 0;
        if (xd > la) {
            in = 1;
            s += md;
            la += md * (xd - la) / s;
        }
        I[d * st] = in;
    }
    bool changed = true;
    while (changed) {  // later passes (ref :59-72)
        changed = false;
        unsigned char in_n = I[0];
        real xm = x[0];
        for (int d = 0; d < D; d++) {
            const unsigned char in = in_n;
            const real xd = xm;
            if (d + 1 < D) { in_n = I[(d + 1) * st]; xm = x[(d + 1) * st]; }
            if (in && xd < la) {
                I[d * st] = 0;
                const real md = m[d * st];
                s -= md;
                la += md * (la - xd) / s;
                changed = true;
            }
        }
    }
    return la;
}

// Projection of x (D <= 64 values, stride 1, in LDS) onto {x >= 0, sum x = a}
// in the metric diag(1/m) by one lane: the active-set sweep of ref
// src/proj_simplex_metric.cpp:41-80, operation for operation, the active
// set in a register bit mask.  Used by the fused vertex sweep (K <= 64),
// whose vertices pack the lanes densely.
template <typename real>
__device__ void proj_simplex_column(real *x, const real *m, int D, real a) {
    unsigned long long act = 1ull;
    real la = (x[0] - a) / m[0];
    x[0] = x[0] / m[0];
    real s = m[0];
    for (int d = 1; d < D; d++) {
        const real md = m[d];
        const real xd = x[d] / md;
        x[d] = xd;
        if (xd > la) {
            act |= 1ull << d;
            s += md;
            la += md * (xd - la) / s;
        }
    }
    bool changed = true;
    while (changed) {
        changed = false;
        for (int d = 0; d < D; d++) {
            if ((act >> d) & 1ull) {
                const real xd = x[d];
                if (xd < la) {
                    act &= ~(1ull << d);
                    const real md = m[d];
                    s -= md;
                    la += md * (la - xd) / s;
                    changed = true;
                }
            }
        }
    }
    for (int d = 0; d < D; d++) x[d] = ((act >> d) & 1ull) ? (x[d] - la) * m[d] : real(0);
}

// The same projection with the coordinates already divided by their metric
// (x[d] / m[d], the reference's division, done in parallel by the item
// lanes) and the raw x[0] aside: the walk keeps only the active-set
// updates' divisions (bit-identical to proj_simplex_column)
template <typename real>
__device__ void proj_simplex_column_div(real *x, const real *m, int D, real x0, real a) {
    unsigned long long act = 1ull;
    real la = (x0 - a) / m[0];
    real s = m[0];
    for (int d = 1; d < D; d++) {
        const real xd = x[d];
        if (xd > la) {
            const real md = m[d];
            act |= 1ull << d;
            s += md;
            la += md * (xd - la) / s;
        }
    }
    bool changed = true;
    while (changed) {
        changed = false;
        for (int d = 0; d < D; d++) {
            if ((act >> d) & 1ull) {
                const real xd = x[d];
                if (xd < la) {
                    act &= ~(1ull << d);
                    const real md = m[d];
                    s -= md;
                    la += md * (la - xd) / s;
                    changed = true;
                }
            }
        }
    }
    for (int d = 0; d < D; d++) x[d] = ((act >> d) & 1ull) ? (x[d] - la) * m[d] : real(0);
}

// ------------------------------------------------------------- kernels --
template <typename real>
__global__ void k_sx_z_init(long EK, int K, const int *__restrict__ Eu,
                            const int *__restrict__ Ev,
                            const real *__restrict__ P, real *__restrict__ Zu,
                            real *__restrict__ Zv) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= EK) return;
    const long e = i / K;
    const int k = (int)(i - e * K);
    Zu[i] = P[(long)Eu[e] * K + k];
    Zv[i] = P[(long)Ev[e] * K + k];
}

// reconditioning, step 1: retrieve the metric before its normalisation
// (ref :92-135).  One thread per vertex.
template <typename real>
__global__ void k_sx_recover(int V, SxConst<real> c, const real *__restrict__ La_f,
                             const real *__restrict__ Q,
                             const real *__restrict__ GaQ,
                             real *__restrict__ Ga) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const int K = c.K;
    const long b = (long)v * K;
    if (c.loss == LOSS_QUAD) {
        if (!La_f) {
            for (int k = 0; k < K; k++) Ga[b + k] = GaQ[b + k];
        } else {
            const real s = real(1) / La_f[v];
            for (int k = 0; k < K; k++) Ga[b + k] = s * GaQ[b + k];
        }
    } else if (c.loss == LOSS_KL) {
        if (!La_f) {
            for (int k = 0; k < K; k++) Ga[b + k] = GaQ[b + k] / (c.alK + c.al1 * Q[b + k]);
        } else {
            const real s = real(1) / La_f[v];
            for (int k = 0; k < K; k++) Ga[b + k] = s * GaQ[b + k] / (c.alK + c.al1 * Q[b + k]);
        }
    } else {
        int imax = 0;
        real qmax = Q[b];
        for (int k = 1; k < K; k++) {
            if (qmax < Q[b + k]) { qmax = Q[b + k]; imax = k; }
        }
        const real s = GaQ[b + imax] / qmax / Ga[b + imax];
        for (int k = 0; k < K; k++) Ga[b + k] *= s;
    }
}

// reconditioning, step 2: auxiliary variables -> subgradients (ref :136-156)
// with the OLD weights a * invAux (A1old null: a = La_d1)
template <typename real>
__global__ void k_sx_subgrad(long EK, SxConst<real> c, const int *__restrict__ Eu,
                             const int *__restrict__ Ev,
                             const real *__restrict__ P,
                             const real *__restrict__ Q,
                             const real *__restrict__ Ga,
                             const real *__restrict__ GaQ,
                             const real *__restrict__ A1old,
                             const real *__restrict__ La_d1,
                             const real *__restrict__ invAux,
                             real *__restrict__ Zu, real *__restrict__ Zv) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= EK) return;
    const int K = c.K;
    const long e = i / K;
    const int k = (int)(i - e * K);
    const long u = (long)Eu[e] * K + k, v = (long)Ev[e] * K + k;
    const real a0 = sx_a(i, e, A1old, La_d1);
    const real wu = a0 * invAux[u], wv = a0 * invAux[v];
    if (c.loss == LOSS_LINEAR) {
        Zu[i] = (wu / Ga[u]) * (P[u] + GaQ[u] - Zu[i]);
        Zv[i] = (wv / Ga[v]) * (P[v] + GaQ[v] - Zv[i]);
    } else if (c.loss == LOSS_QUAD) {
        Zu[i] = (wu / Ga[u]) * (P[u] - GaQ[u] * (P[u] - Q[u]) - Zu[i]);
        Zv[i] = (wv / Ga[v]) * (P[v] - GaQ[v] * (P[v] - Q[v]) - Zv[i]);
    } else {
        Zu[i] = (wu / Ga[u]) * (P[u] + GaQ[u] / (c.alKal1 + P[u]) - Zu[i]);
        Zv[i] = (wv / Ga[v]) * (P[v] + GaQ[v] / (c.alKal1 + P[v]) - Zv[i]);
    }
}

// Hessian of the loss (ref :159-190), one thread per (v, k)
template <typename real>
__global__ void k_sx_hessian(long VK, SxConst<real> c, const real *__restrict__ La_f,
                             const real *__restrict__ P,
                             const real *__restrict__ Q,
                             real *__restrict__ Ga) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= VK) return;
    if (c.loss == LOSS_LINEAR) {
        Ga[i] = real(0);
    } else if (c.loss == LOSS_QUAD) {
        Ga[i] = La_f ? La_f[i / c.K] : real(1);
    } else {
        const real t = c.alKal1 + P[i];
        if (La_f) Ga[i] = La_f[i / c.K] * (c.alK + c.al1 * Q[i]) / (t * t);
        else Ga[i] = (c.alK + c.al1 * Q[i]) / (t * t);
    }
}

// d1 splitting weights a (ref :192-221) into both contribution slots (the
// per-(v, k) sums run through the CSR); on reconditioning also into A1
template <typename real>
__global__ void k_sx_d1_weights(long EK, int K, const int *__restrict__ Eu,
                                const int *__restrict__ Ev,
                                const real *__restrict__ La_d1, int init,
                                real condMin, const real *__restrict__ P,
                                real *__restrict__ A1, real *__restrict__ wz) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= EK) return;
    const long e = i / K;
    const int k = (int)(i - e * K);
    real w;
    if (init) {
        w = La_d1[e];
    } else {
        real a = P[(long)Eu[e] * K + k] - P[(long)Ev[e] * K + k];
        if (a < real(0)) a = -a;
        if (a < condMin) a = condMin;
        w = La_d1[e] / a;
        A1[i] = w;
    }
    wz[i] = w;
    wz[EK + i] = w;
}

// ordered per-(v, k) sum over the contribution CSR (pfdr_halo.hpp): the
// entry of address a (e: u end, E + e: v end, 2E + j: received) lives at
// wz[a*K + k] — wz is [side][e][k] followed by the received tail
template <typename real>
__device__ __forceinline__ real sx_gather(long i, int K, const int *__restrict__ ptr,
                                          const unsigned *__restrict__ idx,
                                          const real *__restrict__ wz) {
    const long v = i / K;
    const int k = (int)(i - v * K);
    const int j0 = ptr[v], j1 = ptr[v + 1];
    real s = real(0);
    for (int j = j0; j < j1; j++) s += wz[(long)idx[j] * K + k];
    return s;
}

// metric of every (v, k), prox weights input and first-order information
// (ref :192-285 per element, :307-335)
template <typename real>
__global__ void k_sx_precond_vertex(long VK, SxConst<real> c,
                                    const int *__restrict__ ptr,
                                    const unsigned *__restrict__ idx,
                                    const real *__restrict__ wz,
                                    const real *__restrict__ La_f,
                                    const real *__restrict__ Q, real cap,
                                    real *__restrict__ Ga,
                                    real *__restrict__ invAux,
                                    real *__restrict__ GaQ) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= VK) return;
    const int K = c.K;
    const real s = sx_gather(i, K, ptr, idx, wz);
    real g;
    if (c.loss == LOSS_LINEAR) {
        // Ga itself accumulated the weights from zero, then was inverted
        g = real(1) / s;
        invAux[i] = g;
    } else {
        g = Ga[i];
        g += s;
        invAux[i] = real(1) / s;
        g = real(1) / g;
    }
    const long v = i / K;
    // cap by the Lipschitz constant of the loss (ref :249-285)
    if (c.loss == LOSS_QUAD) {
        if (La_f) {
            const real cv = cap / La_f[v];
            if (g > cv) g = cv;
        } else if (cap < real(1)) {
            if (g > cap) g = cap;
        }
    } else if (c.loss == LOSS_KL) {
        real b;
        if (!La_f) b = real(1) / (c.alKal1 * c.alKal1);
        else b = La_f[v] * real(1) / (c.alKal1 * c.alKal1);
        const real cv = cap / ((c.alK + c.al1 * Q[i]) * b);
        if (g > cv) g = cv;
    }
    Ga[i] = g;
    // metric times first-order information (ref :307-335)
    if (c.loss == LOSS_LINEAR) {
        GaQ[i] = g * Q[i];
    } else if (c.loss == LOSS_QUAD) {
        GaQ[i] = La_f ? La_f[v] * g : g;
    } else {
        GaQ[i] = La_f ? La_f[v] * g * (c.alK + c.al1 * Q[i]) : g * (c.alK + c.al1 * Q[i]);
    }
}

// reconditioning: subgradients -> auxiliary variables with the new weights
// (ref :337-358)
template <typename real>
__global__ void k_sx_recond_edge(long EK, SxConst<real> c, const int *__restrict__ Eu,
                                 const int *__restrict__ Ev, const real *__restrict__ A1,
                                 const real *__restrict__ invAux,
                                 const real *__restrict__ Ga,
                                 const real *__restrict__ GaQ,
                                 const real *__restrict__ P,
                                 const real *__restrict__ Q,
                                 real *__restrict__ Zu, real *__restrict__ Zv) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= EK) return;
    const int K = c.K;
    const long e = i / K;
    const int k = (int)(i - e * K);
    const long u = (long)Eu[e] * K + k, v = (long)Ev[e] * K + k;
    const real wu = A1[i] * invAux[u];
    const real wv = A1[i] * invAux[v];
    if (c.loss == LOSS_LINEAR) {
        Zu[i] = P[u] + GaQ[u] - (Ga[u] / wu) * Zu[i];
        Zv[i] = P[v] + GaQ[v] - (Ga[v] / wv) * Zv[i];
    } else if (c.loss == LOSS_QUAD) {
        Zu[i] = P[u] - GaQ[u] * (P[u] - Q[u] + Zu[i] / wu);
        Zv[i] = P[v] - GaQ[v] * (P[v] - Q[v] + Zv[i] / wv);
    } else {
        Zu[i] = P[u] + GaQ[u] / (c.alKal1 + P[u]) - (Ga[u] / wu) * Zu[i];
        Zv[i] = P[v] + GaQ[v] / (c.alKal1 + P[v]) - (Ga[v] / wv) * Zv[i];
    }
}

// stored prox weights and thresholds (ref :287-306) from the factored
// splitting weights
template <typename real>
__global__ void k_sx_prox_store(long EK, int K, const int *__restrict__ Eu,
                                const int *__restrict__ Ev, const real *__restrict__ A1,
                                const real *__restrict__ La_d1,
                                const SxR2<real> *__restrict__ GI, real *__restrict__ Wd1u,
                                real *__restrict__ Wd1v, real *__restrict__ Th) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= EK) return;
    const long e = i / K;
    const int k = (int)(i - e * K);
    const SxR2<real> gu = GI[(long)Eu[e] * K + k], gv = GI[(long)Ev[e] * K + k];
    const real la = La_d1[e], a = sx_a(i, e, A1, La_d1);
    sx_prox_weights<real>(a * gu.y, a * gv.y, gu.x, gv.x, la, Wd1u[i], Wd1v[i], Th[i]);
}

// (Ga, invAux) pairs of every (v, k), owned and ghost, before the metric
// is normalised
template <typename real>
__global__ void k_sx_gi_pack(long n, const real *__restrict__ Ga, const real *__restrict__ invAux,
                             SxR2<real> *__restrict__ GI, real *__restrict__ GaU) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SxR2<real> q;
    q.x = Ga[i];
    q.y = invAux[i];
    GI[i] = q;
    if (GaU) GaU[i] = q.x;
}

// normalise the metric of each vertex by its maximum (ref :360-369)
template <typename real>
__global__ void k_sx_normalise(int V, int K, real *__restrict__ Ga) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const long b = (long)v * K;
    real mx = Ga[b];
    for (int k = 1; k < K; k++) if (Ga[b + k] > mx) mx = Ga[b + k];
    for (int k = 0; k < K; k++) Ga[b + k] /= mx;
}

// explicit step FP (ref :567-587)
template <typename real>
__device__ __forceinline__ real sx_explicit(const SxConst<real> &c, real p,
                                            real gaq, real q) {
    if (c.loss == LOSS_LINEAR) return real(2) * p + gaq;
    if (c.loss == LOSS_QUAD) return real(2) * p - gaq * (p - q);
    return real(2) * p + gaq / (c.alKal1 + p);
}

template <typename real>
__global__ void k_sx_explicit(long VK, SxConst<real> c,
                              const real *__restrict__ P,
                              const real *__restrict__ GaQ,
                              const real *__restrict__ Q,
                              SxR2<real> *__restrict__ PF) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= VK) return;
    SxR2<real> q;
    q.x = P[i];
    q.y = sx_explicit(c, q.x, GaQ[i], Q[i]);
    PF[i] = q;
}

// labels of the maximum-likelihood class (ref :447-466)
template <typename real>
__global__ void k_sx_labels(int V, int K, const real *__restrict__ P,
                            real *__restrict__ lab) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const long b = (long)v * K;
    real a = P[b];
    real l = real(0);
    for (int k = 1; k < K; k++) {
        if (P[b + k] > a) { a = P[b + k]; l = (real)k; }
    }
    lab[v] = l;
}

// --------------------------------------------------------- iteration ---
// TV prox + relaxed Z update of one (edge, label) (ref :589-634)
template <typename real>
__device__ __forceinline__ void sx_edge_elem(const SxConst<real> &c, real fpu, real fpv, real pu,
                                             real pv, real &zu, real &zv, real wu, real wv, real th,
                                             real rho) {
    real a = fpu - zu;
    const real b = fpv - zv;
    if (c.loss == LOSS_LINEAR) {
        const real h = real(0.5) * (a + b);
        a = a - b;
        if (a > real(2)) {
            a = real(0.5) * (a - real(2));
            zu += rho * (h + a - pu);
            zv += rho * (h - a - pv);
        } else if (a < real(-2)) {
            a = real(0.5) * (a + real(2));
            zu += rho * (h + a - pu);
            zv += rho * (h - a - pv);
        } else {
            zu += rho * (h - pu);
            zv += rho * (h - pv);
        }
    } else {
        const real h = wu * a + wv * b;
        a = a - b;
        if (a > th) {
            a -= th;
            zu += rho * (h + wv * a - pu);
            zv += rho * (h - wu * a - pv);
        } else if (a < -th) {
            a += th;
            zu += rho * (h + wv * a - pu);
            zv += rho * (h - wu * a - pv);
        } else {
            zu += rho * (h - pu);
            zv += rho * (h - pv);
        }
    }
}

template <typename T, int N>
__device__ __forceinline__ Pk<T, N> sx_ld(const T *p) { return *reinterpret_cast<const Pk<T, N> *>(p); }
template <typename T, int N>
__device__ __forceinline__ void sx_st(T *p, const Pk<T, N> &x) { *reinterpret_cast<Pk<T, N> *>(p) = x; }

// L consecutive (edge, label) entries per lane (L = 2 when K is even: the
// pair shares its edge, so every stream and the four K-run gathers move as
// 8-byte (f32) / 16-byte (f64) accesses, and the endpoint loads and the
// index division are paid once per pair)
// one lane's L entries [i, i + L) of the (edge, label) sweep, i < EK: the
// body of k_sx_edge_sweep, shared with the one-workgroup k_sx_tiny_iterate
// one GPU before any reconditioning: 1/Aux is one value per vertex
// (invV, SxVArgs::invV) and La_d1 may be one value (la0), so the lane reads
// the metric alone per (v, k) (GaU: Ga before its normalisation, 4 B)
// instead of the (Ga, 1/Aux) pair (8 B) at each end; GaU null: off
// AW (one La_d1 value as well): the ratio W / Ga = (la0 * 1/Aux[v]) /
// Ga[v, k] of every (v, k), formed once with the reference's operations
// (k_sx_aw) -- the same for every edge at v, so the lane divides only for
// the threshold and the two weights (3 IEEE divisions per entry, not 5)
template <typename real>
struct SxEdgeFast {
    const real *GaU, *invV, *AW;
    real la0;
    int la_u;
};

template <typename real>
__global__ void k_sx_aw(long n, int K, real la0, const real *__restrict__ invV,
                        const real *__restrict__ GaU, real *__restrict__ AW) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) AW[i] = (la0 * invV[i / K]) / GaU[i];
}

template <typename real, int L>
__device__ __forceinline__ void sx_edge_lane(
    long i, long EK, const SxConst<real> &c, const int *__restrict__ Eu,
    const int *__restrict__ Ev, const SxR2<real> *PF, real *Zu, real *Zv,
    const real *__restrict__ A1, const real *__restrict__ La_d1,
    const SxR2<real> *__restrict__ GI, const real *__restrict__ Wd1u,
    const real *__restrict__ Wd1v, const real *__restrict__ Th, real *wz, real rho,
    SxEdgeFast<real> f = SxEdgeFast<real>{}) {
    const int K = c.K;
    long e;
    int k;
    if (EK <= 0xffffffffl) {  // 32-bit division (uniform branch)
        const unsigned ue = (unsigned)i / (unsigned)K;
        e = ue;
        k = (int)((unsigned)i - ue * (unsigned)K);
    } else {
        e = i / K;
        k = (int)(i - e * K);
    }
    const int eu = Eu[e], ev = Ev[e];
    const long u = (long)eu * K + k, v = (long)ev * K + k;
    Pk<real, L> zu = sx_ld<real, L>(Zu + i), zv = sx_ld<real, L>(Zv + i);
    // (P, explicit step) of both entries in one access per end: the sweep
    // is bound by its texture-address work (profiles/r2/r2zj_c4_counters)
    const Pk<SxR2<real>, L> qu = sx_ld<SxR2<real>, L>(PF + u), qv = sx_ld<SxR2<real>, L>(PF + v);
    Pk<real, L> fpu, fpv, pu, pv;
#pragma unroll
    for (int j = 0; j < L; j++) {
        pu.v[j] = qu.v[j].x; fpu.v[j] = qu.v[j].y;
        pv.v[j] = qv.v[j].x; fpv.v[j] = qv.v[j].y;
    }
    // splitting weights from their factors (prox weights: non-linear losses
    // without stored ones; contributions: only when this sweep stores W*Z)
    real wsu[L], wsv[L], gpu[L], gpv[L], la = real(0);
#pragma unroll
    for (int j = 0; j < L; j++) { wsu[j] = wsv[j] = real(0); gpu[j] = gpv[j] = real(1); }
    if ((c.loss != LOSS_LINEAR && !Th) || wz) {
        la = f.la_u ? f.la0 : La_d1[e];
        if (f.AW && !A1 && !wz) {
            // (the ratios AW below replace the weights and the metric)
        } else if (f.GaU && !A1) {  // (the metric per (v, k), 1/Aux per vertex)
            const Pk<real, L> gu_ = sx_ld<real, L>(f.GaU + u), gv_ = sx_ld<real, L>(f.GaU + v);
            const real iu = f.invV[eu], iv = f.invV[ev];
#pragma unroll
            for (int j = 0; j < L; j++) {
                wsu[j] = la * iu;
                wsv[j] = la * iv;
                gpu[j] = gu_.v[j];
                gpv[j] = gv_.v[j];
            }
        } else {
            // (Ga, 1/Aux) of both entries of a pair in one access at each end
            // (u, v even: K is even when L = 2) -- the sweep is bound by its
            // texture-address work, not by bytes (profiles/r2/r2zj_c4_counters)
            const Pk<SxR2<real>, L> gpu_ = sx_ld<SxR2<real>, L>(GI + u);
            const Pk<SxR2<real>, L> gpv_ = sx_ld<SxR2<real>, L>(GI + v);
#pragma unroll
            for (int j = 0; j < L; j++) {
                const real an = A1 ? A1[i + j] : la;
                const SxR2<real> gu = gpu_.v[j], gv = gpv_.v[j];
                wsu[j] = an * gu.y;
                wsv[j] = an * gv.y;
                gpu[j] = gu.x;
                gpv[j] = gv.x;
            }
        }
    }
    Pk<real, L> du{}, dv{}, th{};
    if (c.loss != LOSS_LINEAR && f.AW && !A1 && !Th) {  // (wsu / gpu never formed)
        const Pk<real, L> au = sx_ld<real, L>(f.AW + u), av = sx_ld<real, L>(f.AW + v);
#pragma unroll
        for (int j = 0; j < L; j++) sx_prox_ab<real>(au.v[j], av.v[j], la, du.v[j], dv.v[j], th.v[j]);
    } else if (c.loss != LOSS_LINEAR) {
        if (Th) {
            du = sx_ld<real, L>(Wd1u + i);
            dv = sx_ld<real, L>(Wd1v + i);
            th = sx_ld<real, L>(Th + i);
        } else {
#pragma unroll
            for (int j = 0; j < L; j++)
                sx_prox_weights<real>(wsu[j], wsv[j], gpu[j], gpv[j], la, du.v[j], dv.v[j], th.v[j]);
        }
    }
#pragma unroll
    for (int j = 0; j < L; j++)
        sx_edge_elem<real>(c, fpu.v[j], fpv.v[j], pu.v[j], pv.v[j], zu.v[j], zv.v[j], du.v[j],
                           dv.v[j], th.v[j], rho);
    sx_st<real, L>(Zu + i, zu);
    sx_st<real, L>(Zv + i, zv);
    if (wz) {
#pragma unroll
        for (int j = 0; j < L; j++) {
            wz[i + j] = wsu[j] * zu.v[j];
            wz[EK + i + j] = wsv[j] * zv.v[j];
        }
    }
}

template <typename real, int L>
__global__ __launch_bounds__(256) void k_sx_edge_sweep(
    long EK, SxConst<real> c, const int *__restrict__ Eu,
    const int *__restrict__ Ev, const SxR2<real> *__restrict__ PF,
    real *__restrict__ Zu, real *__restrict__ Zv,
    const real *__restrict__ A1, const real *__restrict__ La_d1,
    const SxR2<real> *__restrict__ GI, const real *__restrict__ Wd1u,
    const real *__restrict__ Wd1v, const real *__restrict__ Th, real *__restrict__ wz, real rho,
    const Ctrl<real> *ctrl, int nb, int xcd, SxEdgeFast<real> f) {
    if (ctrl && ctrl->halt) return;
    const int blk = xcd_block(blockIdx.x, nb, xcd);
    if (blk >= nb) return;
    const long i = ((long)blk * blockDim.x + threadIdx.x) * L;
    if (i >= EK) return;
    sx_edge_lane<real, L>(i, EK, c, Eu, Ev, PF, Zu, Zv, A1, La_d1, GI, Wd1u, Wd1v, Th, wz, rho, f);
}

// Fused vertex sweep (K <= 64): ordered DR average, metric projection,
// evolution partials and the next explicit step in one pass.  A block owns
// vb = floor(256 / K) consecutive vertices and gives each (vertex, label)
// one lane: the lanes of a vertex read its incidence list together (one
// broadcast load of the slot, then K contiguous contributions, so each
// gathered edge costs one 4K-byte run instead of K scattered words), the
// sums meet in LDS where one lane per vertex runs the projection of
// ref src/proj_simplex_metric.cpp:41-80, and the lanes write P and FP back
// coalesced.  Summation order per (v, k) is increasing slot 2e + side, as in
// the reference's sequential average (ref :636-648).
template <typename real>
struct SxVArgs {
    int V, vb;
    int nb, xcd;  // blocks, XCD-aware order
    long E;
    SxConst<real> c;
    const int *ptr;
    const unsigned *idx;
    const real *wz, *Ga, *GaQ, *Q;
    const real *Zu, *Zv;  // !WZ: contributions W*Z formed in the sweep from
    const real *A1, *La_d1;  // the factors of W (sx_a) and the vertex's invAux
    const real *invAux;      // (read alone: GI's Ga half is the edge sweep's)
    real *P, *lab;
    SxR2<real> *PF;          // (P, explicit step) pairs: the edge sweep's operands
    int track;
    real *part;
    const Ctrl<real> *ctrl;
    real *terms;  // sequential evolution (null: off): |P_ - P| per (v, k) or 0/1 per v
    real *Po;          // where the new P and (P, step) go (null: P, PF in place)
    SxR2<real> *PFo;
    real *xs;            // wide sweep, K > 1024: the averages, projected in place
    unsigned char *act;  // its active flags (one byte per (v, k))
    // 1/Aux per VERTEX (null: per (v, k) in invAux): before any reconditioning
    // every label of a vertex sums the same weights La_d1[e] in the same
    // order (ref :196-217), so its K values are one value
    const real *invV;
    real la0;  // La_d1 when it is one value for every edge (la_u), before A1
    int la_u;
    // P lives in the .x half of PF only (no P store; the evolution reads
    // the old P from PF; SimplexSession::sync_p extracts it when asked)
    int nop;
    // tile-ordered sessions (sx_tile_sum): per vertex block a 32-int record
    // of its runs (null: no tiles; a block whose record says 0 runs takes
    // the CSR gather) and the slot of every edge end in its block's list
    const int *trec;
    const unsigned short *sl;
    int nparts;  // the fused sweep's blocks (the tile sweep's sub-blocks)
    // the fused sweep's per-block incidence lists, padded to capb entries
    // (idxp[blk * capb + j] = idx[ptr[v0] + j]; null: read idx through ptr):
    // a block loads its list with addresses that depend on nothing loaded,
    // beside its CSR pointers -- one round of loads fewer before the gathers
    const unsigned *idxp;
    int capb;
    // zoff: the padded lists hold Z element offsets (u end e: e K, v end e:
    // EK + e K, Zv = Zu + EK) instead of contribution addresses: one add per
    // term, no side / received tests (one GPU, 2 EK + K < 2^32)
    int zoff;
    unsigned EK;
    int zfast;  // the group sweep may address Z by 32-bit offsets (one GPU, one weight)
};

template <typename real>
__device__ __forceinline__ real sx_inv(const SxVArgs<real> &a, long v, long i) {
    return a.invV ? a.invV[v] : a.invAux[i];
}
// the splitting-weight factor of a local incidence (ref :199-217): A1 after
// a reconditioning, else La_d1 (one kernel argument la0 when uniform: the
// caller passes it by value -- a conditional between the argument and an
// array element written as one lvalue made the compiler copy the argument
// to scratch and load the element through a selected pointer)
template <typename real>
__device__ __forceinline__ real sx_wa(const SxVArgs<real> &a, long i, long e, bool lu, real la0) {
    if (a.A1) return a.A1[i];
    if (lu) return la0;
    return a.La_d1[e];
}
template <typename real>
__device__ __forceinline__ real sx_pold(const SxVArgs<real> &a, long i) {
    return a.nop ? a.PF[i].x : a.P[i];
}

// ordered DR average of item (v, k) (ref :636-648): the incidences in the
// reference's (e, side) order, W * Z formed from Z with the reference's
// products; consecutive lanes take consecutive labels, so each incidence is
// a K-contiguous run read coalesced
// (the incidence addresses idx[j0 .. j1): the CSR in memory, or the
// block's list staged in LDS)
template <typename real>
__device__ __forceinline__ real sx_item_sum_from(const SxVArgs<real> &a, long v, int k,
                                                 const unsigned *idx, int j0, int j1, real inv) {
    const int K = a.c.K;
    const bool lu = a.la_u != 0;
    const real la0 = a.la0;
    real s = real(0);
    int j = j0;
    // 8 slots, then 8 contributions in flight per lane; summed in order
    for (; j + 8 <= j1; j += 8) {
        unsigned sl[8];
        real w[8];
#pragma unroll
        for (int q = 0; q < 8; q++) sl[q] = idx[j + q];
        {   // W * Z formed here (the reference's products, same rounding)
            // branch-free: received entries (address 2E + j) sit in the
            // tail of Zv as the sender's W*Z (factor 1), so all 16 loads
            // issue together
            real zq[8], aq[8];
            bool rq[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const long ad = sl[q];
                const bool sv = ad >= a.E;
                const long ea = sv ? ad - a.E : ad;
                rq[q] = ea >= a.E;
                zq[q] = (sv ? a.Zv : a.Zu)[ea * K + k];
                aq[q] = sx_wa(a, rq[q] ? 0 : ea * K + k, rq[q] ? 0 : ea, lu, la0);
            }
#pragma unroll
            for (int q = 0; q < 8; q++) w[q] = rq[q] ? zq[q] : (aq[q] * inv) * zq[q];
        }
#pragma unroll
        for (int q = 0; q < 8; q++) s += w[q];
    }
    for (; j < j1; j++) {
        const long ad = idx[j];
        const bool sv = ad >= a.E;
        const long ea = sv ? ad - a.E : ad;
        const real z = (sv ? a.Zv : a.Zu)[ea * K + k];
        if (ea >= a.E) s += z;
        else s += (sx_wa(a, ea * K + k, ea, lu, la0) * inv) * z;
    }
    return s;
}

// the same sum from a list of Z offsets (SxVArgs::zoff): with one edge
// weight and no A1, every term's splitting weight is the one product
// la0 * 1/Aux, formed once (the reference's product, same rounding)
template <typename real>
__device__ __forceinline__ real sx_item_sum_off(const SxVArgs<real> &a, int k, const unsigned *off,
                                                int j0, int j1, real inv) {
    const real *Z = a.Zu;
    real s = real(0);
    int j = j0;
    if (!a.A1) {
        const real w = a.la0 * inv;
        for (; j + 8 <= j1; j += 8) {
            real z[8];
#pragma unroll
            for (int q = 0; q < 8; q++) z[q] = Z[off[j + q] + k];
#pragma unroll
            for (int q = 0; q < 8; q++) s += w * z[q];
        }
        for (; j < j1; j++) s += w * Z[off[j] + k];
    } else {
        const unsigned EK = a.EK;
        for (; j + 8 <= j1; j += 8) {
            real z[8], an[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const unsigned o = off[j + q];
                z[q] = Z[o + k];
                an[q] = a.A1[(o >= EK ? o - EK : o) + k];
            }
#pragma unroll
            for (int q = 0; q < 8; q++) s += (an[q] * inv) * z[q];
        }
        for (; j < j1; j++) {
            const unsigned o = off[j];
            s += (a.A1[(o >= EK ? o - EK : o) + k] * inv) * Z[o + k];
        }
    }
    return s;
}

template <typename real>
__device__ __forceinline__ real sx_item_sum(const SxVArgs<real> &a, long v, int k) {
    return sx_item_sum_from(a, v, k, a.idx, a.ptr[v], a.ptr[v + 1], sx_inv(a, v, v * a.c.K + k));
}

// ---------------------------------------- tile-ordered sums (K <= 64) ---
// Ordered DR averages of vertex block blk from its tile runs (SxVArgs::trec,
// see k_sx_tile_keys): the u-end rows of Z of the block's own edges (one
// run) and the v-end rows of the (u block, blk) tiles (a few runs), read
// once, coalesced, by this workgroup alone, and written into LDS at their
// SLOT -- the (e, side) rank in the block's CSR-ordered list (sl) -- so
// that each (vertex, label) lane then adds its vertex's entries in the
// reference's order (ref :636-648) with the products of sx_item_sum: the
// same sums bit for bit, one round of loads (record, then the runs) where
// the CSR gather had two dependent ones (pointers, addresses, values).
// Record: [runs n, u start, u count, (v start, count) x (n - 1)] in edge
// units, n <= kSxRuns; the lane's slots [my0, my1) from the CSR pointers.
constexpr int kSxRuns = 15, kSxRec = 32;
template <typename real> struct SxTileCap { static constexpr int v = 2560; };  // LDS reals
template <> struct SxTileCap<double> { static constexpr int v = 1280; };

template <typename real, int M>
struct SxTileLds {
    static constexpr int items = M * kBlock;
    static constexpr int cap = M * SxTileCap<real>::v;  // staged reals (K per list entry)
};

// Stage block blk's runs into LDS by slot: zl[slot * K + k] = Z, and with
// WA the weights (per-edge La_d1: al[slot]; A1: al[slot * K + k]).  All
// lanes of the workgroup take part (barriers).
template <typename real, bool WA, int M>
__device__ __forceinline__ void sx_tile_stage(const SxVArgs<real> &a, int blk, int t, real *zl,
                                              real *al, int *rt) {
    const int K = a.c.K;
    const int lane = t & (kWave - 1);
    const int rv = lane < kSxRec ? a.trec[(long)blk * kSxRec + lane] : 0;
    const int nr = __builtin_amdgcn_readfirstlane(__shfl(rv, 0, kWave));
    // run r in lane r: start, length (edge ends); values K per end (the
    // shuffles run with the whole wave active: a lane reads another's
    // register only while that lane is active)
    const int st = __shfl(rv, min(1 + 2 * lane, kWave - 1), kWave);
    const int lnr = __shfl(rv, min(2 + 2 * lane, kWave - 1), kWave);
    int P = (lane < nr ? lnr : 0) * K;  // inclusive prefix of the runs' values
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int y = __shfl_up(P, o, kWave);
        if (lane >= o) P += y;
    }
    const int tot = __builtin_amdgcn_readlane(P, kWave - 1);
    // the run table in LDS for the item loop below (its lanes diverge)
    if (t < kSxRuns + 1) {
        rt[t] = t < nr ? st : 0;
        rt[kSxRuns + 1 + t] = t < nr ? P : 0x7fffffff;
    }
    __syncthreads();
    const long E = a.E;
    const bool per_e = WA && !a.A1;  // per-edge La_d1: one weight per slot
    const int *rst = rt, *rpr = rt + kSxRuns + 1;
    // off / K as umulhi(off, ceil(2^32 / K)): exact for off < 2^20, K < 4096
    const unsigned mK = (unsigned)((0x100000000ull + K - 1) / K);
    // each lane walks values q = t, t + 256, ...: its run only advances;
    // a block's list fits the LDS (k_sxt_rec), so all of its loads issue in
    // ONE round (U values per lane in flight)
    int r = 0, pend = rpr[0], pbeg = 0;
    constexpr int U = SxTileLds<real, M>::cap / kBlock;
    for (int q0 = t; q0 < tot; q0 += U * kBlock) {
        real z[U], w[U];
        int sl[U], kk[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int q = q0 + u * kBlock;
            ok[u] = q < tot;
            const int qq = ok[u] ? q : tot - 1;
            while (pend <= qq) {
                pbeg = pend;
                pend = rpr[++r];
            }
            const int sr = rst[r];
            const unsigned off = (unsigned)(qq - pbeg);
            const unsigned ei = __umulhi(off, mK);
            kk[u] = (int)(off - ei * (unsigned)K);
            const long p = (long)sr + ei;
            const bool sv = r > 0;
            z[u] = (sv ? a.Zv : a.Zu)[p * K + kk[u]];
            sl[u] = a.sl[(sv ? E : 0) + p];
            w[u] = real(0);
            if (WA) w[u] = a.A1 ? a.A1[p * K + kk[u]] : (kk[u] == 0 ? a.La_d1[p] : real(0));
        }
#pragma unroll
        for (int u = 0; u < U; u++)
            if (ok[u]) {
                zl[sl[u] * K + kk[u]] = z[u];
                if (WA) {
                    if (!per_e) al[sl[u] * K + kk[u]] = w[u];
                    else if (kk[u] == 0) al[sl[u]] = w[u];
                }
            }
    }
    __syncthreads();
}

// the ordered sum of item (v, k) from the staged list: its vertex's slots
// [ptr[v] - ptr[v0], ptr[v + 1] - ptr[v0]) in the reference's order, each
// term (a * 1/Aux) * z as sx_item_sum forms it
template <typename real>
__device__ __forceinline__ real sx_tile_item(const SxVArgs<real> &a, int my0, int my1, int k,
                                             real inv, const real *zl, const real *al, bool wa) {
    const int K = a.c.K;
    const bool per_e = !a.A1;
    const real la0 = a.la0;
    real s = real(0);
    for (int j = my0; j < my1; j++) {
        const real an = !wa ? la0 : (per_e ? al[j] : al[j * K + k]);
        s += (an * inv) * zl[j * K + k];
    }
    return s;
}

// One block of the fused vertex sweep: NT lanes (t = the lane within
// them) with their own xs / ms / red in LDS.  Every lane of the calling
// workgroup reaches the same barriers (a block past the last, blk >= nb, has
// no live lane); the block's evolution partial goes to *part_out (lane 0).
// The body of k_sx_vertex_sweep, shared with the one-workgroup
// k_sx_tiny_iterate (four blocks side by side).
// SPLIT (speculative sessions): the new P and (P, step) go to Po / PFo
// lidx: the padded block list's LDS copy (SxVArgs::idxp); x0s: the raw
// x[0] of each vertex (then the items divide by their metric in parallel and
// the walk takes proj_simplex_column_div), null: the walk divides
template <typename real, int NT, bool SPLIT = false>
__device__ __forceinline__ void sx_vertex_block(const SxVArgs<real> &a, int blk, int t, real *xs,
                                                real *ms, real *red, real *part_out,
                                                unsigned *lidx = nullptr, real *x0s = nullptr) {
    const int K = a.c.K, vb = a.vb;
    const int vl = t / K;
    const int k = t - vl * K;
    const long v0 = (long)blk * vb;
    const long v = v0 + vl;
    const bool live = blk < a.nb && vl < vb && v < a.V;
    const long i = v * K + k;
    // the item's operands before the sum (their latency hides under it)
    real ga = real(0), gaq = real(0), qv = real(0), pold = real(0);
    if (live) {
        ga = a.Ga[i];
        gaq = a.GaQ[i];
        if (a.c.loss == LOSS_QUAD) qv = a.Q[i];
        if (a.track == 1) pold = sx_pold(a, i);
    }
    if (lidx && a.idxp) {  // the padded list into LDS beside the pointers (SxVArgs::idxp)
        const int b0 = a.ptr[v0];
        int j0 = 0, j1 = 0;
        real inv = real(0);
        if (live) {
            j0 = a.ptr[v];
            j1 = a.ptr[v + 1];
            inv = sx_inv(a, v, i);
        }
        const long lb = (long)blk * a.capb;
        for (int q = t; q < a.capb; q += NT) lidx[q] = a.idxp[lb + q];
        j0 -= b0;
        j1 -= b0;
        __syncthreads();
        if (live) {
            const real x = a.zoff ? sx_item_sum_off(a, k, lidx, j0, j1, inv)
                                  : sx_item_sum_from(a, v, k, lidx, j0, j1, inv);
            if (x0s) {  // (ref src/proj_simplex_metric.cpp:44, :49)
                xs[t] = x / ga;
                if (k == 0) x0s[vl] = x;
            } else {
                xs[t] = x;
            }
            ms[t] = ga;
        }
    } else if (live) {
        const real x = sx_item_sum(a, v, k);
        if (x0s) {
            xs[t] = x / ga;
            if (k == 0) x0s[vl] = x;
        } else {
            xs[t] = x;
        }
        ms[t] = ga;
    }
    __syncthreads();
    real dif = real(0);
    if (blk < a.nb && t < vb && v0 + t < a.V) {
        real *x = xs + t * K;
        if (x0s) proj_simplex_column_div<real>(x, ms + t * K, K, x0s[t], real(1));
        else proj_simplex_column<real>(x, ms + t * K, K, real(1));
        if (a.track == 2) {
            real mx = x[0];
            int l = 0;
            for (int d = 1; d < K; d++) if (x[d] > mx) { mx = x[d]; l = d; }
            const real fl = (real)l;
            if (fl != a.lab[v0 + t]) { dif = real(1); a.lab[v0 + t] = fl; }
            if (a.terms) a.terms[v0 + t] = dif;
        }
    }
    __syncthreads();
    if (live) {
        const real p = xs[t];
        if (a.track == 1) {
            real d = pold - p;
            if (d < real(0)) d = -d;
            dif += d;
            if (a.terms) a.terms[i] = d;
        }
        if (!a.nop) (SPLIT ? a.Po : a.P)[i] = p;
        // Q enters the quadratic loss's step only (no load otherwise)
        SxR2<real> q;
        q.x = p;
        q.y = sx_explicit(a.c, p, gaq, qv);
        (SPLIT ? a.PFo : a.PF)[i] = q;
    }
    if (a.track) {
        dif = wave_sum(dif);
        if (NT > kWave) {
            if ((t & (kWave - 1)) == 0) red[t / kWave] = dif;
            __syncthreads();
            if (t == 0) for (int q = 1; q < NT / kWave; q++) dif += red[q];
        }
        if (t == 0 && blk < a.nb) *part_out = dif;
    }
}

constexpr int kSxPadPer = 8;  // entries of a padded block list per lane, at most
constexpr int kSxNtDefault = 256;  // the fused sweep's workgroup width (fused_sweep_setup)
constexpr int kSxMDefault = 2;     // its vertex blocks per workgroup (fused_sweep_setup)
template <typename real, int NT, bool SPLIT = false>
__global__ __launch_bounds__(NT) void k_sx_vertex_sweep(SxVArgs<real> a) {
    if (a.ctrl && a.ctrl->halt) return;
    __shared__ real xs[NT], ms[NT];
    __shared__ real red[NT / kWave];
    __shared__ unsigned lidx[kSxPadPer * NT];
    __shared__ real x0s[NT];
    const int blk = xcd_block(blockIdx.x, a.nb, a.xcd);
    if (blk >= a.nb) return;
    sx_vertex_block<real, NT, SPLIT>(a, blk, threadIdx.x, xs, ms, red, a.part + blk, lidx, x0s);
}

// the padded lists (SxVArgs::idxp) and their width: the largest block's
// list (*capb, atomicMax) first
__global__ void k_sx_block_max(int nb, int vb, int V, const int *__restrict__ ptr,
                               int *__restrict__ capb) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const long v0 = (long)b * vb, v1 = min(v0 + vb, (long)V);
    atomicMax(capb, ptr[v1] - ptr[v0]);
}
// (K > 0: Z offsets, SxVArgs::zoff; else the addresses)
__global__ void k_sx_pad_idx(long n, int capb, int vb, int V, const int *__restrict__ ptr,
                             const unsigned *__restrict__ idx, unsigned *__restrict__ idxp,
                             long E, int K) {
    const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const long b = q / capb;
    const int j = (int)(q - b * capb);
    const long v0 = b * vb, v1 = min(v0 + vb, (long)V);
    const int j0 = ptr[v0];
    unsigned x = 0u;
    if (j < ptr[v1] - j0) {
        const unsigned ad = idx[j0 + j];
        x = K ? (unsigned)(ad >= (unsigned long)E ? E * K + (ad - E) * (long)K : (long)ad * K) : ad;
    }
    idxp[q] = x;
}

// Tile-ordered sessions: one workgroup per tile block of M * vb vertices (M
// items per lane), its sums from the block's tile runs (sx_tile_sum) or,
// for a block without a record, the CSR gather.  M > 1 gives each
// workgroup's load rounds and projection walk M times the work: the sweep
// is bound by the latency of those serial phases, not by its bytes.

// ST: staged tile sums (the block's record); else the CSR gather, from the
// block's padded list in LDS (SxVArgs::idxp over M * vb vertices) when there
// is one -- M items per lane, their gathers in flight together
template <typename real, bool SPLIT, bool WA, int M, bool ST = true>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(ST || M > 2 || sizeof(real) > 4 ? 1 : 8)))
void k_sx_vertex_tile(SxVArgs<real> a) {
    if (a.ctrl && a.ctrl->halt) return;
    using L = SxTileLds<real, M>;
    __shared__ real xs[L::items], ms[L::items], x0s[L::items];
    __shared__ real red[M][kBlock / kWave];
    __shared__ real zl[ST ? L::cap : 1];
    __shared__ real al[ST && WA ? L::cap : 1];
    __shared__ int rt[2 * (kSxRuns + 1)];
    __shared__ unsigned lidx[ST ? 1 : kSxPadPer * kBlock];
    const int blk = xcd_block(blockIdx.x, a.nb, a.xcd);
    if (blk >= a.nb) return;
    const int t = threadIdx.x;
    // M sub-blocks of vb vertices (the fused sweep's blocks): lane t takes
    // item t of each, so every sub-block's evolution partial is formed by
    // the lanes and tree of k_sx_vertex_sweep -- the same partials bit for
    // bit, written where that sweep writes them (part[blk * M + u])
    const int K = a.c.K, vb = a.vb, vbK = vb * K, nv = M * vb;
    const long v0 = (long)blk * nv;
    // the items' operands before the sum (their latency hides under it)
    real ga[M], gaq[M], qv[M], pold[M], x[M], inv[M];
    long vi[M];
    int kk[M], j0[M], j1[M];
    bool live[M];
    const int vt = t / K, kt = t - vt * K;
    const int b0 = a.ptr[v0];  // (the list's slots are relative to the tile block's first)
#pragma unroll
    for (int u = 0; u < M; u++) {
        kk[u] = kt;
        vi[u] = v0 + u * vb + vt;
        live[u] = t < vbK && vi[u] < a.V;
        ga[u] = gaq[u] = qv[u] = pold[u] = x[u] = inv[u] = real(0);
        if (live[u]) {
            const long i = vi[u] * K + kk[u];
            ga[u] = a.Ga[i];
            gaq[u] = a.GaQ[i];
            if (a.c.loss == LOSS_QUAD) qv[u] = a.Q[i];
            if (a.track == 1) pold[u] = sx_pold(a, i);
            inv[u] = sx_inv(a, vi[u], i);
            j0[u] = a.ptr[vi[u]];
            j1[u] = a.ptr[vi[u] + 1];
        }
    }
    if (ST && a.trec[(long)blk * kSxRec] > 0) {  // block-uniform
        sx_tile_stage<real, WA, M>(a, blk, t, zl, al, rt);
#pragma unroll
        for (int u = 0; u < M; u++)
            if (live[u]) x[u] = sx_tile_item(a, j0[u] - b0, j1[u] - b0, kk[u], inv[u], zl, al, WA);
    } else if (!ST && a.idxp) {  // the padded list (SxVArgs::idxp) into LDS
        const long lb = (long)blk * a.capb;
        for (int q = t; q < a.capb; q += kBlock) lidx[q] = a.idxp[lb + q];
        __syncthreads();
        if (a.zoff && !a.A1) {
            // Z offsets, one splitting weight la0 * 1/Aux per item: the M
            // items' 8 gathers each in flight together, added in order
            const real *Z = a.Zu;
            real w[M];
            int j[M], e[M];
#pragma unroll
            for (int u = 0; u < M; u++) {
                w[u] = a.la0 * inv[u];
                j[u] = live[u] ? j0[u] - b0 : 0;
                e[u] = live[u] ? j1[u] - b0 : 0;
            }
            for (;;) {
                bool more = false;
#pragma unroll
                for (int u = 0; u < M; u++) more |= j[u] < e[u];
                if (!more) break;
                real z[M][8];
#pragma unroll
                for (int u = 0; u < M; u++)
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        z[u][q] = j[u] + q < e[u] ? Z[lidx[j[u] + q] + kk[u]] : real(0);
#pragma unroll
                for (int u = 0; u < M; u++) {
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        if (j[u] + q < e[u]) x[u] += w[u] * z[u][q];
                    j[u] += 8;
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < M; u++)
                if (live[u])
                    x[u] = a.zoff ? sx_item_sum_off(a, kk[u], lidx, j0[u] - b0, j1[u] - b0, inv[u])
                                  : sx_item_sum_from(a, vi[u], kk[u], lidx, j0[u] - b0,
                                                     j1[u] - b0, inv[u]);
        }
    } else {
#pragma unroll
        for (int u = 0; u < M; u++)
            if (live[u]) x[u] = sx_item_sum(a, vi[u], kk[u]);
    }
    // divided by the metric here, the raw x[0] aside (ref
    // src/proj_simplex_metric.cpp:44, :49; proj_simplex_column_div)
#pragma unroll
    for (int u = 0; u < M; u++)
        if (live[u]) {
            const int it = u * vbK + t;
            xs[it] = x[u] / ga[u];
            ms[it] = ga[u];
            if (kk[u] == 0) x0s[u * vb + vt] = x[u];
        }
    __syncthreads();
    // one lane per vertex walks its column (all M sub-blocks side by side);
    // a label change is 0 / 1, so its count is exact in any order: x0s
    // takes it for the sub-block sums below
    for (int vl = t; vl < nv; vl += kBlock) {
        if (v0 + vl >= a.V) break;
        real *xc = xs + vl * K;
        proj_simplex_column_div<real>(xc, ms + vl * K, K, x0s[vl], real(1));
        if (a.track == 2) {
            real mx = xc[0];
            int l = 0;
            for (int d = 1; d < K; d++) if (xc[d] > mx) { mx = xc[d]; l = d; }
            const real fl = (real)l;
            real dl = real(0);
            if (fl != a.lab[v0 + vl]) { dl = real(1); a.lab[v0 + vl] = fl; }
            if (a.terms) a.terms[v0 + vl] = dl;
            x0s[vl] = dl;
        }
    }
    __syncthreads();
    real dif[M];
#pragma unroll
    for (int u = 0; u < M; u++) {
        dif[u] = real(0);
        if (!live[u]) continue;
        const long i = vi[u] * K + kk[u];
        const real p = xs[u * vbK + t];
        if (a.track == 1) {
            real d = pold[u] - p;
            if (d < real(0)) d = -d;
            dif[u] = d;
            if (a.terms) a.terms[i] = d;
        }
        if (!a.nop) (SPLIT ? a.Po : a.P)[i] = p;
        SxR2<real> q;
        q.x = p;
        q.y = sx_explicit(a.c, p, gaq[u], qv[u]);
        (SPLIT ? a.PFo : a.PF)[i] = q;
    }
    if (a.track == 2) {  // sub-block u's vertices [u vb, u vb + vb): lane t < vb, as the fused sweep
#pragma unroll
        for (int u = 0; u < M; u++) dif[u] = (t < vb && v0 + u * vb + t < a.V) ? x0s[u * vb + t] : real(0);
    }
    if (a.track) {
#pragma unroll
        for (int u = 0; u < M; u++) {
            const real w = wave_sum(dif[u]);
            if ((t & (kWave - 1)) == 0) red[u][t / kWave] = w;
        }
        __syncthreads();
        if (t < M) {  // (((w0 + w1) + w2) + w3), k_sx_vertex_sweep's order
            const long sb = (long)blk * M + t;
            real d = red[t][0];
            for (int q = 1; q < kBlock / kWave; q++) d += red[t][q];
            if (sb < a.nparts) a.part[sb] = d;
        }
    }
}

// ------------------------------------------ group vertex sweep (K > 64) --
// NV vertices per workgroup (NV <= 64, sized so that their K-long columns
// fit in LDS).  (1) sums: the block's 256 lanes take the group's (vertex,
// label) items, consecutive lanes consecutive labels, two items per lane in
// flight, each item's ordered sum over its incidences (K-contiguous runs of
// Z, read coalesced), divided by its metric, into LDS COLUMNS
// xs[k * (NV + 1) + v]; (2) projection: lane v < NV walks its vertex down its
// column -- the reference's comparisons and threshold updates
// (src/proj_simplex_metric.cpp:41-72), its sequential arithmetic SIMT across
// the group's vertices, conflict-free (consecutive lanes, consecutive words);
// (3) the items again: (x - la) m or 0 (ref :74-80), evolution terms, P and
// (P, step) written back as coalesced rows (then the label scan, if asked).  The metric
// projection costs K steps of one lane per vertex: a typical column (an
// averaged distribution, which enters the active set element by element)
// has ~K events, so a whole wave per vertex (one ballot per event) spent 64
// lanes' issue slots on each step and ran the C4 law at K = 100 at 5.2 ms
// (0.9 TB/s) where this layout shares them among NV vertices.
template <typename real>
struct SxGroup {
    static constexpr int kMaxNV = 64;
    // vertices per group, at most: C4's law at K = 100 (1M vertices), group
    // sweep 1.69 / 1.73 / 1.75 ms at 16 / 32 / 64 -- the walking lanes per CU
    // are set by the LDS whatever the split, and smaller groups keep more
    // workgroups' loads in flight
    static constexpr int kNV = 16;
    static constexpr int kInc = 16;            // staged incidences per vertex, on average
    static constexpr size_t kLds = 60 * 1024;  // bytes of dynamic LDS per workgroup, at most
    // per (vertex, label): x and m (reals) and the active flag (a byte);
    // per staged incidence: its Z offset (int64, side and received bits on top)
    // and its weight a_e (real)
    static size_t bytes(int K, int nv) {
        const size_t col = (size_t)K * (nv + 1) * (2 * sizeof(real) + 1);
        return (col + 7) / 8 * 8 + (size_t)kInc * nv * (8 + sizeof(real));
    }
    // vertices per group for K labels (0: K too wide for LDS)
    static int nv_for(int K, int want) {
        int nv = want;
        while (nv > 1 && bytes(K, nv) > kLds) nv >>= 1;
        return bytes(K, nv) <= kLds ? nv : 0;
    }
};

constexpr long kZv = 1L << 62, kRecv = 1L << 61;  // staged Z offset: v-side / received

// items per lane in flight in the group sweep's sums: C4's law at K = 100
// (1M vertices), group sweep ms: 1 item 2.0, 2 items 1.69, 4 items 2.2-3.1
constexpr int SXU = 2;
#ifndef PFDR_SXU_FAST
#define PFDR_SXU_FAST 2
#endif
constexpr int kSxuFast = PFDR_SXU_FAST;  // (fast variant: 3 or 4 spill at eight waves)

// FAST: launched while SxVArgs::zfast holds and there is no A1 (the 32-bit
// offset sums only: fewer registers, more workgroups in flight)
template <typename real, bool SPLIT, bool FAST = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(FAST && sizeof(real) == 4 ? 8 : 1)))
void k_sx_vertex_group(SxVArgs<real> a) {
    constexpr int XU = FAST ? kSxuFast : SXU;  // items per lane in the sums
    if (a.ctrl && a.ctrl->halt) return;
    extern __shared__ double lds_group[];
    __shared__ real red[kBlock / kWave];
    __shared__ real x0s[SxGroup<real>::kMaxNV], las[SxGroup<real>::kMaxNV];
    __shared__ int lptr[SxGroup<real>::kMaxNV + 1];
    const int K = a.c.K, NV = a.vb, st = NV + 1, t = threadIdx.x;
    real *xs = reinterpret_cast<real *>(lds_group);
    real *ms = xs + (size_t)K * st;
    unsigned char *I = reinterpret_cast<unsigned char *>(ms + (size_t)K * st);
    long *zo = reinterpret_cast<long *>(lds_group) +
               ((size_t)K * st * (2 * sizeof(real) + 1) + 7) / 8;
    real *wa = reinterpret_cast<real *>(zo + SxGroup<real>::kInc * NV);
    const long v0 = (long)blockIdx.x * NV;
    const int nv = (int)(a.V - v0 < NV ? a.V - v0 : NV);  // this group's vertices
    const int nitems = nv * K;
    // (0) the group's incidence lists (one contiguous CSR range), decoded once
    // into LDS: every item of a vertex then issues its K-run loads of Z at once
    if (t <= nv) lptr[t] = a.ptr[v0 + t];
    __syncthreads();
    const int jb = lptr[0], nj = lptr[nv] - jb;
    const bool staged = nj <= SxGroup<real>::kInc * NV;
    // one GPU, one edge weight, no A1 (SxVArgs::zfast): the incidences as
    // 32-bit Z offsets (u end e: e K, v end: EK + e K), and every term's
    // splitting weight the item's one product la0 * 1/Aux
    const bool fast = FAST;
    unsigned *zo32 = reinterpret_cast<unsigned *>(zo);
    if (staged && fast) {
        for (int q = t; q < nj; q += kBlock) {
            const unsigned ad = a.idx[jb + q];
            zo32[q] = ad >= (unsigned)a.E ? a.EK + (ad - (unsigned)a.E) * (unsigned)K : ad * (unsigned)K;
        }
        __syncthreads();
    } else if (staged) {
        const bool lu = a.la_u != 0;
        const real la0 = a.la0;
        for (int q = t; q < nj; q += kBlock) {
            const long ad = a.idx[jb + q];
            const bool sv = ad >= a.E;
            const long ea = sv ? ad - a.E : ad;
            const bool rq = ea >= a.E;  // received: the sender's W * Z in the tail of Zv
            zo[q] = ea * K | (sv ? kZv : 0) | (rq ? kRecv : 0);
            real w = real(0);
            if (!rq && !a.A1) w = lu ? la0 : a.La_d1[ea];
            wa[q] = w;
        }
        __syncthreads();
    }
    // (1) ordered sums (ref :636-648), divided by their metric (the first
    // pass's x[d] / m[d], ref :44, :49), raw x[0] aside; XU items per lane,
    // their XU x 8 K-run loads of Z in flight together
    for (int it0 = t; it0 < nitems; it0 += XU * kBlock) {
        real x[XU];
        int vl[XU], k[XU];
        long i[XU];
        bool ok[XU];
#pragma unroll
        for (int u = 0; u < XU; u++) {
            const int it = it0 + u * kBlock;
            ok[u] = it < nitems;
            vl[u] = ok[u] ? it / K : 0;
            k[u] = ok[u] ? it - vl[u] * K : 0;
            i[u] = v0 * K + (ok[u] ? it : 0);
            x[u] = real(0);
        }
        real m[XU];  // the metric, loaded with the first round of the sum's loads
#pragma unroll
        for (int u = 0; u < XU; u++) m[u] = ok[u] ? a.Ga[i[u]] : real(1);
        if (staged && fast) {
            const real *Z = a.Zu;
            real w[XU];
            int j[XU], j1[XU];
#pragma unroll
            for (int u = 0; u < XU; u++) {
                w[u] = ok[u] ? a.la0 * sx_inv(a, v0 + vl[u], i[u]) : real(0);
                j[u] = ok[u] ? lptr[vl[u]] - jb : 0;
                j1[u] = ok[u] ? lptr[vl[u] + 1] - jb : 0;
            }
            for (;;) {
                bool more = false;
#pragma unroll
                for (int u = 0; u < XU; u++) more |= j[u] < j1[u];
                if (!more) break;  // 8 K-run loads per item, added in order
                real zq[XU][8];
#pragma unroll
                for (int u = 0; u < XU; u++)
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        zq[u][q] = j[u] + q < j1[u] ? Z[zo32[j[u] + q] + k[u]] : real(0);
#pragma unroll
                for (int u = 0; u < XU; u++) {
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        if (j[u] + q < j1[u]) x[u] += w[u] * zq[u][q];
                    j[u] += 8;
                }
            }
        } else if (!FAST && staged) {
            real inv[XU];
            int j[XU], j1[XU];
#pragma unroll
            for (int u = 0; u < XU; u++) {
                inv[u] = ok[u] ? sx_inv(a, v0 + vl[u], i[u]) : real(0);
                j[u] = ok[u] ? lptr[vl[u]] - jb : 0;
                j1[u] = ok[u] ? lptr[vl[u] + 1] - jb : 0;
            }
            for (;;) {
                bool more = false;
#pragma unroll
                for (int u = 0; u < XU; u++) more |= j[u] < j1[u];
                if (!more) break;  // 8 K-run loads per item, added in order
                real zq[XU][8], aq[XU][8];
                bool rq[XU][8];
#pragma unroll
                for (int u = 0; u < XU; u++)
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        rq[u][q] = true;
                        zq[u][q] = aq[u][q] = real(0);
                        if (j[u] + q < j1[u]) {
                            const long o = zo[j[u] + q];
                            const long e = o & (kRecv - 1);
                            rq[u][q] = (o & kRecv) != 0;
                            zq[u][q] = ((o & kZv) ? a.Zv : a.Zu)[e + k[u]];
                            aq[u][q] = (a.A1 && !rq[u][q]) ? a.A1[e + k[u]] : wa[j[u] + q];
                        }
                    }
#pragma unroll
                for (int u = 0; u < XU; u++) {
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        if (j[u] + q < j1[u])
                            x[u] += rq[u][q] ? zq[u][q] : (aq[u][q] * inv[u]) * zq[u][q];
                    j[u] += 8;
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < XU; u++)  // (a hub-sized group: the CSR from memory)
                if (ok[u]) x[u] = sx_item_sum(a, v0 + vl[u], k[u]);
        }
#pragma unroll
        for (int u = 0; u < XU; u++) {
            if (!ok[u]) continue;
            if (k[u] == 0) x0s[vl[u]] = x[u];
            xs[k[u] * st + vl[u]] = x[u] / m[u];
            ms[k[u] * st + vl[u]] = m[u];
        }
    }
    // (3)'s first FU items per lane: their operands loaded now, their latency
    // under the walk
    constexpr int FU = 8;
    real pold[FU], gq[FU], qq[FU];
    auto fin_load = [&](int it0) {
#pragma unroll
        for (int u = 0; u < FU; u++) {
            const int it = it0 + u * kBlock;
            pold[u] = gq[u] = qq[u] = real(0);
            if (it < nitems) {
                const long i = v0 * K + it;  // (items are the group's rows, in order)
                if (a.track == 1) pold[u] = sx_pold(a, i);
                gq[u] = a.GaQ[i];
                if (a.c.loss == LOSS_QUAD) qq[u] = a.Q[i];
            }
        }
    };
    fin_load(t);
    __syncthreads();
    real dif = real(0);
    if (t < nv)  // (2) one lane per vertex down its column
        las[t] = proj_simplex_walk<real>(xs + t, ms + t, I + t, K, st, x0s[t], real(1));
    __syncthreads();
    // (3) finalise (ref :74-80), rows back out; FU items per lane, loads first
    for (int it0 = t; it0 < nitems; it0 += FU * kBlock) {
        if (it0 != t) fin_load(it0);
#pragma unroll
        for (int u = 0; u < FU; u++) {
            const int it = it0 + u * kBlock;
            if (it >= nitems) break;
            const int vl = it / K, k = it - vl * K;
            const long i = v0 * K + it;
            const int c = k * st + vl;
            const real p = I[c] ? (xs[c] - las[vl]) * ms[c] : real(0);
            if (a.track == 2) xs[c] = p;  // for the label scan
            if (a.track == 1) {
                real d = pold[u] - p;
                if (d < real(0)) d = -d;
                dif += d;
                if (a.terms) a.terms[i] = d;
            }
            if (!a.nop) (SPLIT ? a.Po : a.P)[i] = p;
            SxR2<real> q;
            q.x = p;
            q.y = sx_explicit(a.c, p, gq[u], qq[u]);
            (SPLIT ? a.PFo : a.PF)[i] = q;
        }
    }
    if (a.track == 2) {  // maximum-likelihood label of each vertex (ref :656-676)
        __syncthreads();
        if (t < nv) {
            const real *x = xs + t;
            real mx = x[0];
            int l = 0;
            for (int d = 1; d < K; d++) if (x[d * st] > mx) { mx = x[d * st]; l = d; }
            const real fl = (real)l;
            if (fl != a.lab[v0 + t]) { dif = real(1); a.lab[v0 + t] = fl; }
            if (a.terms) a.terms[v0 + t] = dif;
        }
    }
    if (a.track) {
        dif = block_sum(dif, red);
        if (t == 0) a.part[blockIdx.x] = dif;
    }
}

// ------------------------ wide vertex sweep in memory (K past the LDS) --
// One WAVE per vertex, lane l holding the labels k = l + 64 j: every
// incidence is one K-contiguous run of Z read coalesced by the wave, the
// averages go to xs (projected in place by the whole wave, pfdr_proj.hpp:
// one ballot per active-set event, bit-exact with ref
// src/proj_simplex_metric.cpp:41-80, the active set in act), and P and
// (P, step) go back as coalesced rows.  For K whose column does not fit a
// group's LDS (f32 K > 3,413, f64 K > 1,807).
constexpr int kSxWideVpw = 4;  // vertices per wave; a block's 4 waves interleave

// ordered DR average (ref :636-648) of labels k = k0 + lane + 64 j of vertex
// v (wave-uniform): the incidences in the reference's (e, side) order, W * Z
// formed with the fused sweep's operations (sx_item_sum); B incidences'
// loads in flight, added in order
template <typename real, int J>
__device__ __forceinline__ void sx_wide_sums(const SxVArgs<real> &a, long v, int k0, int lane,
                                             real (&s)[J]) {
    constexpr int B = J >= 8 ? 1 : 8 / J;
    const int K = a.c.K;
    const long b = v * K;
    const bool lu = a.la_u != 0;
    const real la0 = a.la0;
    real inv[J];
    bool ok[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int k = k0 + lane + 64 * j;
        ok[j] = k < K;
        inv[j] = ok[j] ? sx_inv(a, v, b + k) : real(0);
        s[j] = real(0);
    }
    const int j0 = a.ptr[v], j1 = a.ptr[v + 1];
    int q = j0;
    for (; q + B <= j1; q += B) {
        real z[B][J], an[B][J];
        bool rq[B];
#pragma unroll
        for (int u = 0; u < B; u++) {
            const long ad = a.idx[q + u];
            const bool sv = ad >= a.E;
            const long ea = sv ? ad - a.E : ad;
            rq[u] = ea >= a.E;  // received: the sender's W * Z in the tail of Zv
            const real *zp = (sv ? a.Zv : a.Zu) + ea * K;
            real la = real(0);
            if (!a.A1 && !rq[u]) la = lu ? la0 : a.La_d1[ea];
#pragma unroll
            for (int j = 0; j < J; j++) {
                const long k = k0 + lane + 64 * j;
                z[u][j] = ok[j] ? zp[k] : real(0);
                an[u][j] = (a.A1 && !rq[u] && ok[j]) ? a.A1[ea * K + k] : la;
            }
        }
#pragma unroll
        for (int u = 0; u < B; u++)
#pragma unroll
            for (int j = 0; j < J; j++) s[j] += rq[u] ? z[u][j] : (an[u][j] * inv[j]) * z[u][j];
    }
    for (; q < j1; q++) {
        const long ad = a.idx[q];
        const bool sv = ad >= a.E;
        const long ea = sv ? ad - a.E : ad;
        const bool rq = ea >= a.E;
        const real *zp = (sv ? a.Zv : a.Zu) + ea * K;
        real la = real(0);
        if (!a.A1 && !rq) la = lu ? la0 : a.La_d1[ea];
#pragma unroll
        for (int j = 0; j < J; j++) {
            const long k = k0 + lane + 64 * j;
            const real z = ok[j] ? zp[k] : real(0);
            const real an = (a.A1 && !rq && ok[j]) ? a.A1[ea * K + k] : la;
            s[j] += rq ? z : (an * inv[j]) * z;
        }
    }
}

// evolution term, new P and (P, step) of one (v, k); the label scan's candidate
template <typename real, bool SPLIT>
__device__ __forceinline__ void sx_wide_out(const SxVArgs<real> &a, long b, int k, real p,
                                            real &dif, real &mv, int &mi) {
    const long i = b + k;
    if (a.track == 1) {
        real d = sx_pold(a, i) - p;
        if (d < real(0)) d = -d;
        dif += d;
        if (a.terms) a.terms[i] = d;
    } else if (a.track == 2) {
        argmax_take(p, k, mv, mi);
    }
    if (!a.nop) (SPLIT ? a.Po : a.P)[i] = p;
    SxR2<real> q;
    q.x = p;
    q.y = sx_explicit(a.c, p, a.GaQ[i], a.c.loss == LOSS_QUAD ? a.Q[i] : real(0));
    (SPLIT ? a.PFo : a.PF)[i] = q;
}

template <typename real, bool SPLIT>
__global__ __launch_bounds__(kBlock) void k_sx_vertex_wide(SxVArgs<real> a) {
    if (a.ctrl && a.ctrl->halt) return;
    __shared__ real red[kBlock / kWave];
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = (int)(threadIdx.x & (kWave - 1));
    const int K = a.c.K;
    real dif = real(0);
    for (int q = 0; q < kSxWideVpw; q++) {
        const long v = ((long)blockIdx.x * kSxWideVpw + q) * (kBlock / kWave) + w;
        if (v >= a.V) break;  // wave-uniform
        const long b = v * K;
        real mv = real(0);
        int mi = 0x7fffffff;
        for (int k0 = 0; k0 < K; k0 += 4 * 64) {
            real s4[4];
            sx_wide_sums<real, 4>(a, v, k0, lane, s4);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int k = k0 + lane + 64 * j;
                if (k < K) a.xs[b + k] = s4[j];
            }
        }
        proj_wave_mem<real>(a.xs + b, a.Ga + b, K, real(1), a.act + b);
        const real p0 = lane_read(lane == 0 ? a.xs[b] : real(0), 0);
        for (int k = lane; k < K; k += 64) sx_wide_out<real, SPLIT>(a, b, k, a.xs[b + k], dif, mv, mi);
        if (a.track == 2) {  // maximum-likelihood label (ref :656-676)
            const int l = wave_argmax(mv, mi, p0 != p0);
            if (lane == 0) {
                real d = real(0);
                const real fl = (real)l;
                if (fl != a.lab[v]) { d = real(1); a.lab[v] = fl; }
                if (a.terms) a.terms[v] = d;
                dif += d;
            }
        }
    }
    if (a.track) {
        dif = block_sum(dif, red);
        if (threadIdx.x == 0) a.part[blockIdx.x] = dif;
    }
}

// ------------------------------- standalone metric projection (any D) --
// proj_simplex_metric (ref src/proj_simplex_metric.cpp:18-83): one segment
// of G lanes per column, coordinates in J registers per lane
template <typename real, int G, int J>
__global__ __launch_bounds__(kBlock) void k_proj_wave(real *X, const real *M, int D, int N,
                                                      int nm, const real *A, int na) {
    const Seg<G> sg;
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if ((t - (t & (kWave - 1))) / G >= N) return;  // the whole wave is past the last column
    const long col = t / G;
    const bool live = col < N;
    const real *m = M + (size_t)D * (live && nm > col ? col : nm - 1);
    const real a = live ? (na > col ? A[col] : A[na - 1]) : real(1);
    real x[J], mm[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int d = j * G + sg.sl;
        const bool ok = live && d < D;
        x[j] = ok ? X[(size_t)D * col + d] : real(0);
        mm[j] = ok ? m[d] : real(1);
    }
    proj_segment<real, G, J>(sg, x, mm, live ? D : 0, a);
#pragma unroll
    for (int j = 0; j < J; j++) {
        const int d = j * G + sg.sl;
        if (live && d < D) X[(size_t)D * col + d] = x[j];
    }
}

// D > 1024: one wave per column in memory, active flags in I (D bytes per column)
template <typename real>
__global__ __launch_bounds__(kBlock) void k_proj_mem(real *X, const real *M, int D, int N, int nm,
                                                     const real *A, int na, unsigned char *I) {
    const long col = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (col >= N) return;  // wave-uniform
    const real *m = M + (size_t)D * (nm > col ? col : nm - 1);
    const real a = na > col ? A[col] : A[na - 1];
    proj_wave_mem<real>(X + (size_t)D * col, m, D, a, I + (size_t)D * col);
}

// ------------------------------------------ small problems, one launch --
// Up to `iters` whole iterations of a small single-GPU simplex problem in ONE
// workgroup of 1024 lanes: the edge pass (sx_edge_lane over the (edge,
// label) entries), the vertex pass four 256-lane blocks side by side
// (sx_vertex_block, the fused vertex sweep's blocks with their partials in
// LDS), then k_sx_finalize's reduction and decision on a register copy of
// the control block.  The same device code and operation order as the
// three-launch loop, so the iterates, iteration counts and the evolution
// record are identical bit for bit; what goes is the launches that bound
// cut pursuit's reduced problems.
constexpr int kSxTiny = 1024;
constexpr int kSxTinyMaxBlocks = 32;
// default limits (PFDR_SX_TINY widens the entry limit and the block cap to
// 32): against the three launches (graph-replayed), us/iteration on 8-nbr
// grids, K = 4 (profiles/r2/r3m_exp_sx_tiny.log): f32 1 block 6.6 vs 11.0,
// 4 blocks 11.1 vs 11.9, 9 blocks 25 vs 11.8; f64 1 block 8.0 vs 12.4, 4
// blocks 14.2 vs 12.7 -- one CU's throughput loses beyond a few blocks
template <typename real> struct SxTinyBlocks { static constexpr int v = 4; };
template <> struct SxTinyBlocks<double> { static constexpr int v = 2; };
constexpr long kSxTinyEK = 1L << 16;

template <typename real>
struct SxTinyArgs {
    long EK;
    SxConst<real> c;
    const int *Eu, *Ev;
    real *Zu, *Zv;
    const real *A1, *La_d1, *Wd1u, *Wd1v, *Th;
    const SxR2<real> *GI;
    real rho;
    SxVArgs<real> va;   // every block of the fused vertex sweep
    Ctrl<real> *ctrl;   // null: no tracking, run exactly `iters`
    real *Dif;
    long V;             // vertices (the l1 evolution's normalisation)
    int iters;
};

template <typename real, int L>
__global__ __launch_bounds__(kSxTiny) void k_sx_tiny_iterate(SxTinyArgs<real> t) {
    constexpr int NB = kSxTiny / kBlock;  // vertex blocks side by side
    __shared__ real xs[kSxTiny], ms[kSxTiny];
    __shared__ real red[kSxTiny / kWave];
    __shared__ real bpart[kSxTinyMaxBlocks + NB];
    __shared__ real wred[kBlock / kWave];
    __shared__ int halt;
    const int tid = threadIdx.x, sub = tid / kBlock, lt = tid & (kBlock - 1);
    const SxVArgs<real> &a = t.va;
    Ctrl<real> c{};
    if (tid == 0) {
        if (t.ctrl) c = *t.ctrl;
        halt = t.ctrl ? c.halt : 0;
    }
    __syncthreads();
    for (int it = 0; it < t.iters; it++) {
        if (halt) break;  // uniform (set by lane 0 before the last barrier)
        for (long i = (long)tid * L; i < t.EK; i += (long)kSxTiny * L)
            sx_edge_lane<real, L>(i, t.EK, t.c, t.Eu, t.Ev, a.PF, t.Zu, t.Zv, t.A1, t.La_d1, t.GI,
                                  t.Wd1u, t.Wd1v, t.Th, nullptr, t.rho);
        __syncthreads();
        for (int b0 = 0; b0 < a.nb; b0 += NB) {
            const int blk = b0 + sub;
            sx_vertex_block<real, kBlock>(a, blk, lt, xs + sub * kBlock, ms + sub * kBlock,
                                                 red + sub * (kBlock / kWave), bpart + blk);
            __syncthreads();  // xs / ms / red reused by the next four blocks
        }
        if (t.ctrl) {  // k_sx_finalize on the first 256 lanes: its loop and block_sum's tree
            real sm = real(0);
            if (a.track) {
                if (tid < kBlock)
                    for (int i = tid; i < a.nb; i += kBlock) sm += bpart[i];
                sm = wave_sum(sm);
                if ((tid & (kWave - 1)) == 0 && tid < kBlock) wred[tid / kWave] = sm;
            }
            __syncthreads();
            if (tid == 0) {
                real s = real(0);
                if (a.track)
                    for (int i = 0; i < kBlock / kWave; i++) s += wred[i];
                int itc = c.it;
                if (a.track) {
                    real dif = s;
                    if (a.track == 1) dif /= t.V;  // relative l1 evolution (ref :688)
                    c.dif = dif;
                    if (t.Dif) t.Dif[itc] = dif;
                }
                itc++;
                c.it = itc;
                const real dif = c.dif;
                if (itc >= c.itMax || dif < c.difTol) {
                    c.stop = 1;
                    c.halt = 1;
                } else if (dif < c.difRcd) {
                    c.recond = 1;
                    c.halt = 1;
                }
                *t.ctrl = c;
                halt = c.halt;
            }
        }
        __syncthreads();
    }
}

template <typename real>
__global__ void k_fill(long n, real *p, real v) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// K-wide W*Z of the pushed v ends (address E + e) / u ends (address e),
// packed in the plan's push order
template <typename real>
__global__ void k_sx_pack_wz(long n, int K, long E, const unsigned *__restrict__ addr,
                             const int *__restrict__ Eu, const int *__restrict__ Ev,
                             const real *__restrict__ A1, const real *__restrict__ La_d1,
                             const SxR2<real> *__restrict__ GI, const real *__restrict__ Zu,
                             const real *__restrict__ Zv, real *__restrict__ out) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * K) return;
    const long i = t / K;
    const int k = (int)(t - i * K);
    const long ad = addr[i];
    const bool sv = ad >= E;
    const long e = sv ? ad - E : ad;
    const long row = sv ? Ev[e] : Eu[e];
    const real w = sx_a(e * K + k, e, A1, La_d1) * GI[row * K + k].y;
    out[t] = w * (sv ? Zv : Zu)[e * K + k];
}

// sum of the evolution partials (distributed: all-reduced before the decision)
template <typename real>
__global__ __launch_bounds__(256) void k_sx_partsum(int nparts, const real *__restrict__ part,
                                                   const Ctrl<real> *ctrl, real *out) {
    __shared__ real red[kBlock / kWave];
    if (ctrl->halt) return;
    real s = real(0);
    for (int i = threadIdx.x; i < nparts; i += kBlock) s += part[i];
    s = block_sum(s, red);
    if (threadIdx.x == 0) *out = s;
}

template <typename real>
__global__ __launch_bounds__(256) void k_sx_finalize(int nparts,
                                                     const real *__restrict__ part,
                                                     long V, int track,
                                                     Ctrl<real> *ctrl,
                                                     real *__restrict__ Dif,
                                                     const real *total) {
    __shared__ real red[kBlock / kWave];
    if (ctrl->halt) return;
    real s = real(0);
    if (track) {
        if (total) {
            s = *total;
        } else {
            for (int i = threadIdx.x; i < nparts; i += kBlock) s += part[i];
            s = block_sum(s, red);
        }
    }
    if (threadIdx.x != 0) return;
    int it = ctrl->it;
    if (track) {
        real dif = s;
        if (track == 1) dif /= V;  // relative l1 evolution (ref :688)
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

// objective (ref :476-544): loss partials per vertex, TV partials per edge
template <typename real>
__global__ __launch_bounds__(256) void k_sx_obj_vertex(int V, SxConst<real> c,
                                                       const real *__restrict__ La_f,
                                                       const real *__restrict__ P,
                                                       const real *__restrict__ Q,
                                                       real *__restrict__ part,
                                                       const Ctrl<real> *ctrl) {
    if (ctrl && ctrl->obj_it >= ctrl->it) return;
    __shared__ real red[kBlock / kWave];
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    real t = real(0);
    if (v < V) {
        const int K = c.K;
        const long b = (long)v * K;
        if (c.loss == LOSS_LINEAR) {
            for (int k = 0; k < K; k++) t -= P[b + k] * Q[b + k];
        } else if (c.loss == LOSS_QUAD) {
            real s = real(0);
            for (int k = 0; k < K; k++) { const real d = P[b + k] - Q[b + k]; s += d * d; }
            t = La_f ? La_f[v] * s : s;
        } else {
            real s = real(0);
            for (int k = 0; k < K; k++) {
                const real q = c.alK + c.al1 * Q[b + k];
                // the reference evaluates log in double (C ::log)
                s = (real)((double)s + (double)q * log((double)(q / (c.alK + c.al1 * P[b + k]))));
            }
            t = La_f ? La_f[v] * s : s;
        }
    }
    t = block_sum(t, red);
    if (threadIdx.x == 0) part[blockIdx.x] = t;
}

template <typename real>
__global__ __launch_bounds__(256) void k_sx_obj_edge(long E, int K,
                                                     const int *__restrict__ Eu,
                                                     const int *__restrict__ Ev,
                                                     const real *__restrict__ La_d1,
                                                     const real *__restrict__ P,
                                                     real *__restrict__ part,
                                                     const Ctrl<real> *ctrl) {
    if (ctrl && ctrl->obj_it >= ctrl->it) return;
    __shared__ real red[kBlock / kWave];
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    real t = real(0);
    if (e < E) {
        const long u = (long)Eu[e] * K, v = (long)Ev[e] * K;
        real b = real(0);
        for (int k = 0; k < K; k++) {
            const real d = P[u + k] - P[v + k];
            if (d < real(0)) b -= d; else b += d;
        }
        t = La_d1[e] * b;
    }
    t = block_sum(t, red);
    if (threadIdx.x == 0) part[blockIdx.x] = t;
}

template <typename real>
__global__ __launch_bounds__(256) void k_sx_obj_finalize(const real *__restrict__ part,
                                                         int nbv, int nbe, int quad,
                                                         Ctrl<real> *ctrl,
                                                         real *__restrict__ Obj,
                                                         real *__restrict__ sums) {
    __shared__ real red[2][kBlock / kWave];
    if (ctrl->obj_it >= ctrl->it) return;
    real l = real(0), tv = real(0);
    for (int i = threadIdx.x; i < nbv; i += kBlock) l += part[i];
    for (int i = threadIdx.x; i < nbe; i += kBlock) tv += part[nbv + i];
    l = block_sum(l, red[0]);
    tv = block_sum(tv, red[1]);
    if (threadIdx.x != 0) return;
    if (sums) {  // distributed: all-reduced, then k_sx_obj_write
        sums[0] = l;
        sums[1] = tv;
        return;
    }
    if (quad) l *= real(0.5);
    Obj[ctrl->it] = l + tv;
    ctrl->obj_it = ctrl->it;
}

template <typename real>
__global__ void k_sx_obj_write(const real *__restrict__ sums, int quad, Ctrl<real> *ctrl,
                               real *__restrict__ Obj) {
    if (ctrl->obj_it >= ctrl->it) return;
    real l = sums[0];
    if (quad) l *= real(0.5);
    Obj[ctrl->it] = l + sums[1];
    ctrl->obj_it = ctrl->it;
}

// ---------------------------------------------------------------- session
// --------------------------------------- tile order (K <= 64, one GPU) --
// Large single-GPU sessions keep their edges in TILE order: stably sorted
// by (u block, v block), the blocks the fused vertex sweep's workgroups own
// (vb vertices).  Every edge-indexed array (Zu, Zv, A1, La_d1, Eu, Ev)
// follows, so block b's u-end rows of Z are one contiguous run and its v-end
// rows a few runs, one per (u block, b) tile, each read by workgroup b alone:
// on a grid in its natural order the v ends of a row's edges interleave
// with the in-row ones, so the K-wide Z runs of one 128-byte line belonged
// to two workgroups a grid row apart and were fetched twice.  The
// incidence keys keep the original edge ids, so every per-(v, k) sum still
// runs in the reference's (e, side) order (ref :636-648).
__global__ void k_sx_tile_keys(long E, int vb, int vbits, const int *__restrict__ Eu,
                               const int *__restrict__ Ev, unsigned long long *__restrict__ keys,
                               unsigned *__restrict__ vals) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    keys[e] = ((unsigned long long)(Eu[e] / vb) << vbits) | (unsigned)(Ev[e] / vb);
    vals[e] = (unsigned)e;
}

// position p takes edge perm[p] (its original id: the incidence keys)
__global__ void k_sx_tile_order(long E, const unsigned *__restrict__ perm,
                                const int *__restrict__ Eu, const int *__restrict__ Ev,
                                int *__restrict__ nEu, int *__restrict__ nEv) {
    const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= E) return;
    const unsigned q = perm[p];
    nEu[p] = Eu[q];
    nEv[p] = Ev[q];
}

template <typename real>
__global__ void k_sx_permute(long E, const unsigned *__restrict__ perm, const real *__restrict__ src,
                             real *__restrict__ dst) {
    const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < E) dst[p] = src[perm[p]];
}

// sl[address] = the slot of the edge end at that address (e: u end, E + e:
// v end) in its vertex block's CSR list (vb vertices per block; clamped:
// a block past 65,535 entries has no record)
__global__ void k_sxt_slots(int V, int vb, const int *__restrict__ ptr,
                            const unsigned *__restrict__ idx, unsigned short *__restrict__ sl) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const int base = ptr[v - v % vb];
    for (int j = ptr[v]; j < ptr[v + 1]; j++) {
        const int d = j - base;
        sl[idx[j]] = (unsigned short)(d < 65535 ? d : 65535);
    }
}

// ustart[b] = first position whose u end lies in block >= b (edges sorted
// by u block), ustart[nb] = E
__global__ void k_sxt_ustart(long E, int nb, int vb, const int *__restrict__ Eu,
                             int *__restrict__ ustart) {
    const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p > E) return;
    const int lo = p == 0 ? 0 : Eu[p - 1] / vb + 1;
    const int hi = p == E ? nb : Eu[p] / vb;
    for (int b = lo; b <= hi; b++) ustart[b] = (int)p;
}

// v-end runs: maximal stretches of positions whose v end lies in one block
__global__ void k_sxt_runs_count(long E, int vb, const int *__restrict__ Ev, int *__restrict__ cnt) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= E) return;
    const int b = Ev[i] / vb;
    if (i == 0 || Ev[i - 1] / vb != b) atomicAdd(cnt + b, 1);
}
__global__ void k_sxt_runs_fill(long E, int vb, const int *__restrict__ Ev,
                                const int *__restrict__ tptr, int *__restrict__ fill,
                                int *__restrict__ tstart, int *__restrict__ tlen) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= E) return;
    const int b = Ev[i] / vb;
    if (i != 0 && Ev[i - 1] / vb == b) return;
    long q = i + 1;
    while (q < E && Ev[q] / vb == b) q++;
    const int j = tptr[b] + atomicAdd(fill + b, 1);
    tstart[j] = (int)i;
    tlen[j] = (int)(q - i);
}

// block b's record (sx_tile_sum): [runs, u start, u count, (v start, v
// count) x runs - 1]; 0 runs (the CSR gather) when it has more than kSxRuns
// runs or its list exceeds the LDS (cap reals, K per entry)
__global__ void k_sxt_rec(int nb, int V, int vb, int K, int cap, const int *__restrict__ ptr,
                          const int *__restrict__ ustart, const int *__restrict__ tptr,
                          const int *__restrict__ tstart, const int *__restrict__ tlen,
                          int *__restrict__ rec, int *__restrict__ nok) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    int *r = rec + (long)b * kSxRec;
    for (int q = 0; q < kSxRec; q++) r[q] = 0;
    const long v0 = (long)b * vb, v1 = min(v0 + vb, (long)V);
    const long n = (long)ptr[v1] - ptr[v0];
    const int t0 = tptr[b], nt = tptr[b + 1] - t0;
    if (nt + 1 > kSxRuns || n * K > cap) return;
    r[0] = nt + 1;
    r[1] = ustart[b];
    r[2] = ustart[b + 1] - ustart[b];
    for (int q = 0; q < nt; q++) {
        r[3 + 2 * q] = tstart[t0 + q];
        r[4 + 2 * q] = tlen[t0 + q];
    }
    atomicAdd(nok, 1);
}

// *bad += the entries of La_d1 that differ from La_d1[0]
template <typename real>
__global__ void k_sx_uniform_check(long E, const real *__restrict__ x, int *__restrict__ bad) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < E && x[e] != x[0]) atomicAdd(bad, 1);
}

// 1/Aux per vertex: label 0's (every label's, before a reconditioning)
template <typename real>
__global__ void k_sx_inv_vertex(int V, int K, const real *__restrict__ invAux,
                                real *__restrict__ invV) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < V) invV[v] = invAux[(long)v * K];
}

// P from the .x half of the (P, step) pairs (SxVArgs::nop)
template <typename real>
__global__ void k_sx_p_from_pf(long n, const SxR2<real> *__restrict__ PF, real *__restrict__ P) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) P[i] = PF[i].x;
}

template <typename real>
static void sx_copy_in(DevBuf<real> &d, const void *src, size_t n, int mem, hipStream_t s,
                       HostPins &pins) {
    if (!src || !n) { d.release(); return; }
    d.alloc(n);
    if (mem == PFDR_MEM_DEVICE)
        PFDR_HIP(hipMemcpyAsync(d.p, src, n * sizeof(real), hipMemcpyDeviceToDevice, s));
    else
        pins.copy(d.p, src, n * sizeof(real), hipMemcpyHostToDevice);
}

// proj_simplex_metric: a segment of G = 4..64 lanes per column with J
// coordinates per lane (D <= 1024), else a wave per column in memory
template <typename real>
static void launch_proj(real *X, const real *M, int D, int N, int nm, const real *A, int na,
                        unsigned char *I, hipStream_t s) {
    auto reg = [&](auto Gc, auto Jc) {
        constexpr int G = decltype(Gc)::value, J = decltype(Jc)::value;
        k_proj_wave<real, G, J><<<grid_for((long)N * G), kBlock, 0, s>>>(X, M, D, N, nm, A, na);
    };
    using std::integral_constant;
    if (D <= 4) reg(integral_constant<int, 4>{}, integral_constant<int, 1>{});
    else if (D <= 8) reg(integral_constant<int, 8>{}, integral_constant<int, 1>{});
    else if (D <= 16) reg(integral_constant<int, 16>{}, integral_constant<int, 1>{});
    else if (D <= 32) reg(integral_constant<int, 32>{}, integral_constant<int, 1>{});
    else if (D <= 64) reg(integral_constant<int, 64>{}, integral_constant<int, 1>{});
    else if (D <= 128) reg(integral_constant<int, 64>{}, integral_constant<int, 2>{});
    else if (D <= 256) reg(integral_constant<int, 64>{}, integral_constant<int, 4>{});
    else if (D <= 512) reg(integral_constant<int, 64>{}, integral_constant<int, 8>{});
    else if (D <= 1024) reg(integral_constant<int, 64>{}, integral_constant<int, 16>{});
    else k_proj_mem<real><<<grid_for((long)N * kWave), kBlock, 0, s>>>(X, M, D, N, nm, A, na, I);
    PFDR_HIP(hipGetLastError());
}

template <typename real>
class SimplexSession final : public SessionBase {
  public:
    explicit SimplexSession(const pfdr_problem *p);
    ~SimplexSession() override {
        if (hctrl_) {
            (void)hipStreamSynchronize(stream);  // no control-block copy in flight
            pinned_small_put(hctrl_);
        }
        for (Ctrl<real> *c : snap_) if (c) pinned_small_put(c);
        for (hipEvent_t e : snapev_) if (e) (void)hipEventDestroy(e);
        drop_graphs();
        for (hipEvent_t e : evv_) if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : evd_) if (e) (void)hipEventDestroy(e);
        if (evs_) {
            (void)hipStreamSynchronize(evs_);
            (void)hipStreamDestroy(evs_);
        }
    }
    int run(int iters) override;
    void result(void *X_host, int *it, void *Obj_host, void *Dif_host) override;
    void *device_x() override {
        sync_p(it_);
        PFDR_HIP(hipStreamSynchronize(stream));
        return Pb(it_);
    }
    void on_stop_or_recond();

  private:
    SxConst<real> c_;
    int V_, K_, itMax_, verbose_;
    int Vg_;        // owned + ghost vertices (distributed)
    long Vglob_;    // vertices over all ranks
    long E_, EK_, VK_, R_ = 0;
    std::unique_ptr<Halo> halo_;  // vertex partition (null on one GPU)
    void wait_stream();
    DevBuf<real> red_;            // all-reduced scalars
    real rho_, condMin_, difTol_, difRcd_, cap_;
    bool rec_obj_, rec_dif_;
    int track_;  // 0, 1 (l1 evolution), 2 (labels)
    // evolution sum with the reference's sequential rounding (PFDR_EVOLUTION_*,
    // include/pfdr_mi355x.h): the vertex sweep stores the terms in the
    // reference's order (v K + k, or v for label changes), one binade-scan sum
    // (mono_sum) replaces the block partials' tree
    bool seqdif_ = false;
    long nterms_ = 0;
    DevBuf<real> terms_;
    DevBuf<char> dws_;
    static constexpr long kSeqDifMin = 1L << 17;  // AUTO: sums of at least this many terms
    // partitions: the ranks' terms summed rank to rank in the caller's order
    // (ChainSum); a relabelled partition (vtx_label) first routes each
    // vertex's K terms to the rank whose caller-order slice holds its label
    // (TermRoute), then chains.  Label counts (track 2) add 0 / 1: exact in
    // any order, so partitions keep the tree for them.
    ChainSum<real> chain_;
    TermRoute<real> route_;
    // the evolution sums' transport: a speculative partition's own split one
    // (beside the next iteration's exchanges, QuadSession::evtr_)
    std::unique_ptr<Transport> evtr_;
    Transport &etr() { return evtr_ ? *evtr_ : *halo_->tr; }
    void seq_evolution(real *terms, hipStream_t s);
    // Speculative iteration (sequential evolution, difRcd = 0, no objective
    // record; one GPU or a partition), as the quadratic session's spec_: the
    // sum and the decision on iteration t run on evs_ beside the sweeps of
    // t + 1 ... t + D - 1 (depth D = sd_: 2, or 4 on three or more ranks), P
    // and (P, step) cycle through D buffers (iteration t reads Pb(t - 1),
    // writes Pb(t)), the terms through D; a stop at t leaves P_t in Pb(t) and
    // the speculative iterations after it are discarded.
    static constexpr int kSpecMax = 4;
    bool spec_ = false;
    int sd_ = 2;
    int it0_ = 0;
    DevBuf<real> Px_[kSpecMax - 1];           // P buffers 1 .. D - 1 (0 is P_)
    DevBuf<SxR2<real>> PFx_[kSpecMax - 1];    // (P, step) likewise
    real *Pb(int t) { return spec_ && t % sd_ ? Px_[t % sd_ - 1].p : P_.p; }
    SxR2<real> *PFb(int t) { return spec_ && t % sd_ ? PFx_[t % sd_ - 1].p : PF_.p; }
    hipStream_t evs_ = nullptr;  // the decisions' stream (null: PFDR_SPEC_SERIAL, the session's)
    hipStream_t evs() const { return evs_ ? evs_ : stream; }
    hipEvent_t evv_[kSpecMax] = {}, evd_[kSpecMax] = {};
    // pipelined gated runs (QuadSession::run_pipelined): control-block
    // snapshots of two chunks in flight
    Ctrl<real> *snap_[2] = {};
    hipEvent_t snapev_[2] = {};
    void body_spec(int i, int n);
    void sweeps(const Ctrl<real> *c, int t);  // edge + vertex pass of iteration t
    DevBuf<int> Eu_, Ev_;
    DevBuf<real> La_d1_, La_f_, Q_, P_, Pavg_, Ga_, GaQ_, invAux_, lab_;
    // (P, explicit step) pairs per (v, k), ghosts included: written with P
    // by the vertex sweep, one access per edge end in the edge sweep
    DevBuf<SxR2<real>> PF_;
    DevBuf<real> Zu_, A1_, wz_, part_, opart_, Obj_, Dif_;
    real *zv_ = nullptr;  // the v ends' Z (inside Zu_'s allocation)
    DevBuf<SxR2<real>> GI_;  // (Ga before normalisation, 1/Aux) per (v, k), ghosts included
    DevBuf<real> GaU_;       // its Ga half alone (one GPU: the edge sweep's SxEdgeFast)
    DevBuf<real> AW_;        // W / Ga per (v, k) with one La_d1 value (SxEdgeFast::AW)
    // stored prox weights/thresholds of the non-linear losses for odd K (one
    // (e, k) per lane); even K takes two per lane and recomputes them from
    // the factors (C4: 1.076 -> 0.950 ms, r1zw; odd K stored: 1.24 vs 1.30 ms)
    DevBuf<real> Wd1u_, Wd1v_, Th_;
    bool sx_pw_ = true;
    DevBuf<Ctrl<real>> ctrl_;
    Ctrl<real> *hctrl_ = nullptr;
    Incidence inc_;
    HostPins pins_;  // caller arrays pinned for the setup copies
    int nbv_, nbe_;
    int vb_ = 0, nbs_ = 0;  // fused vertex sweep (K <= 64): vertices per block, blocks
    int nbw_ = 0;           // wide vertex sweep (K > 64): blocks
    int gnv_ = 0;           // its vertices per group (0: a wave per vertex, in memory)
    DevBuf<unsigned char> act_;  // its active sets when K > 1024
    // tile order (k_sx_tile_keys; PFDR_SX_TILE = 0 off, 1 on, default from
    // kSxTileMinVK (edge, label) entries)
    bool sxtile_ = false;
    static constexpr long kSxTileMinVK = 1L << 21;
    int sxtm_ = 2, tbv_ = 0, nbt_ = 0;  // items per lane, tile block vertices, tile blocks
    DevBuf<int> trec_;              // per tile block: its runs (k_sxt_rec)
    DevBuf<unsigned short> sl_;     // slot of every edge end (k_sxt_slots)
    DevBuf<unsigned> idxp_;         // padded block lists (SxVArgs::idxp), capb_ wide
    int capb_ = 0;
    // the one-GPU fused sweep's workgroups: snt_ lanes, svb_ vertices,
    // snb_ blocks (PFDR_SX_NT = 64, 128, 256; fused_sweep_setup)
    int snt_ = kBlock, svb_ = 0, snb_ = 0;
    bool zoff_ = false;  // the padded lists hold Z offsets (SxVArgs::zoff)
    // the one-GPU fused sweep on workgroups of M vertex blocks (M items per
    // lane, k_sx_vertex_tile without staging; PFDR_SX_M = 1, 2, 4): sxm_ > 1
    int sxm_ = 1;
    void fused_sweep_setup();
    void build_sx_tiles();
    // one La_d1 for every edge (k_sx_uniform_check at setup): a kernel argument
    bool la_u_ = false;
    real la0_ = real(0);
    DevBuf<real> invV_;  // 1/Aux per vertex (SxVArgs::invV), before any reconditioning
    // P kept only in PF's .x half by the sweeps (SxVArgs::nop): every session
    // but the one-workgroup one; sync_p(t) writes Pb(t) from PFb(t) for the
    // readers of P (objective, reconditioning, result)
    bool plazy_ = false;
    void sync_p(int t);
    // the edge sweep's metric-only gathers (SxEdgeFast): one GPU, before A1
    SxEdgeFast<real> efast() const {
        SxEdgeFast<real> f{};
        f.la0 = la0_;
        f.la_u = la_u_ ? 1 : 0;
        if (GaU_.p && !A1_.p) {
            f.GaU = GaU_.p;
            f.invV = invV_.p;
            f.AW = AW_.p;
        }
        return f;
    }
    // the fused vertex sweep forms W*Z from the gathered Z and W (K contiguous
    // words per incidence), so the edge sweep neither reads W nor writes
    // contributions: 28 instead of 44 streamed bytes per (e, k) (C4: 2.42 ->
    // 2.17 ms/iteration)
    // XCD-aware block order: runs of 64 edge blocks per XCD (C4 edge sweep
    // 1.275 -> 1.244 ms, r1zm); the vertex sweep in plain order
    static constexpr int sx_xcd_e_ = 64, sx_xcd_v_ = 0;
    int it_ = 0;
    bool stopped_ = false;
    int chunk_ = 32;
    int next_print_ = 0;
    // hipGraph of a chunk of bodies (single GPU, no objective record,
    // unprofiled; re-captured after a reconditioning): small problems --
    // cut pursuit's reduced ones -- are otherwise bound by the host's three
    // launches per iteration.
    bool graphs_ok_ = false;
    std::map<int, hipGraphExec_t> graphs_;
    void run_bodies(int n);
    bool capturable_ = false;  // prepare(): graphs of any run length on request
  public:
    void prepare(int iters) override;
  private:
    // small single-GPU problems: a chunk of iterations in one workgroup
    // (k_sx_tiny_iterate; PFDR_SX_TINY = most (edge, label) entries, 0 off)
    bool tiny_ = false;
    void tiny_chunk(int n);
    hipGraphExec_t chunk_graph(int n);
    void drop_graphs() {
        for (auto &kv : graphs_) (void)hipGraphExecDestroy(kv.second);
        graphs_.clear();
    }

    void precondition(bool init);
    void objective();
    void body();
    // K-wide ghost rows of a [Vg][K] array from their owners
    void pullK(DevBuf<real> &b) {
        if (halo_) halo_->pull(b.p, K_ * (int)sizeof(real), stream);
    }
    void pullPF() {
        if (halo_) halo_->pull(PF_.p, K_ * (int)sizeof(SxR2<real>), stream);
    }
    void push_wz();
    template <bool SPLIT>
    void launch_m_s(const SxVArgs<real> &a) {
        const int g = xcd_grid(a.nb, a.xcd);
        if (sxm_ == 2) k_sx_vertex_tile<real, SPLIT, false, 2, false><<<g, kBlock, 0, stream>>>(a);
        else k_sx_vertex_tile<real, SPLIT, false, 4, false><<<g, kBlock, 0, stream>>>(a);
    }
    void launch_m(const SxVArgs<real> &a, bool split) {
        split ? launch_m_s<true>(a) : launch_m_s<false>(a);
    }
    template <bool SPLIT>
    void launch_fused(const SxVArgs<real> &a, int g) {
        if (snt_ == 64) k_sx_vertex_sweep<real, 64, SPLIT><<<g, 64, 0, stream>>>(a);
        else if (snt_ == 128) k_sx_vertex_sweep<real, 128, SPLIT><<<g, 128, 0, stream>>>(a);
        else k_sx_vertex_sweep<real, kBlock, SPLIT><<<g, kBlock, 0, stream>>>(a);
    }
    template <bool SPLIT, bool WA>
    void launch_tile_m(const SxVArgs<real> &a) {
        const int g = xcd_grid(a.nb, a.xcd);
        if (sxtm_ == 1) k_sx_vertex_tile<real, SPLIT, WA, 1><<<g, kBlock, 0, stream>>>(a);
        else if (sxtm_ == 2) k_sx_vertex_tile<real, SPLIT, WA, 2><<<g, kBlock, 0, stream>>>(a);
        else k_sx_vertex_tile<real, SPLIT, WA, 4><<<g, kBlock, 0, stream>>>(a);
    }
    void launch_tile(const SxVArgs<real> &a, bool split, bool wa) {
        if (split) wa ? launch_tile_m<true, true>(a) : launch_tile_m<true, false>(a);
        else wa ? launch_tile_m<false, true>(a) : launch_tile_m<false, false>(a);
    }
    template <bool SPLIT>
    void launch_wide(SxVArgs<real> a) {
        if (gnv_) {  // groups of gnv_ vertices, columns in LDS
            a.vb = gnv_;
            const size_t lds = SxGroup<real>::bytes(K_, gnv_);
            if (a.zfast && !a.A1)
                k_sx_vertex_group<real, SPLIT, true><<<nbw_, kBlock, lds, stream>>>(a);
            else
                k_sx_vertex_group<real, SPLIT><<<nbw_, kBlock, lds, stream>>>(a);
        } else {
            k_sx_vertex_wide<real, SPLIT><<<nbw_, kBlock, 0, stream>>>(a);
        }
    }
};

template <typename real>
SimplexSession<real>::SimplexSession(const pfdr_problem *p) {
    if (p->K <= 0 || p->V <= 0 || p->E < 0) throw std::runtime_error("K, V must be > 0 and E >= 0");
    if (!p->X || !p->Y || !p->Eu || !p->Ev || !p->La_d1)
        throw std::runtime_error("P, Q, Eu, Ev and La_d1 are required");
    PFDR_HIP(hipGetDevice(&device));
    stream = lib_stream();
    pins_.set_stream(stream);
    hipStream_t s = stream;
    V_ = p->V; K_ = p->K; E_ = p->E;
    EK_ = E_ * K_; VK_ = (long)V_ * K_;
    itMax_ = p->itMax; verbose_ = p->verbose;
    const real al = (real)p->al;
    c_.K = K_;
    c_.alK = c_.al1 = c_.alKal1 = real(0);
    if (al == real(0)) c_.loss = LOSS_LINEAR;
    else if (al == real(1)) c_.loss = LOSS_QUAD;
    else c_.loss = LOSS_KL;  // al > 0 branch of the reference (also al > 1)
    if (real(0) < al && al < real(1)) {  // ref :387-391
        c_.alK = al / K_;
        c_.al1 = real(1) - al;
        c_.alKal1 = c_.alK / c_.al1;
    }
    if (al < real(0)) throw std::runtime_error("al must be >= 0");
    rho_ = (real)p->rho; condMin_ = (real)p->condMin;
    difTol_ = (real)p->difTol; difRcd_ = (real)p->difRcd;
    rec_obj_ = p->record_obj != 0;
    rec_dif_ = p->record_dif != 0;
    track_ = (difTol_ > real(0) || difRcd_ > real(0) || rec_dif_) ? (difTol_ >= real(1) ? 2 : 1) : 0;
    cap_ = real(1.9) * (real(2) - rho_);
    const int evo = p->evolution;
    if (evo < PFDR_EVOLUTION_AUTO || evo > PFDR_EVOLUTION_TREE)
        throw std::runtime_error("evolution must be PFDR_EVOLUTION_AUTO, _SEQUENTIAL or _TREE");
    nterms_ = track_ == 2 ? (long)V_ : (long)V_ * K_;

    const int mem = p->mem;
    const auto kind = mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    DevBuf<unsigned> eg;
    long e_offset = 0;
    if (p->nranks > 1 || p->comm) {  // vertex partition with K-wide halos
        partition_setup(p, V_, E_, halo_, Eu_, Ev_, eg, &e_offset, s);
        Vg_ = V_ + halo_->G;
        ghosts = halo_->G;
        R_ = halo_->R;
        Vglob_ = (long)halo_->off.back();
        red_.alloc(2);
    } else {
        Vg_ = V_;
        Vglob_ = V_;
        Eu_.alloc(E_ ? E_ : 1); Ev_.alloc(E_ ? E_ : 1);
        if (E_ && kind == hipMemcpyHostToDevice) {
            pins_.copy(Eu_.p, p->Eu, E_ * sizeof(int), kind);
            pins_.copy(Ev_.p, p->Ev, E_ * sizeof(int), kind);
        } else if (E_) {
            PFDR_HIP(hipMemcpyAsync(Eu_.p, p->Eu, E_ * sizeof(int), kind, s));
            PFDR_HIP(hipMemcpyAsync(Ev_.p, p->Ev, E_ * sizeof(int), kind, s));
        }
    }
    check_endpoints(Eu_.p, Ev_.p, E_, Vg_, s);
    DevBuf<unsigned> perm;  // tile order: position -> original edge id
    {
        const char *t = getenv("PFDR_SX_TILE");
        const int want = t ? atoi(t) : -1;
        // tile blocks of M vertex blocks (the staged sweep k_sx_vertex_tile,
        // PFDR_SX_STAGE=1; PFDR_SX_TILEM = 1, 2, 4; the CSR gather's blocks
        // are the M = 1 ones)
        const char *tm = getenv("PFDR_SX_TILEM");
        const char *stg = getenv("PFDR_SX_STAGE");
        sxtm_ = tm ? atoi(tm) : (stg && stg[0] == '1') ? 2 : 1;
        if (sxtm_ != 1 && sxtm_ != 2 && sxtm_ != 4) throw std::runtime_error("PFDR_SX_TILEM: 1, 2 or 4");
        const int vb = K_ <= 64 ? sxtm_ * (kBlock / K_) : 0;
        const long nb = vb ? ((long)V_ + vb - 1) / vb : 0;
        tbv_ = vb;
        nbt_ = (int)nb;
        sxtile_ = !halo_ && vb && E_ > 1 && want != 0 && (want > 0 || VK_ >= kSxTileMinVK);
        if (sxtile_) {
            int vbits = 1;
            while (vbits < 31 && (1L << vbits) < nb) vbits++;
            DevBuf<unsigned long long> k(E_), ks(E_);
            DevBuf<unsigned> v(E_);
            perm.alloc(E_);
            k_sx_tile_keys<<<grid_for(E_), kBlock, 0, s>>>(E_, vb, vbits, Eu_.p, Ev_.p, k.p, v.p);
            PFDR_HIP(hipGetLastError());
            radix_sort_pairs_stable<unsigned long long>(k.p, ks.p, v.p, perm.p, E_, 2 * vbits, s);
            DevBuf<int> nu(E_), nv(E_);
            k_sx_tile_order<<<grid_for(E_), kBlock, 0, s>>>(E_, perm.p, Eu_.p, Ev_.p, nu.p, nv.p);
            PFDR_HIP(hipGetLastError());
            std::swap(Eu_.p, nu.p);
            std::swap(Ev_.p, nv.p);
            PFDR_HIP(hipStreamSynchronize(s));
        }
        tiled_blocks = sxtile_ ? nb : 0;  // tile blocks (every one's edges in tile order)
    }
    contribution_incidence(Eu_.p, Ev_.p, E_, V_, sxtile_ ? perm.p : eg.p, e_offset, halo_.get(),
                           inc_, s);
    const size_t VgK = (size_t)Vg_ * K_;
    sx_copy_in(La_d1_, p->La_d1, E_, mem, s, pins_);
    if (sxtile_) {
        DevBuf<real> t(E_);
        k_sx_permute<real><<<grid_for(E_), kBlock, 0, s>>>(E_, perm.p, La_d1_.p, t.p);
        PFDR_HIP(hipGetLastError());
        std::swap(La_d1_.p, t.p);
        PFDR_HIP(hipStreamSynchronize(s));
    }
    if (E_) {
        DevBuf<int> bad(1);
        PFDR_HIP(hipMemsetAsync(bad.p, 0, sizeof(int), s));
        k_sx_uniform_check<real><<<grid_for(E_), kBlock, 0, s>>>(E_, La_d1_.p, bad.p);
        PFDR_HIP(hipGetLastError());
        int h = 1;
        PFDR_HIP(hipMemcpyAsync(&h, bad.p, sizeof(int), hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipMemcpyAsync(&la0_, La_d1_.p, sizeof(real), hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
        la_u_ = h == 0;
        la_uniform = la_u_ ? 1 : 0;
    }
    if (c_.loss != LOSS_LINEAR) sx_copy_in(La_f_, p->La_l1, V_, mem, s, pins_);
    for (auto q : {std::make_pair(&Q_, p->Y), std::make_pair(&P_, (const void *)p->X)}) {
        q.first->alloc(VgK);  // owned rows, then the ghosts' from their owners
        if (kind == hipMemcpyHostToDevice) pins_.copy(q.first->p, q.second, VK_ * sizeof(real), kind);
        else PFDR_HIP(hipMemcpyAsync(q.first->p, q.second, VK_ * sizeof(real), kind, s));
        pullK(*q.first);
    }
    if (K_ <= 64) {
        vb_ = kBlock / K_;
        nbs_ = (int)((V_ + vb_ - 1) / vb_);
        svb_ = vb_;  // (fused_sweep_setup may narrow the one-GPU sweep's blocks)
        snb_ = nbs_;
        // the staged tile sweep (k_sx_vertex_tile) is opt-in: PFDR_SX_STAGE=1.
        // On C4 it measured slower than the CSR gather over the same
        // tile-ordered edges (1.10 vs 0.69 ms: its staging costs more issue
        // and LDS work than the gather's one extra load round)
        const char *st = getenv("PFDR_SX_STAGE");
        if (sxtile_ && st && st[0] == '1') build_sx_tiles();
    } else {  // groups of vertices with their columns in LDS, or a wave per vertex
        gnv_ = SxGroup<real>::nv_for(K_, SxGroup<real>::kNV);
        const long per = gnv_ ? gnv_ : (long)kSxWideVpw * (kBlock / kWave);
        nbw_ = (int)((V_ + per - 1) / per);
        if (!gnv_) {  // averages and active sets in memory
            Pavg_.alloc(VK_);
            act_.alloc(VK_);
        }
    }
    PF_.alloc(VgK); Ga_.alloc(VgK); GaQ_.alloc(VgK); invAux_.alloc(VgK);
    const size_t EKn = EK_ ? EK_ : 1;
    // Zv carries the received contributions (the senders' W*Z) after its
    // E*K entries for the fused vertex sweep
    // one allocation, u ends then v ends (zv_ = Zu_.p + EKn): the fused
    // sweep's padded lists address both sides from one base (SxVArgs::zoff)
    Zu_.alloc(2 * EKn + (size_t)R_ * K_);
    zv_ = Zu_.p + EKn;
    GI_.alloc(VgK);
    if (!halo_ && E_ > 0) GaU_.alloc(VgK);
    sx_pw_ = K_ % 2 != 0;
    if (sx_pw_ && c_.loss != LOSS_LINEAR) { Wd1u_.alloc(EKn); Wd1v_.alloc(EKn); Th_.alloc(EKn); }
    wz_.alloc(2 * EKn + (size_t)R_ * K_);  // [side][e][k], then the received tail
    nbv_ = grid_for(V_);
    nbe_ = grid_for(E_);
    part_.alloc(std::max(std::max(nbv_, nbs_), nbw_));  // (nbt_ <= nbs_)
    if (rec_obj_) { opart_.alloc((size_t)nbv_ + nbe_ + 1); Obj_.alloc((size_t)itMax_ + 1); }
    if (rec_dif_) Dif_.alloc(itMax_ > 0 ? itMax_ : 1);
    if (track_ == 2) {
        lab_.alloc(V_);
        k_sx_labels<real><<<nbv_, kBlock, 0, s>>>(V_, K_, P_.p, lab_.p);
    }

    ctrl_.alloc(1);
    static_assert(sizeof(Ctrl<real>) <= kPinnedSmall, "control block");
    hctrl_ = static_cast<Ctrl<real> *>(pinned_small_get());
    std::memset(hctrl_, 0, sizeof(Ctrl<real>));
    hctrl_->obj_it = -1;
    hctrl_->itMax = itMax_;
    hctrl_->dif = difTol_ > difRcd_ ? difTol_ : difRcd_;  // ref :445
    hctrl_->difTol = difTol_;
    hctrl_->difRcd = difRcd_;
    PFDR_HIP(hipMemcpyAsync(ctrl_.p, hctrl_, sizeof(Ctrl<real>), hipMemcpyHostToDevice, s));

    if (EK_) k_sx_z_init<real><<<grid_for(EK_), kBlock, 0, s>>>(EK_, K_, Eu_.p, Ev_.p, P_.p, Zu_.p, zv_);
    precondition(true);
    invV_.alloc(V_);
    k_sx_inv_vertex<real><<<nbv_, kBlock, 0, s>>>(V_, K_, invAux_.p, invV_.p);
    if (GaU_.p && la_u_ && c_.loss != LOSS_LINEAR) {  // (the edge sweep's ratios, before A1)
        AW_.alloc(VK_);
        k_sx_aw<real><<<grid_for(VK_), kBlock, 0, s>>>(VK_, K_, la0_, invV_.p, GaU_.p, AW_.p);
    }
    k_sx_explicit<real><<<grid_for(VK_), kBlock, 0, s>>>(VK_, c_, P_.p, GaQ_.p, Q_.p, PF_.p);
    PFDR_HIP(hipGetLastError());
    pullPF();
    if (rec_obj_) objective();
    PFDR_HIP(hipStreamSynchronize(s));
    pins_.release();  // the stream was synchronised above
    stopped_ = itMax_ <= 0;
    // (RCCL partitions replay captured chunks too; loopback ranks rendezvous on the host)
    capturable_ = (!halo_ || halo_->tr->capturable()) && !rec_obj_;
    graphs_ok_ = capturable_ && itMax_ >= 2 * chunk_;
    {
        const char *t = getenv("PFDR_SX_TINY");
        const long maxEK = t ? atol(t) : kSxTinyEK;
        tiny_ = maxEK > 0 && !halo_ && !rec_obj_ && vb_ &&
                EK_ > 0 && EK_ <= maxEK && nbs_ <= (t ? kSxTinyMaxBlocks : SxTinyBlocks<real>::v) &&
                !(track_ && evo == PFDR_EVOLUTION_SEQUENTIAL);
        tiny = tiny_ ? 1 : 0;
        if (tiny_) graphs_ok_ = capturable_ = false;
        plazy_ = !tiny_;
    }
    const long nglob = track_ == 2 ? Vglob_ : Vglob_ * K_;  // terms over all ranks
    seqdif_ = track_ && !tiny_ && !(halo_ && track_ == 2) &&
              (evo == PFDR_EVOLUTION_SEQUENTIAL ||
               (evo == PFDR_EVOLUTION_AUTO && nglob >= kSeqDifMin));
    if (seqdif_) {
        const bool routed = halo_ && p->vtx_label;
        const long n = nterms_;
        terms_.alloc((size_t)n);
        if (!halo_) dws_.alloc(mono_ws_bytes<real>(n, 1));
        red_.alloc(2);
        if (routed) {
            std::vector<int64_t> h64(V_);
            PFDR_HIP(hipMemcpy(h64.data(), p->vtx_label, sizeof(int64_t) * V_,
                               mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToHost : hipMemcpyHostToHost));
            std::vector<int> h32(V_);
            for (int v = 0; v < V_; v++) {
                if (h64[v] < 0 || h64[v] >= Vglob_)
                    throw std::runtime_error("vtx_label outside [0, V_global)");
                h32[v] = (int)h64[v];
            }
            DevBuf<int> dl(V_);
            PFDR_HIP(hipMemcpy(dl.p, h32.data(), sizeof(int) * V_, hipMemcpyHostToDevice));
            check_permutation(dl.p, V_, Vglob_, *halo_->tr, s);
            route_.init(h32, Vglob_, 1, track_ == 1 ? K_ : 1, *halo_->tr, s);
        } else if (halo_) {
            chain_.init(nterms_, 1, *halo_->tr);
        }
        seqdif = 1;
        const int smode = spec_mode(p);
        const bool serial = smode == PFDR_SPEC_SERIAL;
        spec_ = difRcd_ == real(0) && !rec_obj_ && smode != PFDR_SPEC_OFF;
        if (spec_ && halo_ && !serial) evtr_ = halo_->tr->split(s);  // (collective: every rank alike)
        if (spec_) {
            sd_ = halo_ && halo_->tr->nranks >= 3 ? 4 : 2;
            DevBuf<real> t2((size_t)sd_ * n);  // terms of D iterations
            std::swap(terms_.p, t2.p);
            std::swap(terms_.n, t2.n);
            for (int k = 0; k + 1 < sd_; k++) {
                Px_[k].alloc((size_t)Vg_ * K_);
                PFx_[k].alloc((size_t)Vg_ * K_);
            }
            if (!serial) PFDR_HIP(hipStreamCreateWithFlags(&evs_, hipStreamNonBlocking));
            for (int k = 0; k < sd_; k++) {
                PFDR_HIP(hipEventCreateWithFlags(&evv_[k], hipEventDisableTiming));
                PFDR_HIP(hipEventCreateWithFlags(&evd_[k], hipEventDisableTiming));
            }
            speculative = serial ? 2 : 1;
            graphs_ok_ = capturable_ = false;  // launched directly (see QuadSession)
        }
    }
    if (vb_ && !tiny_ && !halo_) fused_sweep_setup();
    if (graphs_ok_) {  // instantiated with the setup
        try {
            (void)chunk_graph(chunk_);
        } catch (const std::exception &) {
            if (!halo_) throw;
            graphs_ok_ = capturable_ = false;  // this transport would not capture: launch directly
            (void)hipGetLastError();
        }
    }
    graphs = graphs_ok_ ? 1 : 0;
    device_bytes = (int64_t)(Eu_.n + Ev_.n + inc_.ptr.n + inc_.idx.n) * 4;
    for (DevBuf<real> *b : {&La_d1_, &La_f_, &Q_, &P_, &Pavg_, &Ga_, &GaQ_, &invAux_, &lab_,
                            &Zu_, &A1_, &Wd1u_, &Wd1v_, &Th_, &wz_, &part_, &opart_, &Obj_,
                            &Dif_, &terms_, &Px_[0], &Px_[1], &Px_[2], &route_.slice})
        device_bytes += (int64_t)(b->n * sizeof(real));
    device_bytes += (int64_t)((GI_.n + PF_.n + PFx_[0].n + PFx_[1].n + PFx_[2].n) *
                              sizeof(SxR2<real>));
}

// the runs and slots of every vertex block of a tile-ordered session (see
// sx_tile_sum); blocks whose runs or list do not fit keep the CSR gather
template <typename real>
void SimplexSession<real>::build_sx_tiles() {
    hipStream_t s = stream;
    const int nb = nbt_, vb = tbv_;
    sl_.alloc((size_t)2 * E_);
    k_sxt_slots<<<grid_for(V_), kBlock, 0, s>>>(V_, vb, inc_.ptr.p, inc_.idx.p, sl_.p);
    DevBuf<int> ustart((size_t)nb + 1), cnt(nb), fill(nb), nok(1);
    k_sxt_ustart<<<grid_for(E_ + 1), kBlock, 0, s>>>(E_, nb, vb, Eu_.p, ustart.p);
    PFDR_HIP(hipMemsetAsync(cnt.p, 0, sizeof(int) * nb, s));
    PFDR_HIP(hipMemsetAsync(fill.p, 0, sizeof(int) * nb, s));
    PFDR_HIP(hipMemsetAsync(nok.p, 0, sizeof(int), s));
    k_sxt_runs_count<<<grid_for(E_), kBlock, 0, s>>>(E_, vb, Ev_.p, cnt.p);
    PFDR_HIP(hipGetLastError());
    std::vector<int> h(nb), tp((size_t)nb + 1, 0);
    PFDR_HIP(hipMemcpyAsync(h.data(), cnt.p, sizeof(int) * nb, hipMemcpyDeviceToHost, s));
    PFDR_HIP(hipStreamSynchronize(s));
    for (int b = 0; b < nb; b++) tp[b + 1] = tp[b] + h[b];
    DevBuf<int> tptr((size_t)nb + 1), tstart(tp[nb] ? tp[nb] : 1), tlen(tp[nb] ? tp[nb] : 1);
    PFDR_HIP(hipMemcpyAsync(tptr.p, tp.data(), sizeof(int) * (nb + 1), hipMemcpyHostToDevice, s));
    k_sxt_runs_fill<<<grid_for(E_), kBlock, 0, s>>>(E_, vb, Ev_.p, tptr.p, fill.p, tstart.p, tlen.p);
    trec_.alloc((size_t)nb * kSxRec);
    k_sxt_rec<<<grid_for(nb), kBlock, 0, s>>>(nb, V_, vb, K_, sxtm_ * SxTileCap<real>::v, inc_.ptr.p,
                                              ustart.p, tptr.p, tstart.p, tlen.p, trec_.p, nok.p);
    PFDR_HIP(hipGetLastError());
    int n = 0;
    PFDR_HIP(hipMemcpyAsync(&n, nok.p, sizeof(int), hipMemcpyDeviceToHost, s));
    PFDR_HIP(hipStreamSynchronize(s));
    record_blocks = n;  // (tiled_blocks: every block's edges are in tile order)
}

// ref :64-370
template <typename real>
void SimplexSession<real>::precondition(bool init) {
    hipStream_t s = stream;
    ProfScope ps(prof, init ? "precondition" : "recondition", s);
    const int gE = grid_for(EK_), gV = grid_for(VK_);
    const bool first_recond = !init && !A1_.p;
    if (!init) {
        k_sx_recover<real><<<nbv_, kBlock, 0, s>>>(V_, c_, La_f_.p, Q_.p, GaQ_.p, Ga_.p);
        pullK(Ga_);
        if (EK_) k_sx_subgrad<real><<<gE, kBlock, 0, s>>>(EK_, c_, Eu_.p, Ev_.p, P_.p, Q_.p, Ga_.p,
                                                          GaQ_.p, first_recond ? nullptr : A1_.p,
                                                          La_d1_.p, invAux_.p, Zu_.p, zv_);
    }
    if (first_recond) A1_.alloc(EK_ ? EK_ : 1);  // a leaves La_d1 for good
    k_sx_hessian<real><<<gV, kBlock, 0, s>>>(VK_, c_, La_f_.p, P_.p, Q_.p, Ga_.p);
    if (EK_) k_sx_d1_weights<real><<<gE, kBlock, 0, s>>>(EK_, K_, Eu_.p, Ev_.p, La_d1_.p, init ? 1 : 0,
                                                         condMin_, P_.p, A1_.p, wz_.p);
    if (halo_) halo_->push(wz_.p, wz_.p + 2 * EK_, K_ * (int)sizeof(real), s);
    k_sx_precond_vertex<real><<<gV, kBlock, 0, s>>>(VK_, c_, inc_.ptr.p, inc_.idx.p, wz_.p,
                                                    La_f_.p, Q_.p, cap_, Ga_.p, invAux_.p, GaQ_.p);
    pullK(Ga_);
    pullK(invAux_);
    pullK(GaQ_);
    if (EK_ && !init)
        k_sx_recond_edge<real><<<gE, kBlock, 0, s>>>(EK_, c_, Eu_.p, Ev_.p, A1_.p, invAux_.p, Ga_.p,
                                                     GaQ_.p, P_.p, Q_.p, Zu_.p, zv_);
    k_sx_gi_pack<real><<<grid_for((long)Vg_ * K_), kBlock, 0, s>>>((long)Vg_ * K_, Ga_.p,
                                                                  invAux_.p, GI_.p, GaU_.p);
    if (EK_ && Th_.p)
        k_sx_prox_store<real><<<gE, kBlock, 0, s>>>(EK_, K_, Eu_.p, Ev_.p, A1_.p, La_d1_.p, GI_.p,
                                                    Wd1u_.p, Wd1v_.p, Th_.p);
    k_sx_normalise<real><<<nbv_, kBlock, 0, s>>>(V_, K_, Ga_.p);
    PFDR_HIP(hipGetLastError());
}

template <typename real>
void SimplexSession<real>::objective() {
    hipStream_t s = stream;
    sync_p(0);  // (no objective record in a speculative session: P_)
    k_sx_obj_vertex<real><<<nbv_, kBlock, 0, s>>>(V_, c_, La_f_.p, P_.p, Q_.p, opart_.p, ctrl_.p);
    if (E_) k_sx_obj_edge<real><<<nbe_, kBlock, 0, s>>>(E_, K_, Eu_.p, Ev_.p, La_d1_.p, P_.p,
                                                        opart_.p + nbv_, ctrl_.p);
    k_sx_obj_finalize<real><<<1, kBlock, 0, s>>>(opart_.p, nbv_, E_ ? nbe_ : 0,
                                                 c_.loss == LOSS_QUAD, ctrl_.p, Obj_.p,
                                                 halo_ ? red_.p : nullptr);
    if (halo_) {
        halo_->tr->allreduce_sum(red_.p, 2, sizeof(real) == 4 ? PFDR_F32 : PFDR_F64, s);
        k_sx_obj_write<real><<<1, 1, 0, s>>>(red_.p, c_.loss == LOSS_QUAD, ctrl_.p, Obj_.p);
    }
    PFDR_HIP(hipGetLastError());
}

// The one-GPU fused sweep (K <= 64, not the one-workgroup path): its
// workgroup width and the padded block lists.  Narrower workgroups put more
// of them on a CU: the sweep's time is the latency of each block's chain
// (list and pointers, gathers, projection walk, stores), hidden by the other
// blocks in flight.  Its evolution partials are per workgroup, so a tracked
// solve with the tree statistic keeps the 256-lane blocks (its Dif rounds as
// before); the sequential statistic and untracked solves take PFDR_SX_NT.
template <typename real>
void SimplexSession<real>::fused_sweep_setup() {
    hipStream_t s = stream;
    snt_ = kBlock;
    svb_ = vb_;
    snb_ = nbs_;
    const char *ntv = getenv("PFDR_SX_NT");
    const int nt = ntv ? atoi(ntv) : kSxNtDefault;
    if (nt != 64 && nt != 128 && nt != 256) throw std::runtime_error("PFDR_SX_NT: 64, 128 or 256");
    const char *mv = getenv("PFDR_SX_M");
    sxm_ = mv ? atoi(mv) : kSxMDefault;
    if (sxm_ != 1 && sxm_ != 2 && sxm_ != 4) throw std::runtime_error("PFDR_SX_M: 1, 2 or 4");
    if (trec_.p) sxm_ = 1;  // (the staged sweep has its own blocks)
    if (sxm_ > 1) {  // workgroups of sxm_ vertex blocks (their partials: the 256-lane sweep's)
        tbv_ = sxm_ * vb_;
        nbt_ = (int)((V_ + tbv_ - 1) / tbv_);
        svb_ = tbv_;  // (the padded lists below cover a workgroup's vertices)
        snb_ = nbt_;
    } else if ((!track_ || seqdif_) && !trec_.p && K_ <= nt) {
        snt_ = nt;
        svb_ = nt / K_;
        snb_ = (int)((V_ + svb_ - 1) / svb_);
        if ((size_t)snb_ > part_.n) part_.alloc((size_t)snb_);
    }
    // padded block lists (PFDR_SX_PAD=0 off): when the widest block's list
    // fits the sweep's LDS list and the padding costs at most half the lists'
    // size (regular graphs)
    const char *pd = getenv("PFDR_SX_PAD");
    if (E_ > 0 && !(pd && pd[0] == '0')) {
        DevBuf<int> cb(1);
        PFDR_HIP(hipMemsetAsync(cb.p, 0, sizeof(int), s));
        k_sx_block_max<<<grid_for(snb_), kBlock, 0, s>>>(snb_, svb_, V_, inc_.ptr.p, cb.p);
        PFDR_HIP(hipGetLastError());
        int h = 0;
        PFDR_HIP(hipMemcpyAsync(&h, cb.p, sizeof(int), hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
        const long n = (long)snb_ * h;
        if (h > 0 && h <= kSxPadPer * snt_ && n <= 3 * E_) {  // (2E list entries, at most 1.5 x)
            // (sxm_ > 1: lists of kSxPadPer * 256 entries at most, as snt_ = 256)
            capb_ = h;
            idxp_.alloc((size_t)n);
            // (one GPU: no received entries; one edge weight until A1 exists)
            zoff_ = la_u_ && 2 * EK_ + K_ <= 0xffffffffL;
            k_sx_pad_idx<<<grid_for(n), kBlock, 0, s>>>(n, h, svb_, V_, inc_.ptr.p, inc_.idx.p,
                                                        idxp_.p, E_, zoff_ ? K_ : 0);
            PFDR_HIP(hipGetLastError());
        }
    }
}

// Pb(t) from the (P, step) pairs the sweeps wrote (plazy_), ghost rows
// included (their PF rows were pulled)
template <typename real>
void SimplexSession<real>::sync_p(int t) {
    if (!plazy_) return;
    const long n = (long)Vg_ * K_;
    k_sx_p_from_pf<real><<<grid_for(n), kBlock, 0, stream>>>(n, PFb(t), Pb(t));
    PFDR_HIP(hipGetLastError());
}

// iteration t = it0_ + 1 + i of a speculative session (see spec_)
template <typename real>
void SimplexSession<real>::body_spec(int i, int n) {
    hipStream_t s = stream;
    const int t = it0_ + 1 + i;
    const int b = t % sd_;
    if (i >= sd_) PFDR_HIP(hipStreamWaitEvent(s, evd_[b], 0));  // the decision on t - D
    real *terms = terms_.p + (long)b * (terms_.n / sd_);
    real *const keep = terms_.p;
    terms_.p = terms;
    sweeps(ctrl_.p, t);
    terms_.p = keep;
    PFDR_HIP(hipEventRecord(evv_[b], s));
    const hipStream_t es = evs();
    PFDR_HIP(hipStreamWaitEvent(es, evv_[b], 0));
    seq_evolution(terms, es);  // overlaps the sweeps of t + 1 (not when serial)
    k_sx_finalize<real><<<1, kBlock, 0, es>>>(0, nullptr, Vglob_, track_, ctrl_.p,
                                                rec_dif_ ? Dif_.p : nullptr, red_.p);
    PFDR_HIP(hipGetLastError());
    PFDR_HIP(hipEventRecord(evd_[b], es));
    if (i == n - 1) PFDR_HIP(hipStreamWaitEvent(s, evd_[b], 0));  // join: the chunk's last
}

template <typename real>
void SimplexSession<real>::body() {
    hipStream_t s = stream;
    const bool gated = track_ || rec_obj_;
    const Ctrl<real> *c = gated ? ctrl_.p : nullptr;
    sweeps(c, 0);
    // (the staged tile sweep writes the 256-lane fused sweep's partials)
    const int nparts = (trec_.p || sxm_ > 1) ? nbs_ : vb_ ? snb_ : nbw_;
    if (seqdif_) {
        // the reference's sequential sum (ref :655-689), then its decision
        ProfScope ps(prof, "seq_evolution", s);
        seq_evolution(terms_.p, s);
        k_sx_finalize<real><<<1, kBlock, 0, s>>>(0, nullptr, Vglob_, track_, ctrl_.p,
                                                 rec_dif_ ? Dif_.p : nullptr, red_.p);
    } else if (gated && halo_) {
        if (track_) {
            k_sx_partsum<real><<<1, kBlock, 0, s>>>(nparts, part_.p, ctrl_.p, red_.p);
            halo_->tr->allreduce_sum(red_.p, 1, sizeof(real) == 4 ? PFDR_F32 : PFDR_F64, s);
        }
        k_sx_finalize<real><<<1, kBlock, 0, s>>>(0, nullptr, Vglob_, track_, ctrl_.p,
                                                 rec_dif_ ? Dif_.p : nullptr, red_.p);
    } else if (gated) {
        k_sx_finalize<real><<<1, kBlock, 0, s>>>(nparts, part_.p, Vglob_, track_, ctrl_.p,
                                                 rec_dif_ ? Dif_.p : nullptr, nullptr);
    }
    PFDR_HIP(hipGetLastError());
    if (rec_obj_) objective();
}

// the edge and vertex passes of one iteration (t: its number in a
// speculative session, whose P buffers alternate; else 0, in place)
template <typename real>
void SimplexSession<real>::sweeps(const Ctrl<real> *c, int t) {
    hipStream_t s = stream;
    SxR2<real> *PFin = spec_ ? PFb(t - 1) : PF_.p;
    real *Pin = spec_ ? Pb(t - 1) : P_.p;
    real *Po = spec_ ? Pb(t) : nullptr;
    SxR2<real> *PFo = spec_ ? PFb(t) : nullptr;
    if (EK_) {
        ProfScope ps(prof, "sx_edge_sweep", s);
        const int pair = K_ % 2 == 0 ? 2 : 1;  // see k_sx_edge_sweep
        const int nb = grid_for(EK_ / pair);
        const int xm = xcd_fit(nb, sx_xcd_e_);
        if (pair == 2)
            k_sx_edge_sweep<real, 2><<<xcd_grid(nb, xm), kBlock, 0, s>>>(EK_, c_, Eu_.p, Ev_.p, PFin,
                                                               Zu_.p, zv_, A1_.p, La_d1_.p, GI_.p,
                                                               Wd1u_.p, Wd1v_.p, Th_.p,
                                                               nullptr,
                                                               rho_, c, nb, xm, efast());
        else
            k_sx_edge_sweep<real, 1><<<xcd_grid(nb, xm), kBlock, 0, s>>>(EK_, c_, Eu_.p, Ev_.p, PFin,
                                                               Zu_.p, zv_, A1_.p, La_d1_.p, GI_.p,
                                                               Wd1u_.p, Wd1v_.p, Th_.p,
                                                               nullptr,
                                                               rho_, c, nb, xm, efast());
    }
    if (halo_) {
        ProfScope ps(prof, "halo_push", s);
        push_wz();
    }
    SxVArgs<real> a{};
    a.V = V_; a.vb = vb_; a.E = E_; a.c = c_; a.ptr = inc_.ptr.p; a.idx = inc_.idx.p;
    a.wz = wz_.p; a.Ga = Ga_.p; a.GaQ = GaQ_.p; a.Q = Q_.p; a.P = Pin; a.PF = PFin;
    a.Po = Po; a.PFo = PFo;
    a.lab = lab_.p; a.track = track_; a.part = part_.p; a.ctrl = c;
    a.terms = seqdif_ ? terms_.p : nullptr;
    a.Zu = Zu_.p; a.Zv = zv_; a.A1 = A1_.p; a.La_d1 = La_d1_.p; a.invAux = invAux_.p;
    a.invV = A1_.p ? nullptr : invV_.p;
    a.la0 = la0_; a.la_u = la_u_ ? 1 : 0;
    a.nop = plazy_ ? 1 : 0;
    a.idxp = idxp_.p;
    a.capb = capb_;
    a.zoff = zoff_ ? 1 : 0;
    a.EK = (unsigned)EK_;
    a.zfast = (!halo_ && la_u_ && 2 * EK_ + K_ <= 0xffffffffL) ? 1 : 0;
    if (vb_) {
        ProfScope ps(prof, "sx_vertex_sweep", s);
        a.vb = svb_;
        a.nb = snb_; a.xcd = xcd_fit(snb_, sx_xcd_v_);
        const int g = xcd_grid(snb_, a.xcd);
        if (trec_.p) {  // tile runs staged by slot (sx_tile_stage)
            a.trec = trec_.p;
            a.sl = sl_.p;
            a.nparts = nbs_;  // (a.vb: the 256-lane sweep's; the tile blocks are M of them)
            a.vb = vb_;
            a.nb = nbt_;
            a.xcd = xcd_fit(nbt_, sx_xcd_v_);
            launch_tile(a, Po != nullptr, A1_.p || !la_u_);  // (weights staged with the runs)
        } else if (sxm_ > 1) {  // workgroups of sxm_ vertex blocks, the CSR gather
            a.nparts = nbs_;
            a.vb = vb_;
            a.nb = nbt_;
            a.xcd = xcd_fit(nbt_, sx_xcd_v_);
            launch_m(a, Po != nullptr);
        } else if (Po) {
            launch_fused<true>(a, g);
        } else {
            launch_fused<false>(a, g);
        }
    } else {
        ProfScope ps(prof, "sx_vertex_wide", s);
        a.nb = nbw_; a.xs = Pavg_.p; a.act = act_.p;
        if (Po) launch_wide<true>(a);
        else launch_wide<false>(a);
    }
    if (halo_) {  // the ghosts of the buffers just written (speculative: Pb(t), PFb(t))
        ProfScope ps(prof, "halo_pull", s);
        if (!plazy_) halo_->pull(Po ? Po : P_.p, K_ * (int)sizeof(real), s);
        halo_->pull(PFo ? PFo : PF_.p, K_ * (int)sizeof(SxR2<real>), s);
    }
    PFDR_HIP(hipGetLastError());
}

// red_[0] = the evolution sum over every (vertex, label) in the caller's
// order, rounded as the reference's one-thread loop
template <typename real>
void SimplexSession<real>::seq_evolution(real *terms, hipStream_t s) {
    const int *halt = &ctrl_.p->halt;
    if (!halo_) {
        mono_sum<real>(nterms_, terms, nullptr, 0, nullptr, red_.p, nullptr, dws_.p, s, 1, 0,
                       halt);
    } else if (!route_.ready()) {
        chain_.run(etr(), terms, 0, red_.p, halt, s);
    } else {
        route_.run(etr(), terms, 0, red_.p, halt, s);
    }
}

// K-wide DR contributions of ghost-vertex ends to their owners
template <typename real>
void SimplexSession<real>::push_wz() {
    const int eb = K_ * (int)sizeof(real);
    const long n = halo_->push_send_off[halo_->tr->nranks];
    real *buf = (real *)halo_->push_buffer(eb);
    if (n) {
        k_sx_pack_wz<real><<<grid_for(n * K_), kBlock, 0, stream>>>(n, K_, E_, halo_->push_addr.p,
                                                                    Eu_.p, Ev_.p, A1_.p, La_d1_.p, GI_.p,
                                                                    Zu_.p, zv_, buf);
        PFDR_HIP(hipGetLastError());
    }
    halo_->push_packed(buf, zv_ + EK_, eb, stream);  // the tail of Zv (vertex sweep)
}

template <typename real>
void SimplexSession<real>::tiny_chunk(int n) {
    const bool gated = track_ || rec_obj_;
    SxTinyArgs<real> t{};
    t.EK = EK_; t.c = c_; t.Eu = Eu_.p; t.Ev = Ev_.p; t.Zu = Zu_.p; t.Zv = zv_;
    t.A1 = A1_.p; t.La_d1 = La_d1_.p; t.Wd1u = Wd1u_.p; t.Wd1v = Wd1v_.p; t.Th = Th_.p;
    t.GI = GI_.p; t.rho = rho_;
    SxVArgs<real> &a = t.va;
    a.V = V_; a.vb = vb_; a.E = E_; a.c = c_; a.ptr = inc_.ptr.p; a.idx = inc_.idx.p;
    a.wz = wz_.p; a.Ga = Ga_.p; a.GaQ = GaQ_.p; a.Q = Q_.p; a.P = P_.p; a.PF = PF_.p;
    a.lab = lab_.p; a.track = track_; a.part = part_.p; a.ctrl = nullptr;
    a.Zu = Zu_.p; a.Zv = zv_; a.A1 = A1_.p; a.La_d1 = La_d1_.p; a.invAux = invAux_.p;
    a.nb = nbs_; a.xcd = 0;
    t.ctrl = gated ? ctrl_.p : nullptr;
    t.Dif = rec_dif_ ? Dif_.p : nullptr;
    t.V = Vglob_;
    t.iters = n;
    ProfScope ps(prof, "sx_tiny_iterate", stream);
    if (K_ % 2 == 0) k_sx_tiny_iterate<real, 2><<<1, kSxTiny, 0, stream>>>(t);
    else k_sx_tiny_iterate<real, 1><<<1, kSxTiny, 0, stream>>>(t);
    PFDR_HIP(hipGetLastError());
}

// the captured graph of a whole chunk (chunk_ bodies), instantiated once --
// at the end of the setup, and again after a reconditioning dropped it
template <typename real>
hipGraphExec_t SimplexSession<real>::chunk_graph(int n) {
    const int key = kSpecMax * n + (spec_ ? it0_ % sd_ : 0);  // speculative: P buffers by t mod D
    auto it = graphs_.find(key);
    if (it != graphs_.end()) return it->second;
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    PFDR_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    try {
        for (int i = 0; i < n; i++) spec_ ? body_spec(i, n) : body();
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

template <typename real>
void SimplexSession<real>::run_bodies(int n) {
    it0_ = it_;
    const int key = kSpecMax * n + (spec_ ? it0_ % sd_ : 0);
    if (!prof.on && capturable_ && graphs_.count(key)) {  // prepared (or whole) chunk
        PFDR_HIP(hipGraphLaunch(graphs_[key], stream));
        return;
    }
    if (!graphs_ok_ || prof.on || n != chunk_) {
        for (int i = 0; i < n; i++) spec_ ? body_spec(i, n) : body();
        return;
    }
    PFDR_HIP(hipGraphLaunch(chunk_graph(chunk_), stream));
}

// the graphs a run of `iters` iterations will replay, built now
template <typename real>
void SimplexSession<real>::prepare(int iters) {
    if (!capturable_ || iters <= 0) return;
    it0_ = it_;
    if (iters >= chunk_) (void)chunk_graph(chunk_);
    if (iters % chunk_) (void)chunk_graph(iters % chunk_);
    PFDR_HIP(hipStreamSynchronize(stream));
}

template <typename real>
int SimplexSession<real>::run(int iters) {
    const bool gated = track_ || rec_obj_;
    const int target = (int)std::min<long>((long)it_ + std::max(iters, 0), (long)itMax_);
    if (gated && !halo_ && !spec_) {
        // two chunks in flight, as QuadSession::run_pipelined: chunk k + 1 is
        // launched before the host reads chunk k's control-block snapshot; a
        // chunk launched after a stop or a reconditioning request runs
        // halted (every kernel returns at once)
        for (int k = 0; k < 2; k++) {
            if (!snap_[k]) snap_[k] = static_cast<Ctrl<real> *>(pinned_small_get());
            if (!snapev_[k]) PFDR_HIP(hipEventCreateWithFlags(&snapev_[k], hipEventDisableTiming));
        }
        int k = 0, nq = 0, ahead = it_;
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
            if (hctrl_->recond && !hctrl_->stop) {
                wait_stream();  // the chunk queued behind it ran halted
                nq = 0;
                ahead = it_;
            }
            on_stop_or_recond();
            if (!stopped_ && nq == 0 && ahead >= target) break;
        }
        wait_stream();
        if (prof.on) prof.resolve();
        return it_;
    }
    while (!stopped_ && it_ < target) {
        const int n = std::min(target - it_, chunk_);
        if (tiny_) tiny_chunk(n);
        else run_bodies(n);
        if (gated) {
            PFDR_HIP(hipMemcpyAsync(hctrl_, ctrl_.p, sizeof(Ctrl<real>), hipMemcpyDeviceToHost, stream));
            wait_stream();
            it_ = hctrl_->it;
            on_stop_or_recond();
        } else {
            it_ += n;
            if (it_ >= itMax_) stopped_ = true;
            on_stop_or_recond();
        }
    }
    wait_stream();
    if (prof.on) prof.resolve();
    return it_;
}

// after a chunk: the stop or reconditioning the control block (hctrl_, just
// read) asks for, then the progress line
template <typename real>
void SimplexSession<real>::on_stop_or_recond() {
    const bool gated = track_ || rec_obj_;
    if (gated) {
        if (hctrl_->stop) {
            stopped_ = true;
        } else if (hctrl_->recond) {
            if (verbose_) { printf("Reconditioning... "); fflush(stdout); }
            sync_p(it_);
            precondition(false);
            drop_graphs();  // kernel arguments (A1_, stored weights) may have changed
            k_sx_explicit<real><<<grid_for(VK_), kBlock, 0, stream>>>(VK_, c_, P_.p, GaQ_.p, Q_.p, PF_.p);
            PFDR_HIP(hipGetLastError());
            pullPF();
            difRcd_ *= real(0.1);  // ref :563
            hctrl_->difRcd = difRcd_;
            hctrl_->recond = 0;
            hctrl_->halt = 0;
            PFDR_HIP(hipMemcpyAsync(ctrl_.p, hctrl_, sizeof(Ctrl<real>), hipMemcpyHostToDevice, stream));
            if (verbose_) { printf("done.\n"); fflush(stdout); }
        }
    }
    if (verbose_ && (it_ >= next_print_ || stopped_)) {
        printf("iteration %d (max. %d)\n", it_, itMax_);
        if (track_ == 2)
            printf("label evolution %d (recond. %d; tol. %d)\n", (int)hctrl_->dif,
                   (int)hctrl_->difRcd, (int)difTol_);
        else if (track_ == 1)
            printf("iterate evolution %g (recond. %g; tol. %g)\n", (double)hctrl_->dif,
                   (double)hctrl_->difRcd, (double)difTol_);
        fflush(stdout);
        next_print_ = it_ + verbose_;
    }
}

// host wait for the session stream (partitioned: under the transport's watchdog)
template <typename real>
void SimplexSession<real>::wait_stream() {
    if (!halo_) { PFDR_HIP(hipStreamSynchronize(stream)); return; }
    halo_->tr->phase = "iterations";
    halo_->tr->iteration = it_;
    halo_->tr->wait(stream);
}

template <typename real>
void SimplexSession<real>::result(void *X_host, int *it, void *Obj_host, void *Dif_host) {
    hipStream_t s = stream;
    HostPins hp(s);
    if (X_host) {
        sync_p(it_);
        hp.copy(X_host, Pb(it_), sizeof(real) * VK_, hipMemcpyDeviceToHost);
    }
    if (it) *it = it_;
    if (Obj_host && rec_obj_)
        hp.copy(Obj_host, Obj_.p, sizeof(real) * (it_ + 1), hipMemcpyDeviceToHost);
    if (Dif_host && rec_dif_ && it_ > 0)
        hp.copy(Dif_host, Dif_.p, sizeof(real) * it_, hipMemcpyDeviceToHost);
    hp.release();
    PFDR_HIP(hipStreamSynchronize(s));
}

SessionBase *create_simplex_session(const pfdr_problem *p) {
    if (p->dtype == PFDR_F32) return new SimplexSession<float>(p);
    if (p->dtype == PFDR_F64) return new SimplexSession<double>(p);
    throw std::runtime_error("dtype must be PFDR_F32 or PFDR_F64");
}

template <typename real>
static int simplex_host(const char *fn, int K, int V, int E, real al, const real *La_f, real *P,
                        const real *Q, const int *Eu, const int *Ev, const real *La_d1, real rho,
                        real condMin, real difRcd, real difTol, int itMax, int *it, real *Obj,
                        real *Dif, int verbose) {
    pfdr_problem p{};
    p.kind = PFDR_KIND_SIMPLEX;
    p.dtype = sizeof(real) == 4 ? PFDR_F32 : PFDR_F64;
    p.mem = PFDR_MEM_HOST;
    p.V = V; p.E = E; p.K = K; p.al = al;
    p.X = P; p.Y = Q; p.Eu = Eu; p.Ev = Ev; p.La_d1 = La_d1; p.La_l1 = La_f;
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
            tr.finish(V, E, 0, K, its);
            return PFDR_OK;
        }
        std::unique_ptr<SimplexSession<real>> s(new SimplexSession<real>(&p));
        if (verbose) { printf("done.\nPreconditioned forward-Douglas-Rachford algorithm\n"); fflush(stdout); }
        tr.setup_done();
        s->run(itMax);
        tr.run_done();
        int its = 0;
        s->result(P, &its, Obj, Dif);
        if (it) *it = its;
        s.reset();
        tr.finish(V, E, 0, K, its);
    } catch (const HipError &h) {
        return report_error(fn, h);
    } catch (const std::exception &ex) {
        return report_error(fn, ex.what());
    }
    return PFDR_OK;
}

template <typename real>
static int proj_host(const char *fn, real *X, const real *M, int D, int N, int nm, const real *A,
                     int na) {
    if (D <= 0 || N < 0 || nm <= 0 || na <= 0 || !X || !M || !A)
        return report_error(fn, "invalid arguments");
    if (N == 0) return PFDR_OK;
    try {
        hipStream_t s = lib_stream();
        const int mm = std::min(nm, N), aa = std::min(na, N);
        DevBuf<real> dX, dM, dA;
        DevBuf<unsigned char> dI;  // active flags of the in-memory columns
        if (D > 1024) dI.alloc((size_t)D * N);
        dX.alloc((size_t)D * N);
        dM.alloc((size_t)D * mm);
        dA.alloc(aa);
        PFDR_HIP(hipMemcpyAsync(dX.p, X, sizeof(real) * D * (size_t)N, hipMemcpyHostToDevice, s));
        PFDR_HIP(hipMemcpyAsync(dM.p, M, sizeof(real) * D * (size_t)mm, hipMemcpyHostToDevice, s));
        PFDR_HIP(hipMemcpyAsync(dA.p, A, sizeof(real) * aa, hipMemcpyHostToDevice, s));
        launch_proj<real>(dX.p, dM.p, D, N, mm, dA.p, aa, dI.p, s);
        PFDR_HIP(hipMemcpyAsync(X, dX.p, sizeof(real) * D * (size_t)N, hipMemcpyDeviceToHost, s));
        PFDR_HIP(hipStreamSynchronize(s));
    } catch (const HipError &h) {
        return report_error(fn, h);
    }
    return PFDR_OK;
}

}  // namespace pfdr

extern "C" int pfdr_loss_d1_simplex_f32(int K, int V, int E, float al, const float *La_f, float *P,
                                        const float *Q, const int *Eu, const int *Ev,
                                        const float *La_d1, float rho, float condMin,
                                        float difRcd, float difTol, int itMax, int *it,
                                        float *Obj, float *Dif, int verbose) {
    return pfdr::simplex_host<float>("pfdr_loss_d1_simplex_f32", K, V, E, al, La_f, P, Q, Eu, Ev,
                                     La_d1, rho, condMin, difRcd, difTol, itMax, it, Obj, Dif,
                                     verbose);
}
extern "C" int pfdr_loss_d1_simplex_f64(int K, int V, int E, double al, const double *La_f,
                                        double *P, const double *Q, const int *Eu, const int *Ev,
                                        const double *La_d1, double rho, double condMin,
                                        double difRcd, double difTol, int itMax, int *it,
                                        double *Obj, double *Dif, int verbose) {
    return pfdr::simplex_host<double>("pfdr_loss_d1_simplex_f64", K, V, E, al, La_f, P, Q, Eu, Ev,
                                      La_d1, rho, condMin, difRcd, difTol, itMax, it, Obj, Dif,
                                      verbose);
}
extern "C" int pfdr_proj_simplex_metric_f32(float *X, const float *M, int D, int N, int nm,
                                            const float *A, int na) {
    return pfdr::proj_host<float>("pfdr_proj_simplex_metric_f32", X, M, D, N, nm, A, na);
}
extern "C" int pfdr_proj_simplex_metric_f64(double *X, const double *M, int D, int N, int nm,
                                            const double *A, int na) {
    return pfdr::proj_host<double>("pfdr_proj_simplex_metric_f64", X, M, D, N, nm, A, na);
}
