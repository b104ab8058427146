// Cut-pursuit reduced-problem builder: from the
// CP's connected components (rVc offsets into the vertex list Vc, ref
// src/CP_PFDR_graph_quadratic_d1_l1.cpp:571-597) build what CP hands to PFDR
// on every iteration (:663-841):
//   N > 0: rA = component column sums of A; preAt: rAA = rA^t rA, rY = rA^t Y
//   N < 0: rY = component sums of A^tY, rAA = double component sums of A^tA
//   N = 0: rY as above, rAA = component sums of the diagonal (or sizes)
//   L: Jacobi equilibration, squared operator norm of the equilibrated
//      matrix (pfdr_gram.hip's power method), L = l^2 c (:772-839).
// Every sum runs sequentially in the reference's order (one lane per output
// entry, products rounded before the add as with -ffp-contract=off), so rA,
// rAA and rY are bit-identical to the restatement (oracle/cp_reduce_body.h);
// the equilibrate-then-revert round trip is reproduced as the reference
// does it (its revert does not restore every bit).  Only the operator norm
// differs: the reference's starts are time-seeded (:182), ours are fixed.
// Large reduced problems (rV^2 N > 2^34 multiply-adds) compute rAA on the
// matrix cores instead (pfdr_gram.hip; tolerance, not bit-exact).
#include <cmath>
#include <stdexcept>

#include "pfdr_graph.hpp"
#include "pfdr_session.hpp"

namespace pfdr {

template <typename real>
real operator_norm_device(int M, int N, const real *A, real nTol, int itMax, int nbInit,
                          int verbose, hipStream_t s, double *gram_ms);
template <typename real>
void gram(int which, int P, long K, const real *A, long ld, real *G, hipStream_t s);

// rA[n + N rv] = sum over the component's vertices, in list order (:676-687)
template <typename real>
__global__ void k_cp_colsum(int N, int rV, const real *__restrict__ A, const int *__restrict__ rVc,
                            const int *__restrict__ Vc, real *__restrict__ rA) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    for (int rv = blockIdx.y; rv < rV; rv += gridDim.y) {
        real a = real(0);
        int s = rVc[rv];
        const int t = rVc[rv + 1];
        for (; s + 8 <= t; s += 8) {  // 8 column loads in flight, adds in order
            real x[8];
#pragma unroll
            for (int u = 0; u < 8; u++) x[u] = A[(size_t)N * Vc[s + u] + n];
#pragma unroll
            for (int u = 0; u < 8; u++) a += x[u];
        }
        for (; s < t; s++) a += A[(size_t)N * Vc[s] + n];
        rA[(size_t)N * rv + n] = a;
    }
}

// upper triangle rAA[rv + rV ru] (rv <= ru) = sum_n rA[n, rv] rA[n, ru] (:689-702)
template <typename real>
__global__ void k_cp_gram_seq(int N, int rV, const real *__restrict__ rA, real *__restrict__ rAA) {
    const int rv = blockIdx.x * blockDim.x + threadIdx.x;
    if (rv >= rV) return;
    for (int ru = blockIdx.y; ru < rV; ru += gridDim.y) {
        if (rv > ru) continue;
        // the reference's loop: a += rA[i++] * Av[n], i running down column rv
        const real *a = rA + (size_t)N * rv, *b = rA + (size_t)N * ru;
        real s = real(0);
        for (int n = 0; n < N; n++) s += a[n] * b[n];
        rAA[rv + (size_t)rV * ru] = s;
    }
}

// rY[rv] = sum_n rA[n, rv] Y[n] (:704-711)
template <typename real>
__global__ void k_cp_rY_dot(int N, int rV, const real *__restrict__ rA, const real *__restrict__ Y,
                            real *__restrict__ rY) {
    const int rv = blockIdx.x * blockDim.x + threadIdx.x;
    if (rv >= rV) return;
    const real *a = rA + (size_t)N * rv;
    real s = real(0);
    for (int n = 0; n < N; n++) s += a[n] * Y[n];
    rY[rv] = s;
}

// identity (:756-758): rAA[rv] = component size
template <typename real>
__global__ void k_cp_sizes(int rV, const int *__restrict__ rVc, real *__restrict__ rAA) {
    const int rv = blockIdx.x * blockDim.x + threadIdx.x;
    if (rv < rV) rAA[rv] = (real)(rVc[rv + 1] - rVc[rv]);
}

// upper triangle of the double component sums of A^tA (:724-741)
template <typename real>
__global__ void k_cp_ata(int V, int rV, const real *__restrict__ A, const int *__restrict__ rVc,
                         const int *__restrict__ Vc, real *__restrict__ rAA) {
    const int rv = blockIdx.x * blockDim.x + threadIdx.x;
    if (rv >= rV) return;
    for (int ru = blockIdx.y; ru < rV; ru += gridDim.y) {
        if (rv > ru) continue;
        real a = real(0);
        for (int s = rVc[ru], t = rVc[ru + 1]; s < t; s++) {
            const real *Av = A + (size_t)V * Vc[s];
            for (int q = rVc[rv], r = rVc[rv + 1]; q < r; q++) a += Av[Vc[q]];
        }
        rAA[rv + (size_t)rV * ru] = a;
    }
}

// lower triangle from the upper (:761-770)
template <typename real>
__global__ void k_cp_mirror(int rV, real *rAA) {
    const int rv = blockIdx.x * blockDim.x + threadIdx.x;
    if (rv >= rV) return;
    for (int ru = blockIdx.y; ru < rV; ru += gridDim.y)
        if (rv > ru) rAA[rv + (size_t)rV * ru] = rAA[ru + (size_t)rV * rv];
}

// l[rv] = sqrt(rAA[rv, rv]) (:778)
template <typename real>
__global__ void k_cp_diag_sqrt(int rV, const real *__restrict__ rAA, real *__restrict__ l) {
    const int rv = blockIdx.x * blockDim.x + threadIdx.x;
    if (rv < rV) l[rv] = std::sqrt(rAA[(size_t)rv * (rV + 1)]);
}

// l[rv] = ||rA[:, rv]|| summed sequentially (:803-812)
template <typename real>
__global__ void k_cp_colnorm(int N, int rV, const real *__restrict__ rA, real *__restrict__ l) {
    const int rv = blockIdx.x * blockDim.x + threadIdx.x;
    if (rv >= rV) return;
    const real *a = rA + (size_t)N * rv;
    real s = real(0);
    for (int n = 0; n < N; n++) {
        const real b = a[n];
        s += b * b;
    }
    l[rv] = std::sqrt(s);
}

// symmetric: M[rv + rV ru] /= (or *=) l[ru] l[rv] (:779-800)
template <typename real>
__global__ void k_cp_scale_sym(int rV, real *M, const real *__restrict__ l, int mul) {
    const int rv = blockIdx.x * blockDim.x + threadIdx.x;
    if (rv >= rV) return;
    for (int ru = blockIdx.y; ru < rV; ru += gridDim.y) {
        const real a = l[ru];
        real &m = M[rv + (size_t)rV * ru];
        if (mul) m *= (a * l[rv]);
        else m /= (a * l[rv]);
    }
}

// columns: M[n + N rv] /= (or *=) l[rv] (:813-825)
template <typename real>
__global__ void k_cp_scale_cols(int N, int rV, real *M, const real *__restrict__ l, int mul) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    for (int rv = blockIdx.y; rv < rV; rv += gridDim.y) {
        real &m = M[n + (size_t)N * rv];
        if (mul) m *= l[rv];
        else m /= l[rv];
    }
}

// L[rv] = l[rv] (l[rv] c) (:827-839)
template <typename real>
__global__ void k_cp_lipschitz(int rV, const real *__restrict__ l, real c, real *__restrict__ L) {
    const int rv = blockIdx.x * blockDim.x + threadIdx.x;
    if (rv >= rV) return;
    real x = l[rv];
    x *= l[rv] * c;
    L[rv] = x;
}

template <typename real>
static int cp_reduce_host(const char *fn, int N, int V, const real *A, const real *Y, int rV,
                          const int *rVc, const int *Vc, int preAt, int mem, real normTol,
                          int normItMax, int normNbInit, real *rA, real *rAA, real *rY, real *L,
                          real *Leq) {
    if (V <= 0 || rV <= 0 || rV > V || !Y || !rVc || !Vc)
        return report_error(fn, "invalid arguments");
    if (N > 0 && (!A || !rA)) return report_error(fn, "N > 0 needs A and rA");
    if (N < 0 && (!A || -N != V)) return report_error(fn, "N < 0 needs A = A^tA and N = -V");
    if (N <= 0) preAt = 1;  // ref :671
    if (preAt && (!rAA || !rY)) return report_error(fn, "rAA and rY are required for this case");
    // N > 0 without preAt: CP hands PFDR the whole Y and rA (ref :847-859), no rY
    try {
        hipStream_t s = lib_stream();
        const bool dev = mem == PFDR_MEM_DEVICE;
        const auto kin = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
        auto in = [&](DevBuf<real> &b, const real *h, size_t n) -> const real * {
            if (dev || !h) return h;
            b.alloc(n);
            PFDR_HIP(hipMemcpyAsync(b.p, h, n * sizeof(real), kin, s));
            return b.p;
        };
        DevBuf<real> bA, bY, brA, brAA, brY, bL, bl;
        DevBuf<int> bptr, bVc;
        const size_t asz = N > 0 ? (size_t)N * V : N < 0 ? (size_t)V * V : (size_t)V;
        const real *dA = in(bA, A, asz);
        const real *dY = in(bY, Y, N > 0 ? (size_t)N : (size_t)V);
        const int *dptr = rVc, *dVc = Vc;
        if (!dev) {
            bptr.alloc(rV + 1);
            bVc.alloc(V);
            PFDR_HIP(hipMemcpyAsync(bptr.p, rVc, (rV + 1) * 4, hipMemcpyHostToDevice, s));
            PFDR_HIP(hipMemcpyAsync(bVc.p, Vc, (size_t)V * 4, hipMemcpyHostToDevice, s));
            dptr = bptr.p;
            dVc = bVc.p;
        }
        auto out = [&](DevBuf<real> &b, real *h, size_t n) -> real * {
            if (dev && h) return h;
            b.alloc(n ? n : 1);
            return b.p;
        };
        const size_t rAAn = N == 0 ? (size_t)rV : (size_t)rV * rV;
        real *drA = N > 0 ? out(brA, rA, (size_t)N * rV) : nullptr;
        real *drAA = preAt ? out(brAA, rAA, rAAn) : nullptr;
        real *drY = preAt ? out(brY, rY, rV) : nullptr;
        bl.alloc(rV);
        real *dl = bl.p;
        const int gy = rV < 65535 ? rV : 65535;  // rows per launch; kernels loop over the rest
        const dim3 b1(kBlock), gV(grid_for(rV));
        const dim3 gVV(grid_for(rV), gy);
        if (N > 0) {
            k_cp_colsum<real><<<dim3(grid_for(N), gy), b1, 0, s>>>(N, rV, dA, dptr, dVc, drA);
            if (preAt) {
                const double work = (double)rV * rV * N / 2;
                if (work <= 17179869184.0) {
                    k_cp_gram_seq<real><<<gVV, b1, 0, s>>>(N, rV, drA, drAA);
                    k_cp_mirror<real><<<gVV, b1, 0, s>>>(rV, drAA);
                } else {
                    gram<real>(0, rV, N, drA, N, drAA, s);  // matrix cores, mirrored
                }
                k_cp_rY_dot<real><<<gV, b1, 0, s>>>(N, rV, drA, dY, drY);
            }
        } else {
            // rY = component sums of Y (:715-723); N = 0: rAA = component sums
            // of the diagonal (:744-755) or the sizes (:756-758) — each sum in
            // Vc order, giant components by one LDS-staged workgroup
            ordered_segment_sums<real>(rV, dptr, dVc, dY, drY, s);
            if (N == 0 && dA) ordered_segment_sums<real>(rV, dptr, dVc, dA, drAA, s);
            else if (N == 0) k_cp_sizes<real><<<gV, b1, 0, s>>>(rV, dptr, drAA);
            if (N < 0) {
                k_cp_ata<real><<<gVV, b1, 0, s>>>(V, rV, dA, dptr, dVc, drAA);
                k_cp_mirror<real><<<gVV, b1, 0, s>>>(rV, drAA);
            }
        }
        PFDR_HIP(hipGetLastError());
        if (N != 0) {
            real c;
            if (preAt) {  // equilibrate rAA, norm, revert (:776-800)
                k_cp_diag_sqrt<real><<<gV, b1, 0, s>>>(rV, drAA, dl);
                k_cp_scale_sym<real><<<gVV, b1, 0, s>>>(rV, drAA, dl, 0);
                c = operator_norm_device<real>(0, rV, drAA, normTol, normItMax, normNbInit, 0, s,
                                               nullptr);
                k_cp_scale_sym<real><<<gVV, b1, 0, s>>>(rV, drAA, dl, 1);
            } else {  // equilibrate rA (:801-825)
                k_cp_colnorm<real><<<gV, b1, 0, s>>>(N, rV, drA, dl);
                k_cp_scale_cols<real><<<dim3(grid_for(N), gy), b1, 0, s>>>(N, rV, drA, dl, 0);
                c = operator_norm_device<real>(N, rV, drA, normTol, normItMax, normNbInit, 0, s,
                                               nullptr);
                k_cp_scale_cols<real><<<dim3(grid_for(N), gy), b1, 0, s>>>(N, rV, drA, dl, 1);
            }
            if (L) {
                real *dL = out(bL, L, rV);
                k_cp_lipschitz<real><<<gV, b1, 0, s>>>(rV, dl, c, dL);
                if (!dev) PFDR_HIP(hipMemcpyAsync(L, dL, rV * sizeof(real), hipMemcpyDeviceToHost, s));
            }
            if (Leq) PFDR_HIP(hipMemcpyAsync(Leq, dl, rV * sizeof(real),
                                             dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
        } else if (L) {
            PFDR_HIP(hipMemcpyAsync(L, drAA, rV * sizeof(real),
                                    dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
        }
        PFDR_HIP(hipGetLastError());
        if (!dev) {
            if (drA) PFDR_HIP(hipMemcpyAsync(rA, drA, (size_t)N * rV * sizeof(real), hipMemcpyDeviceToHost, s));
            if (drAA) PFDR_HIP(hipMemcpyAsync(rAA, drAA, rAAn * sizeof(real), hipMemcpyDeviceToHost, s));
            if (drY) PFDR_HIP(hipMemcpyAsync(rY, drY, rV * sizeof(real), hipMemcpyDeviceToHost, s));
        }
        PFDR_HIP(hipStreamSynchronize(s));
    } catch (const HipError &h) {
        return report_error(fn, h);
    } catch (const std::exception &ex) {
        return report_error(fn, ex.what());
    }
    return PFDR_OK;
}

}  // namespace pfdr

extern "C" int pfdr_cp_reduce_f32(int N, int V, const float *A, const float *Y, int rV,
                                  const int *rVc, const int *Vc, int preAt, int mem,
                                  float normTol, int normItMax, int normNbInit, float *rA,
                                  float *rAA, float *rY, float *L, float *Leq) {
    return pfdr::cp_reduce_host<float>("pfdr_cp_reduce_f32", N, V, A, Y, rV, rVc, Vc, preAt, mem,
                                       normTol, normItMax, normNbInit, rA, rAA, rY, L, Leq);
}
extern "C" int pfdr_cp_reduce_f64(int N, int V, const double *A, const double *Y, int rV,
                                  const int *rVc, const int *Vc, int preAt, int mem,
                                  double normTol, int normItMax, int normNbInit, double *rA,
                                  double *rAA, double *rY, double *L, double *Leq) {
    return pfdr::cp_reduce_host<double>("pfdr_cp_reduce_f64", N, V, A, Y, rV, rVc, Vc, preAt,
                                        mem, normTol, normItMax, normNbInit, rA, rAA, rY, L, Leq);
}
