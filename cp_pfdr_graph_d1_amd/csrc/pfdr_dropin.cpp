// The reference's C++ entry points, defined on top of the C ABI so that the
// cut-pursuit drivers (reference src/CP_PFDR_graph_*.cpp) and the MEX
// wrappers link against libpfdr_mi355x.so unchanged.  Explicit
// instantiations for float and double, emitted weak exactly like the
// reference's (src/PFDR_graph_quadratic_d1_l1.cpp:555-566,
// src/PFDR_graph_quadratic_d1_bounds.cpp:532-543,
// src/PFDR_graph_loss_d1_simplex.cpp:717-726,
// src/proj_simplex_metric.cpp:85-89, src/operator_norm_matrix.cpp:215-219):
// same mangled names.
#include <cstdio>
#include <cstdlib>

#include "../../include/PFDR_graph_loss_d1_simplex.hpp"
#include "../../include/PFDR_graph_quadratic_d1_bounds.hpp"
#include "../../include/PFDR_graph_quadratic_d1_l1.hpp"
#include "../../include/pfdr_mi355x.h"
#include "../../include/operator_norm_matrix.hpp"
#include "../../include/proj_simplex.hpp"

namespace {

// the reference returns void and has no error channel: fail loudly
void check(int status) {
    if (status != PFDR_OK) {
        fprintf(stderr, "libpfdr_mi355x: %s\n", pfdr_last_error());
        fflush(stderr);
        abort();
    }
}

int q_l1(int V, int E, int N, float *X, const float *Y, const float *A, const int *Eu,
         const int *Ev, const float *Ld, const float *Ll, int pos, int Lt, const float *L,
         float rho, float cm, float rcd, float tol, int itMax, int *it, float *Obj,
         float *Dif, int vb) {
    return pfdr_quadratic_d1_l1_f32(V, E, N, X, Y, A, Eu, Ev, Ld, Ll, pos, Lt, L, rho, cm, rcd,
                                    tol, itMax, it, Obj, Dif, vb);
}
int q_l1(int V, int E, int N, double *X, const double *Y, const double *A, const int *Eu,
         const int *Ev, const double *Ld, const double *Ll, int pos, int Lt, const double *L,
         double rho, double cm, double rcd, double tol, int itMax, int *it, double *Obj,
         double *Dif, int vb) {
    return pfdr_quadratic_d1_l1_f64(V, E, N, X, Y, A, Eu, Ev, Ld, Ll, pos, Lt, L, rho, cm, rcd,
                                    tol, itMax, it, Obj, Dif, vb);
}
int q_bd(int V, int E, int N, float *X, const float *Y, const float *A, const int *Eu,
         const int *Ev, const float *Ld, float mn, float mx, int Lt, const float *L, float rho,
         float cm, float rcd, float tol, int itMax, int *it, float *Obj, float *Dif, int vb) {
    return pfdr_quadratic_d1_bounds_f32(V, E, N, X, Y, A, Eu, Ev, Ld, mn, mx, Lt, L, rho, cm,
                                        rcd, tol, itMax, it, Obj, Dif, vb);
}
int q_bd(int V, int E, int N, double *X, const double *Y, const double *A, const int *Eu,
         const int *Ev, const double *Ld, double mn, double mx, int Lt, const double *L,
         double rho, double cm, double rcd, double tol, int itMax, int *it, double *Obj,
         double *Dif, int vb) {
    return pfdr_quadratic_d1_bounds_f64(V, E, N, X, Y, A, Eu, Ev, Ld, mn, mx, Lt, L, rho, cm,
                                        rcd, tol, itMax, it, Obj, Dif, vb);
}
int sx(int K, int V, int E, float al, const float *Lf, float *P, const float *Q, const int *Eu,
       const int *Ev, const float *Ld, float rho, float cm, float rcd, float tol, int itMax,
       int *it, float *Obj, float *Dif, int vb) {
    return pfdr_loss_d1_simplex_f32(K, V, E, al, Lf, P, Q, Eu, Ev, Ld, rho, cm, rcd, tol, itMax,
                                    it, Obj, Dif, vb);
}
int sx(int K, int V, int E, double al, const double *Lf, double *P, const double *Q,
       const int *Eu, const int *Ev, const double *Ld, double rho, double cm, double rcd,
       double tol, int itMax, int *it, double *Obj, double *Dif, int vb) {
    return pfdr_loss_d1_simplex_f64(K, V, E, al, Lf, P, Q, Eu, Ev, Ld, rho, cm, rcd, tol, itMax,
                                    it, Obj, Dif, vb);
}
int pj(float *X, const float *M, int D, int N, int nm, const float *A, int na) {
    return pfdr_proj_simplex_metric_f32(X, M, D, N, nm, A, na);
}
int pj(double *X, const double *M, int D, int N, int nm, const double *A, int na) {
    return pfdr_proj_simplex_metric_f64(X, M, D, N, nm, A, na);
}

int on(int M, int N, const float *A, float tol, int itMax, int nb, int vb, float *out) {
    return pfdr_operator_norm_f32(M, N, A, PFDR_MEM_HOST, tol, itMax, nb, vb, out, nullptr);
}
int on(int M, int N, const double *A, double tol, int itMax, int nb, int vb, double *out) {
    return pfdr_operator_norm_f64(M, N, A, PFDR_MEM_HOST, tol, itMax, nb, vb, out, nullptr);
}

}  // namespace

template <typename real>
real operator_norm_matrix(int M, int N, const real *A, const real nTol, const int itMax,
                          int nbInit, const int verbose) {
    real out = real(0);
    check(on(M, N, A, nTol, itMax, nbInit, verbose, &out));
    return out;
}

template <typename real>
void PFDR_graph_quadratic_d1_l1(const int V, const int E, const int N, real *X, const real *Y,
                                const real *A, const int *Eu, const int *Ev, const real *La_d1,
                                const real *La_l1, const int positivity, const Lipschtype Ltype,
                                const real *L, const real rho, const real condMin, real difRcd,
                                const real difTol, const int itMax, int *it, real *Obj,
                                real *Dif, const int verbose) {
    check(q_l1(V, E, N, X, Y, A, Eu, Ev, La_d1, La_l1, positivity, Ltype == DIAG ? 1 : 0, L,
               rho, condMin, difRcd, difTol, itMax, it, Obj, Dif, verbose));
}

template <typename real>
void PFDR_graph_quadratic_d1_bounds(const int V, const int E, const int N, real *X, const real *Y,
                                    const real *A, const int *Eu, const int *Ev,
                                    const real *La_d1, const real min, const real max,
                                    const Lipschtype Ltype, const real *L, const real rho,
                                    const real condMin, real difRcd, const real difTol,
                                    const int itMax, int *it, real *Obj, real *Dif,
                                    const int verbose) {
    check(q_bd(V, E, N, X, Y, A, Eu, Ev, La_d1, min, max, Ltype == DIAG ? 1 : 0, L, rho, condMin,
               difRcd, difTol, itMax, it, Obj, Dif, verbose));
}

template <typename real>
void PFDR_graph_loss_d1_simplex(const int K, const int V, const int E, const real al,
                                const real *La_f, real *P, const real *Q, const int *Eu,
                                const int *Ev, const real *La_d1, const real rho,
                                const real condMin, real difRcd, const real difTol,
                                const int itMax, int *it, real *Obj, real *Dif,
                                const int verbose) {
    check(sx(K, V, E, al, La_f, P, Q, Eu, Ev, La_d1, rho, condMin, difRcd, difTol, itMax, it,
             Obj, Dif, verbose));
}

template <typename real>
void proj_simplex_metric(real *X, const real *M, const int D, const int N, const int nm,
                         const real *A, const int na) {
    check(pj(X, M, D, N, nm, A, na));
}

template void PFDR_graph_quadratic_d1_l1<float>(const int, const int, const int, float *,
    const float *, const float *, const int *, const int *, const float *, const float *,
    const int, const Lipschtype, const float *, const float, const float, float, const float,
    const int, int *, float *, float *, const int);
template void PFDR_graph_quadratic_d1_l1<double>(const int, const int, const int, double *,
    const double *, const double *, const int *, const int *, const double *, const double *,
    const int, const Lipschtype, const double *, const double, const double, double,
    const double, const int, int *, double *, double *, const int);
template void PFDR_graph_quadratic_d1_bounds<float>(const int, const int, const int, float *,
    const float *, const float *, const int *, const int *, const float *, const float,
    const float, const Lipschtype, const float *, const float, const float, float, const float,
    const int, int *, float *, float *, const int);
template void PFDR_graph_quadratic_d1_bounds<double>(const int, const int, const int, double *,
    const double *, const double *, const int *, const int *, const double *, const double,
    const double, const Lipschtype, const double *, const double, const double, double,
    const double, const int, int *, double *, double *, const int);
template void PFDR_graph_loss_d1_simplex<float>(const int, const int, const int, const float,
    const float *, float *, const float *, const int *, const int *, const float *, const float,
    const float, float, const float, const int, int *, float *, float *, const int);
template void PFDR_graph_loss_d1_simplex<double>(const int, const int, const int, const double,
    const double *, double *, const double *, const int *, const int *, const double *,
    const double, const double, double, const double, const int, int *, double *, double *,
    const int);
template void proj_simplex_metric<float>(float *, const float *, const int, const int,
    const int, const float *, const int);
template void proj_simplex_metric<double>(double *, const double *, const int, const int,
    const int, const double *, const int);
template float operator_norm_matrix<float>(int, int, const float *, const float, const int, int,
                                           const int);
template double operator_norm_matrix<double>(int, int, const double *, const double, const int,
                                             int, const int);
