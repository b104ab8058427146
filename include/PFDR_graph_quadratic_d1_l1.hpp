/* Drop-in declaration of the MI355X PFDR solver for
 *     F(x) = 1/2 ||y - A x||^2 + sum_{uv in E} la_uv |x_u - x_v|
 *            + sum_v la_v |x_v|   (+ positivity constraint)
 * Signature identical to the reference
 * (ai3DVision/CP_PFDR_graph_d1 include/PFDR_graph_quadratic_d1_l1.hpp:36-42),
 * argument meaning identical (see that header).  Definitions for
 * real = float and real = double live in libpfdr_mi355x.so
 * (cp_pfdr_graph_d1_amd/csrc/pfdr_dropin.cpp) and forward to the C ABI of
 * include/pfdr_mi355x.h.  Synchronous; host pointers; a device failure is
 * reported on stderr and aborts (the reference returns void). */
#ifndef PFDR_GRAPH_QUADRATIC_D1_L1_H
#define PFDR_GRAPH_QUADRATIC_D1_L1_H
#include "pfdr_lipschtype.hpp"

template <typename real>
void PFDR_graph_quadratic_d1_l1(const int V, const int E, const int N,
    real *X, const real *Y, const real *A, const int *Eu, const int *Ev,
    const real *La_d1, const real *La_l1, const int positivity,
    const Lipschtype Ltype, const real *L, const real rho, const real condMin,
    real difRcd, const real difTol, const int itMax, int *it,
    real *Obj, real *Dif, const int verbose);
#endif
