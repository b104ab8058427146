/* Drop-in declaration of the MI355X PFDR solver for
 *     F(x) = 1/2 ||y - A x||^2 + sum_{uv in E} la_uv |x_u - x_v|
 *            + i_{[min, max]}(x)
 * Signature identical to the reference
 * (include/PFDR_graph_quadratic_d1_bounds.hpp:34-40); min / max are
 * -HUGE_VAL / HUGE_VAL (or HUGE_VALF) for no bound.  Defined in
 * libpfdr_mi355x.so for float and double. */
#ifndef PFDR_GRAPH_QUADRATIC_D1_BOUNDS_H
#define PFDR_GRAPH_QUADRATIC_D1_BOUNDS_H
#include "pfdr_lipschtype.hpp"

template <typename real>
void PFDR_graph_quadratic_d1_bounds(const int V, const int E, const int N,
    real *X, const real *Y, const real *A, const int *Eu, const int *Ev,
    const real *La_d1, const real min, const real max,
    const Lipschtype Ltype, const real *L, const real rho, const real condMin,
    real difRcd, const real difTol, const int itMax, int *it,
    real *Obj, real *Dif, const int verbose);
#endif
