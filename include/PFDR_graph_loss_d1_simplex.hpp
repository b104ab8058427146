/* Drop-in declaration of the MI355X PFDR solver for
 *     F(p) = f(p; q) + sum_{k, uv in E} la_uv |p_uk - p_vk| + i_simplex(p)
 * with f linear (al = 0), smoothed Kullback-Leibler (0 < al < 1) or
 * quadratic (al = 1).  Signature identical to the reference
 * (include/PFDR_graph_loss_d1_simplex.hpp:24-30).  Defined in
 * libpfdr_mi355x.so for float and double. */
#ifndef PFDR_GRAPH_LOSS_D1_SIMPLEX_H
#define PFDR_GRAPH_LOSS_D1_SIMPLEX_H

template <typename real>
void PFDR_graph_loss_d1_simplex(const int K, const int V, const int E,
    const real al, const real *La_f, real *P, const real *Q,
    const int *Eu, const int *Ev, const real *La_d1,
    const real rho, const real condMin,
    real difRcd, const real difTol, const int itMax, int *it,
    real *Obj, real *Dif, const int verbose);
#endif
