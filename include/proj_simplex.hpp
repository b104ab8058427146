/* Drop-in declaration of the MI355X projection of each D-column of X onto
 * {x >= 0, sum x = a} in the metric diag(1/m).  Signature identical to the
 * reference (include/proj_simplex.hpp:33-35).  The reference also declares
 * an unweighted proj_simplex (:14-15) that it never defines; it is not
 * provided here either.  Defined in libpfdr_mi355x.so for float and double. */
#ifndef PROJ_SIMPLEX_H
#define PROJ_SIMPLEX_H

template <typename real>
void proj_simplex_metric(real *X, const real *M, const int D, const int N,
                         const int nm, const real *A, const int na);
#endif
