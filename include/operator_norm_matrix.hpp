/* libpfdr_mi355x: squared operator norm of a dense matrix by the power
 * method, same declaration as the reference's
 * include/operator_norm_matrix.hpp:12-14 (CP calls it on every reduced
 * problem with a dense A, src/CP_PFDR_graph_quadratic_d1_l1.cpp:792,822).
 * MI355X implementation: csrc/pfdr_gram.hip (matrix-core Gram, batched
 * power iterations); C ABI: pfdr_operator_norm_{f32,f64}.
 *   M, N   - A is M-by-N column major; M or N zero: A is the symmetric
 *            (A^tA or AA^t) matrix of the nonzero size
 *   nTol   - stopping criterion on the relative norm evolution
 *   itMax  - maximum iterations; nbInit - number of starting vectors
 * returns ||A||^2. */
#ifndef PFDR_MI355X_OPERATOR_NORM_MATRIX
#define PFDR_MI355X_OPERATOR_NORM_MATRIX

template <typename real>
real operator_norm_matrix(int M, int N, const real *A, const real nTol, const int itMax,
                          int nbInit, const int verbose);

#endif
