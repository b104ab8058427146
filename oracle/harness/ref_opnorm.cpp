/* TEST INFRASTRUCTURE ONLY. C-callable shim over the REFERENCE's own
 * operator_norm_matrix<real> (include/operator_norm_matrix.hpp:12-14),
 * compiled with /root/reference/src/operator_norm_matrix.cpp into
 * oracle/_ref/.  The reference seeds its starts with time(NULL), so its
 * value is an estimate within nTol of ||A||^2, not a fixed number. */
#include "operator_norm_matrix.hpp"

extern "C" float ref_operator_norm_f32(int M, int N, const float *A, float tol, int itMax,
                                       int nbInit) {
    return operator_norm_matrix<float>(M, N, A, tol, itMax, nbInit, 0);
}
extern "C" double ref_operator_norm_f64(int M, int N, const double *A, double tol, int itMax,
                                        int nbInit) {
    return operator_norm_matrix<double>(M, N, A, tol, itMax, nbInit, 0);
}
