/* TEST INFRASTRUCTURE ONLY. C-callable shim over the REFERENCE's own
 * PFDR_graph_quadratic_d1_bounds<real> (include/PFDR_graph_quadratic_d1_bounds.hpp:34-40),
 * compiled with /root/reference/src/PFDR_graph_quadratic_d1_bounds.cpp into
 * oracle/_ref/ by oracle/Makefile.  Separate translation unit because the
 * reference headers both define Lipschtype. */
#include "PFDR_graph_quadratic_d1_bounds.hpp"

#define REF_BOUNDS(T, SFX) \
extern "C" void ref_pfdr_quadratic_d1_bounds_##SFX(int V, int E, int N, T *X, \
    const T *Y, const T *A, const int *Eu, const int *Ev, const T *La_d1, \
    T lo, T hi, int Ltype, const T *L, T rho, T condMin, T difRcd, \
    T difTol, int itMax, int *it, T *Obj, T *Dif) \
{ \
    PFDR_graph_quadratic_d1_bounds<T>(V, E, N, X, Y, A, Eu, Ev, La_d1, lo, \
        hi, Ltype ? DIAG : SCAL, L, rho, condMin, difRcd, difTol, itMax, it, \
        Obj, Dif, 0); \
}
REF_BOUNDS(float, f32)
REF_BOUNDS(double, f64)
