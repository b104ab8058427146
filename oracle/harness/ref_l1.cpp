/* TEST INFRASTRUCTURE ONLY. C-callable shim over the REFERENCE's own
 * PFDR_graph_quadratic_d1_l1<real> (include/PFDR_graph_quadratic_d1_l1.hpp:36-42),
 * compiled together with /root/reference/src/PFDR_graph_quadratic_d1_l1.cpp
 * into oracle/_ref/ by oracle/Makefile.  Nothing here is product code. */
#include "PFDR_graph_quadratic_d1_l1.hpp"

#define REF_L1(T, SFX) \
extern "C" void ref_pfdr_quadratic_d1_l1_##SFX(int V, int E, int N, T *X, \
    const T *Y, const T *A, const int *Eu, const int *Ev, const T *La_d1, \
    const T *La_l1, int positivity, int Ltype, const T *L, T rho, \
    T condMin, T difRcd, T difTol, int itMax, int *it, T *Obj, T *Dif) \
{ \
    PFDR_graph_quadratic_d1_l1<T>(V, E, N, X, Y, A, Eu, Ev, La_d1, La_l1, \
        positivity, Ltype ? DIAG : SCAL, L, rho, condMin, difRcd, difTol, \
        itMax, it, Obj, Dif, 0); \
}
REF_L1(float, f32)
REF_L1(double, f64)
