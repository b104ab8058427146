/* TEST INFRASTRUCTURE ONLY. C-callable shim over the REFERENCE's own
 * PFDR_graph_loss_d1_simplex<real> (include/PFDR_graph_loss_d1_simplex.hpp:24-30)
 * and proj_simplex_metric<real> (include/proj_simplex.hpp:33-35), compiled
 * with the matching /root/reference/src files into oracle/_ref/. */
#include "proj_simplex.hpp"
#include "PFDR_graph_loss_d1_simplex.hpp"

#define REF_SIMPLEX(T, SFX) \
extern "C" void ref_pfdr_loss_d1_simplex_##SFX(int K, int V, int E, T al, \
    const T *La_f, T *P, const T *Q, const int *Eu, const int *Ev, \
    const T *La_d1, T rho, T condMin, T difRcd, T difTol, int itMax, \
    int *it, T *Obj, T *Dif) \
{ \
    PFDR_graph_loss_d1_simplex<T>(K, V, E, al, La_f, P, Q, Eu, Ev, La_d1, \
        rho, condMin, difRcd, difTol, itMax, it, Obj, Dif, 0); \
} \
extern "C" void ref_proj_simplex_metric_##SFX(T *X, const T *M, int D, \
    int N, int nm, const T *A, int na) \
{ \
    proj_simplex_metric<T>(X, M, D, N, nm, A, na); \
}
REF_SIMPLEX(float, f32)
REF_SIMPLEX(double, f64)
