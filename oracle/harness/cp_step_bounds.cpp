/* TEST INFRASTRUCTURE ONLY.  C-callable driver of the REFERENCE's bounds
 * cut pursuit (CP_PFDR_graph_quadratic_d1_bounds<real>, N = 0: identity or
 * diagonal A), compiled by oracle/Makefile from /root/reference/src into
 * oracle/_ref/libcp_step_bounds_ref.so; used only by
 * tests/golden/make_cp_golden.py (bounds cases) and the CPU tests.
 *
 * The twin of harness/cp_step.cpp for src/CP_PFDR_graph_quadratic_d1_bounds.cpp:
 * cp_refb_step runs ONE CP iteration from a given state through the warm
 * restart (CP_itMax = 1) and returns the new state (activity after the
 * merge, last cut's segments, Cv, Vc, rVc, rX) and the reduced problem CP
 * handed to PFDR (recorded by the PFDR_graph_quadratic_d1_bounds defined
 * here, which then runs the reference PFDR compiled as ref_rec_pfdr_bounds).
 * cp_refb_init: the reference's own initial state (CP_itMax = 0). */
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "graph.hpp"
#include "PFDR_graph_quadratic_d1_bounds.hpp"
#include "CP_PFDR_graph_quadratic_d1_bounds.hpp"

/* the warm-restart record as the reference defines it
 * (include/CP_PFDR_graph_quadratic_d1_bounds.hpp:38-46) */
template <typename real> struct CPqb_Restart {
    Graph<real, real, real> *G;
    int *Vc;
    int *rVc;
    real *R;
};

template <typename real>
void ref_rec_pfdr_bounds(const int V, const int E, const int N, real *X, const real *Y,
                         const real *A, const int *Eu, const int *Ev, const real *La_d1,
                         const real min, const real max, const Lipschtype Ltype, const real *L,
                         const real rho, const real condMin, real difRcd, const real difTol,
                         const int itMax, int *it, real *Obj, real *Dif, const int verbose);

struct RecB {
    int called, rV, rE;
    int *rEu, *rEv;
    void *rLa_d1, *rY, *rAA;
};
static RecB *g_recb = nullptr;

template <typename real>
void PFDR_graph_quadratic_d1_bounds(const int V, const int E, const int N, real *X,
                                    const real *Y, const real *A, const int *Eu, const int *Ev,
                                    const real *La_d1, const real min, const real max,
                                    const Lipschtype Ltype, const real *L, const real rho,
                                    const real condMin, real difRcd, const real difTol,
                                    const int itMax, int *it, real *Obj, real *Dif,
                                    const int verbose) {
    if (g_recb) {
        g_recb->called++;
        g_recb->rV = V;
        g_recb->rE = E;
        memcpy(g_recb->rEu, Eu, sizeof(int) * E);
        memcpy(g_recb->rEv, Ev, sizeof(int) * E);
        memcpy(g_recb->rLa_d1, La_d1, sizeof(real) * E);
        memcpy(g_recb->rY, Y, sizeof(real) * V);
        if (A) memcpy(g_recb->rAA, A, sizeof(real) * V);
    }
    ref_rec_pfdr_bounds<real>(V, E, N, X, Y, A, Eu, Ev, La_d1, min, max, Ltype, L, rho, condMin,
                              difRcd, difTol, itMax, it, Obj, Dif, verbose);
}
template void PFDR_graph_quadratic_d1_bounds<float>(const int, const int, const int, float *,
    const float *, const float *, const int *, const int *, const float *, const float,
    const float, const Lipschtype, const float *, const float, const float, float, const float,
    const int, int *, float *, float *, const int);
template void PFDR_graph_quadratic_d1_bounds<double>(const int, const int, const int, double *,
    const double *, const double *, const int *, const int *, const double *, const double,
    const double, const Lipschtype, const double *, const double, const double, double,
    const double, const int, int *, double *, double *, const int);

/* the graph as the reference's initialize() builds it */
template <typename real>
static Graph<real, real, real> *make_graph(int V, int E, const int *Eu, const int *Ev) {
    Graph<real, real, real> *G = new Graph<real, real, real>(V, E);
    G->add_node(V);
    for (int e = 0; e < E; e++) G->add_edge(Eu[e], Ev[e], (real)0, (real)0);
    for (int v = 0; v < V; v++) G->add_tweights(v, (real)0, (real)0);
    return G;
}

template <typename real>
static int init(int V, int E, const real *Y, const real *A, const int *Eu, const int *Ev,
                const real *La_d1, real mn, real mx, real *rX0) {
    int rV = 0, CP_it = 0;
    int *Cv = (int *)malloc(sizeof(int) * V);
    real *rX = nullptr;
    CP_PFDR_graph_quadratic_d1_bounds<real>(V, E, 0, &rV, Cv, &rX, Y, A, Eu, Ev, La_d1, mn, mx,
                                            (real)0, 0, &CP_it, (real)1.5, (real)1e-3, (real)0,
                                            (real)1e-4, 10, nullptr, nullptr, nullptr, 0,
                                            nullptr);
    rX0[0] = rX[0];
    free(rX);
    free(Cv);
    return rV;
}

template <typename real>
static int step(int V, int E, const real *Y, const real *A, const int *Eu, const int *Ev,
                const real *La_d1, real mn, real mx, real CP_difTol, real rho, real condMin,
                real difRcd, real difTol, int itMax, uint8_t *active, int *Cv, int *Vc,
                int *rVc, int *rV, real *rX, uint8_t *segment, int *called, int *rE, int *rEu,
                int *rEv, real *rLa_d1, real *rY, real *rAA) {
    CPqb_Restart<real> rs;
    rs.G = make_graph<real>(V, E, Eu, Ev);
    for (int e = 0; e < E; e++) {
        rs.G->arcs[2 * e].is_active = active[e];
        rs.G->arcs[2 * e + 1].is_active = active[e];
    }
    rs.Vc = (int *)malloc(sizeof(int) * V);
    memcpy(rs.Vc, Vc, sizeof(int) * V);
    rs.rVc = (int *)malloc(sizeof(int) * (*rV + 1));
    memcpy(rs.rVc, rVc, sizeof(int) * (*rV + 1));
    rs.R = nullptr;
    real *x = (real *)malloc(sizeof(real) * (*rV));
    memcpy(x, rX, sizeof(real) * (*rV));
    RecB rec{0, 0, 0, rEu, rEv, rLa_d1, rY, rAA};
    g_recb = &rec;
    int CP_it = 0;
    CP_PFDR_graph_quadratic_d1_bounds<real>(V, E, 0, rV, Cv, &x, Y, A, Eu, Ev, La_d1, mn, mx,
                                            CP_difTol, 1, &CP_it, rho, condMin, difRcd, difTol,
                                            itMax, nullptr, nullptr, nullptr, 0, &rs);
    g_recb = nullptr;
    *called = rec.called;
    *rE = rec.rE;
    for (int e = 0; e < E; e++) active[e] = rs.G->arcs[2 * e].is_active;
    for (int v = 0; v < V; v++) segment[v] = (uint8_t)rs.G->what_segment(v);
    memcpy(Vc, rs.Vc, sizeof(int) * V);
    memcpy(rVc, rs.rVc, sizeof(int) * (*rV + 1));
    memcpy(rX, x, sizeof(real) * (*rV));
    free(x);
    delete rs.G;
    free(rs.Vc);
    free(rs.rVc);
    return CP_it;
}

#define CP_STEPB_API(T, SFX)                                                                  \
    extern "C" int cp_refb_init_##SFX(int V, int E, const T *Y, const T *A, const int *Eu,    \
                                      const int *Ev, const T *La_d1, T mn, T mx, T *rX0) {    \
        return init<T>(V, E, Y, A, Eu, Ev, La_d1, mn, mx, rX0);                               \
    }                                                                                         \
    extern "C" int cp_refb_step_##SFX(                                                        \
        int V, int E, const T *Y, const T *A, const int *Eu, const int *Ev, const T *La_d1,   \
        T mn, T mx, T CP_difTol, T rho, T condMin, T difRcd, T difTol, int itMax,             \
        uint8_t *active, int *Cv, int *Vc, int *rVc, int *rV, T *rX, uint8_t *segment,        \
        int *called, int *rE, int *rEu, int *rEv, T *rLa_d1, T *rY, T *rAA) {                 \
        return step<T>(V, E, Y, A, Eu, Ev, La_d1, mn, mx, CP_difTol, rho, condMin, difRcd,    \
                       difTol, itMax, active, Cv, Vc, rVc, rV, rX, segment, called, rE, rEu,  \
                       rEv, rLa_d1, rY, rAA);                                                 \
    }
CP_STEPB_API(float, f32)
CP_STEPB_API(double, f64)
