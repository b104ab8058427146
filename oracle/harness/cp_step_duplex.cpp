/* TEST INFRASTRUCTURE ONLY.  C-callable driver of the REFERENCE's duplex
 * cut pursuit (CP_PFDR_graph_quadratic_d1_l1_duplex<real>, N = 0, the
 * non-differentiable case: La_l1 or positivity), compiled by
 * oracle/Makefile from /root/reference/src into
 * oracle/_ref/libcp_step_duplex_ref.so; used only by
 * tests/golden/make_cp_golden.py (--duplex) and the CPU tests.
 *
 * The twin of harness/cp_step.cpp for src/CP_PFDR_graph_quadratic_d1_l1_duplex.cpp:
 * its graph has two layers, node v (v1) and node V + v (v2) per vertex
 * (:101-116: arcs 4e / 4e + 1 between u1 and v1, 4e + 2 / 4e + 3 between u2
 * and v2, 4E + 2v / 4E + 2v + 1 between v1 and v2); only the first layer's
 * arcs carry CP's activity.  cp_refd_step runs ONE CP iteration through the
 * warm restart (CP_itMax = 1) and returns the new state, the segments of
 * all 2V nodes after the iteration's single maxflow and the reduced problem
 * handed to PFDR.  cp_refd_init: the reference's initial state.
 * cp_refd_maxflow: the reference's BK maxflow on that graph with given
 * capacities (fresh graph, segments of the 2V nodes).
 *
 * The components' search (:585-591) skips heads w > V, so the arc from
 * vertex 0's first-layer node to node V (w == V) reads Cv[V], one past the
 * caller's array: Cv is given one guard entry here, never -1, so that arc is
 * skipped like every other vertical arc (the evident intent). */
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <ctime>

#include "graph.hpp"
#include "PFDR_graph_quadratic_d1_l1.hpp"
#include "CP_PFDR_graph_quadratic_d1_l1.hpp"

/* the warm-restart record as the duplex source defines it (:203-209) */
template <typename real> struct CPql1_Restart {
    Graph<real, real, real> *G;
    int *Vc;
    int *rVc;
    real *R;
};

template <typename real>
void ref_rec_pfdr_l1(const int V, const int E, const int N, real *X, const real *Y,
                     const real *A, const int *Eu, const int *Ev, const real *La_d1,
                     const real *La_l1, const int positivity, const Lipschtype Ltype,
                     const real *L, const real rho, const real condMin, real difRcd,
                     const real difTol, const int itMax, int *it, real *Obj, real *Dif,
                     const int verbose);

struct RecD {
    int called, rV, rE;
    int *rEu, *rEv;
    void *rLa_d1, *rLa_l1, *rY, *rAA;
};
static RecD *g_recd = nullptr;

extern "C" time_t time(time_t *t) {
    if (t) *t = (time_t)1;
    return (time_t)1;
}

template <typename real>
void PFDR_graph_quadratic_d1_l1(const int V, const int E, const int N, real *X, const real *Y,
                                const real *A, const int *Eu, const int *Ev, const real *La_d1,
                                const real *La_l1, const int positivity, const Lipschtype Ltype,
                                const real *L, const real rho, const real condMin, real difRcd,
                                const real difTol, const int itMax, int *it, real *Obj,
                                real *Dif, const int verbose) {
    if (g_recd) {
        g_recd->called++;
        g_recd->rV = V;
        g_recd->rE = E;
        memcpy(g_recd->rEu, Eu, sizeof(int) * E);
        memcpy(g_recd->rEv, Ev, sizeof(int) * E);
        memcpy(g_recd->rLa_d1, La_d1, sizeof(real) * E);
        if (La_l1) memcpy(g_recd->rLa_l1, La_l1, sizeof(real) * V);
        memcpy(g_recd->rY, Y, sizeof(real) * V);
        if (A) memcpy(g_recd->rAA, A, sizeof(real) * V);
    }
    ref_rec_pfdr_l1<real>(V, E, N, X, Y, A, Eu, Ev, La_d1, La_l1, positivity, Ltype, L, rho,
                          condMin, difRcd, difTol, itMax, it, Obj, Dif, verbose);
}
template void PFDR_graph_quadratic_d1_l1<float>(const int, const int, const int, float *,
    const float *, const float *, const int *, const int *, const float *, const float *,
    const int, const Lipschtype, const float *, const float, const float, float, const float,
    const int, int *, float *, float *, const int);
template void PFDR_graph_quadratic_d1_l1<double>(const int, const int, const int, double *,
    const double *, const double *, const int *, const int *, const double *, const double *,
    const int, const Lipschtype, const double *, const double, const double, double,
    const double, const int, int *, double *, double *, const int);

/* the two-layer graph exactly as the duplex initialize() builds it (:101-116) */
template <typename real>
static Graph<real, real, real> *make_graph2(int V, int E, const int *Eu, const int *Ev) {
    Graph<real, real, real> *G = new Graph<real, real, real>(2 * V, 2 * E + V);
    G->add_node(2 * V);
    for (int e = 0; e < E; e++) {
        G->add_edge(Eu[e], Ev[e], (real)0, (real)0);
        G->add_edge(Eu[e] + V, Ev[e] + V, (real)0, (real)0);
    }
    for (int v = 0; v < V; v++) {
        G->add_tweights(v, (real)0, (real)0);
        G->add_tweights(v + V, (real)0, (real)0);
        G->add_edge(v, v + V, (real)0, (real)0);
    }
    return G;
}

template <typename real>
static int init(int V, int E, const real *Y, const real *A, const int *Eu, const int *Ev,
                const real *La_d1, const real *La_l1, int positivity, real *rX0) {
    int rV = 0, CP_it = 0;
    int *Cv = (int *)malloc(sizeof(int) * (V + 1));
    Cv[V] = 0;
    real *rX = nullptr;
    CP_PFDR_graph_quadratic_d1_l1_duplex<real>(V, E, 0, &rV, Cv, &rX, Y, A, Eu, Ev, La_d1, La_l1,
                                               positivity, (real)0, 0, &CP_it, (real)1.5,
                                               (real)1e-3, (real)0, (real)1e-4, 10, nullptr,
                                               nullptr, nullptr, 0, nullptr);
    rX0[0] = rX[0];
    free(rX);
    free(Cv);
    return rV;
}

template <typename real>
static int step(int V, int E, const real *Y, const real *A, const int *Eu, const int *Ev,
                const real *La_d1, const real *La_l1, int positivity, real CP_difTol, real rho,
                real condMin, real difRcd, real difTol, int itMax, uint8_t *active, int *Cv_io,
                int *Vc, int *rVc, int *rV, real *rX, uint8_t *segment, int *called, int *rE,
                int *rEu, int *rEv, real *rLa_d1, real *rLa_l1, real *rY, real *rAA) {
    CPql1_Restart<real> rs;
    rs.G = make_graph2<real>(V, E, Eu, Ev);
    for (int e = 0; e < E; e++) {
        rs.G->arcs[4 * e].is_active = active[e];
        rs.G->arcs[4 * e + 1].is_active = active[e];
    }
    rs.Vc = (int *)malloc(sizeof(int) * V);
    memcpy(rs.Vc, Vc, sizeof(int) * V);
    rs.rVc = (int *)malloc(sizeof(int) * (*rV + 1));
    memcpy(rs.rVc, rVc, sizeof(int) * (*rV + 1));
    rs.R = nullptr;
    int *Cv = (int *)malloc(sizeof(int) * (V + 1));  // guard entry Cv[V], see above
    memcpy(Cv, Cv_io, sizeof(int) * V);
    Cv[V] = 0;
    real *x = (real *)malloc(sizeof(real) * (*rV));
    memcpy(x, rX, sizeof(real) * (*rV));
    RecD rec{0, 0, 0, rEu, rEv, rLa_d1, rLa_l1, rY, rAA};
    g_recd = &rec;
    int CP_it = 0;
    CP_PFDR_graph_quadratic_d1_l1_duplex<real>(V, E, 0, rV, Cv, &x, Y, A, Eu, Ev, La_d1, La_l1,
                                               positivity, CP_difTol, 1, &CP_it, rho, condMin,
                                               difRcd, difTol, itMax, nullptr, nullptr, nullptr,
                                               0, &rs);
    g_recd = nullptr;
    *called = rec.called;
    *rE = rec.rE;
    for (int e = 0; e < E; e++) active[e] = rs.G->arcs[4 * e].is_active;
    for (int v = 0; v < 2 * V; v++) segment[v] = (uint8_t)rs.G->what_segment(v);
    memcpy(Cv_io, Cv, sizeof(int) * V);
    memcpy(Vc, rs.Vc, sizeof(int) * V);
    memcpy(rVc, rs.rVc, sizeof(int) * (*rV + 1));
    memcpy(rX, x, sizeof(real) * (*rV));
    free(x);
    free(Cv);
    delete rs.G;
    free(rs.Vc);
    free(rs.rVc);
    return CP_it;
}

/* the two-layer graph, the cut's capacities (:504-527), BK maxflow */
template <typename real>
static void maxflow(int V, int E, const int *Eu, const int *Ev, const real *tr_cap,
                    const real *r_link, const real *r_cap, uint8_t *segment) {
    Graph<real, real, real> *G = make_graph2<real>(V, E, Eu, Ev);
    for (int v = 0; v < V; v++) {
        G->nodes[v].tr_cap = tr_cap[v];
        G->nodes[v + V].tr_cap = tr_cap[V + v];
        G->arcs[4 * E + 2 * v].r_cap = r_link[v];
        G->arcs[4 * E + 2 * v + 1].r_cap = (real)0;
    }
    for (int e = 0; e < E; e++)
        for (int k = 0; k < 4; k++) G->arcs[4 * e + k].r_cap = r_cap[e];
    G->maxflow();
    for (int v = 0; v < 2 * V; v++) segment[v] = (uint8_t)G->what_segment(v);
    delete G;
}

#define CP_STEPD_API(T, SFX)                                                                   \
    extern "C" int cp_refd_init_##SFX(int V, int E, const T *Y, const T *A, const int *Eu,     \
                                      const int *Ev, const T *La_d1, const T *La_l1,           \
                                      int positivity, T *rX0) {                                \
        return init<T>(V, E, Y, A, Eu, Ev, La_d1, La_l1, positivity, rX0);                     \
    }                                                                                          \
    extern "C" int cp_refd_step_##SFX(                                                         \
        int V, int E, const T *Y, const T *A, const int *Eu, const int *Ev, const T *La_d1,    \
        const T *La_l1, int positivity, T CP_difTol, T rho, T condMin, T difRcd, T difTol,     \
        int itMax, uint8_t *active, int *Cv, int *Vc, int *rVc, int *rV, T *rX,                \
        uint8_t *segment, int *called, int *rE, int *rEu, int *rEv, T *rLa_d1, T *rLa_l1,      \
        T *rY, T *rAA) {                                                                       \
        return step<T>(V, E, Y, A, Eu, Ev, La_d1, La_l1, positivity, CP_difTol, rho, condMin,  \
                       difRcd, difTol, itMax, active, Cv, Vc, rVc, rV, rX, segment, called,    \
                       rE, rEu, rEv, rLa_d1, rLa_l1, rY, rAA);                                 \
    }                                                                                          \
    extern "C" void cp_refd_maxflow_##SFX(int V, int E, const int *Eu, const int *Ev,          \
                                          const T *tr_cap, const T *r_link, const T *r_cap,    \
                                          uint8_t *segment) {                                  \
        maxflow<T>(V, E, Eu, Ev, tr_cap, r_link, r_cap, segment);                              \
    }
CP_STEPD_API(float, f32)
CP_STEPD_API(double, f64)
