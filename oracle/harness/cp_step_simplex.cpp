/* TEST INFRASTRUCTURE ONLY.  C-callable driver of the REFERENCE's simplex
 * cut pursuit (CP_PFDR_graph_loss_d1_simplex<real>), compiled by
 * oracle/Makefile from /root/reference/src into
 * oracle/_ref/libcp_step_simplex_ref.so; used only by
 * tests/golden/make_cp_golden.py (--simplex) and the CPU tests.
 *
 * The twin of harness/cp_step_bounds.cpp for
 * src/CP_PFDR_graph_loss_d1_simplex.cpp: cp_refs_step runs ONE CP iteration
 * from a given state through the warm restart (CP_itMax = 1) and returns the
 * new state (activity after the merge, the last alpha-expansion's segments,
 * Cv, Vc, rVc, rP) and the reduced problem CP handed to PFDR (recorded by
 * the PFDR_graph_loss_d1_simplex defined here, which then runs the reference
 * PFDR compiled as ref_rec_pfdr_simplex): rEu, rEv, rLa_d1, rQ, rLa_f and
 * the barycentre warm start rP0.  cp_refs_init: the reference's own initial
 * state (CP_itMax = 0).  cp_refs_maxflow: the reference's BK maxflow with
 * the simplex driver's arc capacities (arc 2e from r_cap[e], arc 2e + 1
 * none, src/CP_PFDR_graph_loss_d1_simplex.cpp:563-595). */
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "graph.hpp"
#include "PFDR_graph_loss_d1_simplex.hpp"
#include "CP_PFDR_graph_loss_d1_simplex.hpp"

/* the warm-restart record as the reference defines it
 * (src/CP_PFDR_graph_loss_d1_simplex.cpp:150-155) */
template <typename real> struct CPls_Restart {
    Graph<real, real, real> *G;
    int *Vc;
    int *rVc;
};

template <typename real>
void ref_rec_pfdr_simplex(const int K, const int V, const int E, const real al, const real *La_f,
                          real *P, const real *Q, const int *Eu, const int *Ev, const real *La_d1,
                          const real rho, const real condMin, real difRcd, const real difTol,
                          const int itMax, int *it, real *Obj, real *Dif, const int verbose);

struct RecS {
    int called, rV, rE;
    int *rEu, *rEv;
    void *rLa_d1, *rQ, *rLa_f, *rP0;
};
static RecS *g_recs = nullptr;

template <typename real>
void PFDR_graph_loss_d1_simplex(const int K, const int V, const int E, const real al,
                                const real *La_f, real *P, const real *Q, const int *Eu,
                                const int *Ev, const real *La_d1, const real rho,
                                const real condMin, real difRcd, const real difTol,
                                const int itMax, int *it, real *Obj, real *Dif, const int verbose) {
    if (g_recs) {
        g_recs->called++;
        g_recs->rV = V;
        g_recs->rE = E;
        memcpy(g_recs->rEu, Eu, sizeof(int) * E);
        memcpy(g_recs->rEv, Ev, sizeof(int) * E);
        memcpy(g_recs->rLa_d1, La_d1, sizeof(real) * E);
        memcpy(g_recs->rQ, Q, sizeof(real) * (size_t)V * K);
        memcpy(g_recs->rP0, P, sizeof(real) * (size_t)V * K);
        if (La_f) memcpy(g_recs->rLa_f, La_f, sizeof(real) * V);
    }
    ref_rec_pfdr_simplex<real>(K, V, E, al, La_f, P, Q, Eu, Ev, La_d1, rho, condMin, difRcd,
                               difTol, itMax, it, Obj, Dif, verbose);
}
template void PFDR_graph_loss_d1_simplex<float>(const int, const int, const int, const float,
    const float *, float *, const float *, const int *, const int *, const float *, const float,
    const float, float, const float, const int, int *, float *, float *, const int);
template void PFDR_graph_loss_d1_simplex<double>(const int, const int, const int, const double,
    const double *, double *, const double *, const int *, const int *, const double *,
    const double, const double, double, const double, const int, int *, double *, double *,
    const int);

/* the graph as the reference's initialize() builds it (:86-93) */
template <typename real>
static Graph<real, real, real> *make_graph(int V, int E, const int *Eu, const int *Ev) {
    Graph<real, real, real> *G = new Graph<real, real, real>(V, E);
    G->add_node(V);
    for (int e = 0; e < E; e++) G->add_edge(Eu[e], Ev[e], (real)0, (real)0);
    for (int v = 0; v < V; v++) G->add_tweights(v, (real)0, (real)0);
    return G;
}

template <typename real>
static int init(int K, int V, int E, real al, const real *Q, const int *Eu, const int *Ev,
                const real *La_d1, real *rP0) {
    int rV = 0, CP_it = 0;
    int *Cv = (int *)malloc(sizeof(int) * V);
    real *rP = nullptr;
    CP_PFDR_graph_loss_d1_simplex<real>(K, V, E, al, &rV, Cv, &rP, Q, Eu, Ev, La_d1, (real)0, 0,
                                        &CP_it, (real)1.5, (real)1e-3, (real)0, (real)1e-3, 10,
                                        nullptr, nullptr, nullptr, 0, nullptr);
    memcpy(rP0, rP, sizeof(real) * K);
    free(rP);
    free(Cv);
    return rV;
}

template <typename real>
static int step(int K, int V, int E, real al, const real *Q, const int *Eu, const int *Ev,
                const real *La_d1, real CP_difTol, real rho, real condMin, real difRcd,
                real difTol, int itMax, uint8_t *active, int *Cv, int *Vc, int *rVc, int *rV,
                real *rP, uint8_t *segment, int *called, int *rE, int *rEu, int *rEv,
                real *rLa_d1, real *rQ, real *rLa_f, real *rP0) {
    CPls_Restart<real> rs;
    rs.G = make_graph<real>(V, E, Eu, Ev);
    for (int e = 0; e < E; e++) {
        rs.G->arcs[2 * e].is_active = active[e];
        rs.G->arcs[2 * e + 1].is_active = active[e];
    }
    rs.Vc = (int *)malloc(sizeof(int) * V);
    memcpy(rs.Vc, Vc, sizeof(int) * V);
    rs.rVc = (int *)malloc(sizeof(int) * (*rV + 1));
    memcpy(rs.rVc, rVc, sizeof(int) * (*rV + 1));
    real *x = (real *)malloc(sizeof(real) * (size_t)(*rV) * K);
    memcpy(x, rP, sizeof(real) * (size_t)(*rV) * K);
    RecS rec{0, 0, 0, rEu, rEv, rLa_d1, rQ, rLa_f, rP0};
    g_recs = &rec;
    int CP_it = 0;
    CP_PFDR_graph_loss_d1_simplex<real>(K, V, E, al, rV, Cv, &x, Q, Eu, Ev, La_d1, CP_difTol, 1,
                                        &CP_it, rho, condMin, difRcd, difTol, itMax, nullptr,
                                        nullptr, nullptr, 0, &rs);
    g_recs = nullptr;
    *called = rec.called;
    *rE = rec.rE;
    for (int e = 0; e < E; e++) active[e] = rs.G->arcs[2 * e].is_active;
    for (int v = 0; v < V; v++) segment[v] = (uint8_t)rs.G->what_segment(v);
    memcpy(Vc, rs.Vc, sizeof(int) * V);
    memcpy(rVc, rs.rVc, sizeof(int) * (*rV + 1));
    memcpy(rP, x, sizeof(real) * (size_t)(*rV) * K);
    free(x);
    delete rs.G;
    free(rs.Vc);
    free(rs.rVc);
    return CP_it;
}

/* a fresh graph of the same topology, the driver's capacities, BK maxflow */
template <typename real>
static void maxflow(int V, int E, const int *Eu, const int *Ev, const real *tr_cap,
                    const real *r_cap, uint8_t *segment) {
    Graph<real, real, real> *G = make_graph<real>(V, E, Eu, Ev);
    for (int v = 0; v < V; v++) G->nodes[v].tr_cap = tr_cap[v];
    for (int e = 0; e < E; e++) {
        G->arcs[2 * e].r_cap = r_cap[e];
        G->arcs[2 * e + 1].r_cap = (real)0;
    }
    G->maxflow();
    for (int v = 0; v < V; v++) segment[v] = (uint8_t)G->what_segment(v);
    delete G;
}

#define CP_STEPS_API(T, SFX)                                                                   \
    extern "C" int cp_refs_init_##SFX(int K, int V, int E, T al, const T *Q, const int *Eu,    \
                                      const int *Ev, const T *La_d1, T *rP0) {                 \
        return init<T>(K, V, E, al, Q, Eu, Ev, La_d1, rP0);                                    \
    }                                                                                          \
    extern "C" int cp_refs_step_##SFX(                                                         \
        int K, int V, int E, T al, const T *Q, const int *Eu, const int *Ev, const T *La_d1,   \
        T CP_difTol, T rho, T condMin, T difRcd, T difTol, int itMax, uint8_t *active,         \
        int *Cv, int *Vc, int *rVc, int *rV, T *rP, uint8_t *segment, int *called, int *rE,    \
        int *rEu, int *rEv, T *rLa_d1, T *rQ, T *rLa_f, T *rP0) {                              \
        return step<T>(K, V, E, al, Q, Eu, Ev, La_d1, CP_difTol, rho, condMin, difRcd, difTol, \
                       itMax, active, Cv, Vc, rVc, rV, rP, segment, called, rE, rEu, rEv,      \
                       rLa_d1, rQ, rLa_f, rP0);                                                \
    }                                                                                          \
    extern "C" void cp_refs_maxflow_##SFX(int V, int E, const int *Eu, const int *Ev,          \
                                          const T *tr_cap, const T *r_cap, uint8_t *segment) { \
        maxflow<T>(V, E, Eu, Ev, tr_cap, r_cap, segment);                                      \
    }
CP_STEPS_API(float, f32)
CP_STEPS_API(double, f64)
