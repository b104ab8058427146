/* TEST INFRASTRUCTURE ONLY.  C-callable driver of the REFERENCE's cut-pursuit
 * iteration (CP_PFDR_graph_quadratic_d1_l1<real>, N = 0: identity or
 * diagonal A), compiled by oracle/Makefile from /root/reference/src into
 * oracle/_ref/libcp_step_ref.so, used only by tests/golden/make_cp_golden.py
 * and the CPU tests that pin oracle/cp_graph_body.h.
 *
 * cp_ref_step runs exactly ONE CP iteration of the reference from a given
 * state through its warm-restart path (CP_itMax = 1, CP_restart != NULL,
 * src/CP_PFDR_graph_quadratic_d1_l1.cpp:260-270) and returns the new state:
 * activity of every edge (after the merge), the segment of every vertex in
 * the LAST maxflow, components (Cv, Vc, rVc), component values rX, and the
 * reduced problem CP handed to PFDR (recorded by the PFDR_graph_quadratic_d1_l1
 * defined here, which then runs the reference PFDR: its object is compiled
 * with -DPFDR_graph_quadratic_d1_l1=ref_rec_pfdr_l1).
 * cp_ref_init: the reference's own initial state (CP_itMax = 0).
 * cp_ref_maxflow: the reference's Boykov-Kolmogorov maxflow on given
 * capacities (fresh graph of the same topology), segment of every vertex. */
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <ctime>

#include "graph.hpp"
#include "PFDR_graph_quadratic_d1_l1.hpp"
#include "CP_PFDR_graph_quadratic_d1_l1.hpp"

/* the warm-restart record as the reference defines it (its layout is part
 * of the restart interface, include/CP_PFDR_graph_quadratic_d1_l1.hpp:35-42) */
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

struct Rec {
    int called, rV, rE;
    int *rEu, *rEv;
    void *rLa_d1, *rLa_l1, *rY, *rAA;
    /* dense modes (N != 0): the N handed to PFDR (-rV premultiplied, N
     * direct), its data vector (rY or Y), matrix (rAA rV x rV or rA N x rV)
     * and DIAG Lipschitz metric L[rV] */
    int n, dense;
    void *dY, *dA, *dL;
};
static Rec *g_rec = nullptr;

/* The operator norm of the reduced problem is seeded with time(NULL)
 * (src/operator_norm_matrix.cpp:182): a constant here (this library is
 * linked -Bsymbolic so its own calls bind to it) makes the recorded L
 * reproducible. */
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
    if (g_rec) {
        g_rec->called++;
        g_rec->rV = V;
        g_rec->rE = E;
        memcpy(g_rec->rEu, Eu, sizeof(int) * E);
        memcpy(g_rec->rEv, Ev, sizeof(int) * E);
        memcpy(g_rec->rLa_d1, La_d1, sizeof(real) * E);
        if (La_l1) memcpy(g_rec->rLa_l1, La_l1, sizeof(real) * V);
        g_rec->n = N;
        if (!g_rec->dense) {
            memcpy(g_rec->rY, Y, sizeof(real) * V);
            if (A) memcpy(g_rec->rAA, A, sizeof(real) * V);
        } else {
            memcpy(g_rec->dY, Y, sizeof(real) * (N > 0 ? N : V));
            memcpy(g_rec->dA, A, sizeof(real) * (N > 0 ? (size_t)N * V : (size_t)V * V));
            memcpy(g_rec->dL, L, sizeof(real) * V);
        }
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

/* the graph exactly as the reference's initialize() builds it (:92-97) */
template <typename real>
static Graph<real, real, real> *make_graph(int V, int E, const int *Eu, const int *Ev) {
    Graph<real, real, real> *G = new Graph<real, real, real>(V, E);
    G->add_node(V);
    for (int e = 0; e < E; e++) G->add_edge(Eu[e], Ev[e], (real)0, (real)0);
    for (int v = 0; v < V; v++) G->add_tweights(v, (real)0, (real)0);
    return G;
}

template <typename real>
static int init(int V, int E, int N, const real *Y, const real *A, const int *Eu, const int *Ev,
                const real *La_d1, const real *La_l1, int positivity, real *rX0) {
    int rV = 0, CP_it = 0;
    int *Cv = (int *)malloc(sizeof(int) * V);
    real *rX = nullptr;
    CP_PFDR_graph_quadratic_d1_l1<real>(V, E, N, &rV, Cv, &rX, Y, A, Eu, Ev, La_d1, La_l1,
                                        positivity, (real)0, 0, &CP_it, (real)1.5, (real)1e-3,
                                        (real)0, (real)1e-4, 10, nullptr, nullptr, nullptr, 0,
                                        nullptr);
    rX0[0] = rX[0];
    free(rX);
    free(Cv);
    return rV;
}

template <typename real>
static int step(int V, int E, int N, const real *Y, const real *A, const int *Eu, const int *Ev,
                const real *La_d1, const real *La_l1, int positivity, real CP_difTol,
                real rho, real condMin, real difRcd, real difTol, int itMax,
                /* state in / out */
                uint8_t *active, int *Cv, int *Vc, int *rVc, int *rV, real *rX,
                const real *R_in, uint8_t *segment,
                /* recorded reduced problem */
                int *called, int *rE, int *rEu, int *rEv, real *rLa_d1, real *rLa_l1, real *rY,
                real *rAA, int *n_out, real *dY, real *dA, real *dL) {
    CPql1_Restart<real> rs;
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
    if (N > 0) {  /* the residual Y - A X of the state (the caller's) */
        rs.R = (real *)malloc(sizeof(real) * N);
        memcpy(rs.R, R_in, sizeof(real) * N);
    }
    real *x = (real *)malloc(sizeof(real) * (*rV));
    memcpy(x, rX, sizeof(real) * (*rV));
    Rec rec{0, 0, 0, rEu, rEv, rLa_d1, rLa_l1, rY, rAA, 0, N != 0, dY, dA, dL};
    g_rec = &rec;
    int CP_it = 0;
    CP_PFDR_graph_quadratic_d1_l1<real>(V, E, N, rV, Cv, &x, Y, A, Eu, Ev, La_d1, La_l1,
                                        positivity, CP_difTol, 1, &CP_it, rho, condMin, difRcd,
                                        difTol, itMax, nullptr, nullptr, nullptr, 0, &rs);
    g_rec = nullptr;
    *called = rec.called;
    *rE = rec.rE;
    if (n_out) *n_out = rec.n;
    for (int e = 0; e < E; e++) active[e] = rs.G->arcs[2 * e].is_active;
    for (int v = 0; v < V; v++) segment[v] = (uint8_t)rs.G->what_segment(v);
    memcpy(Vc, rs.Vc, sizeof(int) * V);
    memcpy(rVc, rs.rVc, sizeof(int) * (*rV + 1));
    memcpy(rX, x, sizeof(real) * (*rV));
    free(x);
    delete rs.G;
    free(rs.Vc);
    free(rs.rVc);
    free(rs.R);
    return CP_it;
}

template <typename real>
static real maxflow(int V, int E, const int *Eu, const int *Ev, const real *tr_cap,
                    const real *r_cap, uint8_t *segment) {
    Graph<real, real, real> *G = make_graph<real>(V, E, Eu, Ev);
    for (int v = 0; v < V; v++) G->nodes[v].tr_cap = tr_cap[v];
    for (int e = 0; e < E; e++) {
        G->arcs[2 * e].r_cap = r_cap[e];
        G->arcs[2 * e + 1].r_cap = r_cap[e];
    }
    const real f = G->maxflow();
    for (int v = 0; v < V; v++) segment[v] = (uint8_t)G->what_segment(v);
    delete G;
    return f;
}

#define CP_STEP_API(T, SFX)                                                                   \
    extern "C" int cp_ref_init_##SFX(int V, int E, const T *Y, const T *A, const int *Eu,     \
                                     const int *Ev, const T *La_d1, const T *La_l1, int pos,   \
                                     T *rX0) {                                                 \
        return init<T>(V, E, 0, Y, A, Eu, Ev, La_d1, La_l1, pos, rX0);                         \
    }                                                                                          \
    extern "C" int cp_ref_init_dense_##SFX(int V, int E, int N, const T *Y, const T *A,       \
                                           const int *Eu, const int *Ev, const T *La_d1,       \
                                           const T *La_l1, int pos, T *rX0) {                  \
        return init<T>(V, E, N, Y, A, Eu, Ev, La_d1, La_l1, pos, rX0);                         \
    }                                                                                          \
    extern "C" int cp_ref_step_dense_##SFX(                                                    \
        int V, int E, int N, const T *Y, const T *A, const int *Eu, const int *Ev,             \
        const T *La_d1, const T *La_l1, int pos, T CP_difTol, T rho, T condMin, T difRcd,      \
        T difTol, int itMax, uint8_t *active, int *Cv, int *Vc, int *rVc, int *rV, T *rX,      \
        const T *R, uint8_t *segment, int *called, int *rE, int *rEu, int *rEv, T *rLa_d1,     \
        T *rLa_l1, int *n_out, T *dY, T *dA, T *dL) {                                          \
        return step<T>(V, E, N, Y, A, Eu, Ev, La_d1, La_l1, pos, CP_difTol, rho, condMin,      \
                       difRcd, difTol, itMax, active, Cv, Vc, rVc, rV, rX, R, segment, called,  \
                       rE, rEu, rEv, rLa_d1, rLa_l1, nullptr, nullptr, n_out, dY, dA, dL);     \
    }                                                                                          \
    extern "C" int cp_ref_step_##SFX(                                                          \
        int V, int E, const T *Y, const T *A, const int *Eu, const int *Ev, const T *La_d1,    \
        const T *La_l1, int pos, T CP_difTol, T rho, T condMin, T difRcd, T difTol, int itMax, \
        uint8_t *active, int *Cv, int *Vc, int *rVc, int *rV, T *rX, uint8_t *segment,         \
        int *called, int *rE, int *rEu, int *rEv, T *rLa_d1, T *rLa_l1, T *rY, T *rAA) {       \
        return step<T>(V, E, 0, Y, A, Eu, Ev, La_d1, La_l1, pos, CP_difTol, rho, condMin,      \
                       difRcd, difTol, itMax, active, Cv, Vc, rVc, rV, rX, nullptr, segment,    \
                       called, rE, rEu, rEv, rLa_d1, rLa_l1, rY, rAA, nullptr, nullptr,         \
                       nullptr, nullptr);                                                       \
    }                                                                                          \
    extern "C" T cp_ref_maxflow_##SFX(int V, int E, const int *Eu, const int *Ev,              \
                                      const T *tr_cap, const T *r_cap, uint8_t *segment) {     \
        return maxflow<T>(V, E, Eu, Ev, tr_cap, r_cap, segment);                               \
    }
CP_STEP_API(float, f32)
CP_STEP_API(double, f64)
