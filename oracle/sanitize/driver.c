/* TEST INFRASTRUCTURE ONLY — memory / undefined-behaviour check of the CPU
 * oracle ("ASan on the CPU restatement").
 *
 * Compiled together with the restatement (../pfdr_oracle.c) under
 * -fsanitize=address,undefined -fno-sanitize-recover=all by
 * tests/test_oracle_sanitize.py, and run: every entry point of the oracle
 * on small synthetic problems -- the three PFDR solvers in every mode they
 * have (identity / diagonal / direct N > 0 / A^tA N < 0 A, l1 / positivity /
 * box / one-sided, linear / quadratic / smoothed-KL simplex with and without
 * La_f, reconditioning, Obj and Dif records, edgeless graphs, isolated
 * vertices, self-loops), the metric projection (nm, na < N), the CP
 * reduced-problem builder (direct and premultiplied) and the CP graph steps
 * (components, activation, reduced graph, merge, gradients, capacities of the
 * l1 / bounds / duplex / simplex drivers).  Exit status 0 and a line per
 * group on stdout; a sanitizer report aborts with a non-zero status.
 * Results are not checked here (tests/test_oracle.py pins them against the
 * reference); this run only proves the restatement stays inside its buffers
 * and free of undefined behaviour on all of its paths. */
#include <stdint.h>
#include <stdio.h>

#include "../pfdr_oracle.c"

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static double urand(void)
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (double)(rng_state >> 11) / 9007199254740992.0;
}

/* 4-neighbour grid of nx x ny (edges right and down), plus optional extras */
static int grid(int nx, int ny, int *Eu, int *Ev)
{
    int E = 0;
    for (int y = 0; y < ny; y++)
        for (int x = 0; x < nx; x++) {
            int v = y * nx + x;
            if (x + 1 < nx) { Eu[E] = v; Ev[E] = v + 1; E++; }
            if (y + 1 < ny) { Eu[E] = v; Ev[E] = v + nx; E++; }
        }
    return E;
}

#define DEFINE_RUNS(REALT, S)                                                          \
static void run_quadratic_##S(int V, int E, const int *Eu, const int *Ev)             \
{                                                                                      \
    const int N = 5, itMax = 40;                                                       \
    REALT *X = calloc(V, sizeof(REALT)), *Y = malloc(sizeof(REALT) * (V + N));         \
    REALT *La = malloc(sizeof(REALT) * (E + 1)), *L1 = malloc(sizeof(REALT) * V);      \
    REALT *Ad = malloc(sizeof(REALT) * V), *Adir = malloc(sizeof(REALT) * N * V);      \
    REALT *AtA = malloc(sizeof(REALT) * V * V), *L = malloc(sizeof(REALT) * V);        \
    REALT *Obj = malloc(sizeof(REALT) * (itMax + 1)), *Dif = malloc(sizeof(REALT) * itMax); \
    int it = 0;                                                                        \
    for (int v = 0; v < V; v++) { Y[v] = (REALT)urand(); L1[v] = (REALT)0.01;          \
        Ad[v] = (REALT)(0.5 + urand()); L[v] = (REALT)2; }                              \
    for (int n = 0; n < N; n++) Y[V + n] = (REALT)urand();                             \
    for (int e = 0; e < E; e++) La[e] = (REALT)(0.05 + 0.1 * urand());                 \
    for (long i = 0; i < (long)N * V; i++) Adir[i] = (REALT)(urand() - 0.5);           \
    for (int i = 0; i < V; i++)                                                        \
        for (int j = 0; j < V; j++) {                                                  \
            REALT s = 0;                                                               \
            for (int n = 0; n < N; n++) s += Adir[(long)N * i + n] * Adir[(long)N * j + n]; \
            AtA[(long)V * i + j] = s + (i == j ? (REALT)1 : (REALT)0);                 \
        }                                                                              \
    for (int mode = 0; mode < 4; mode++) {                                             \
        const REALT *A = mode == 0 ? NULL : mode == 1 ? Ad : mode == 2 ? Adir : AtA;   \
        const int n = mode == 2 ? N : mode == 3 ? -V : 0;                              \
        for (int pos = 0; pos < 2; pos++)                                              \
            for (int l1 = 0; l1 < 2; l1++) {                                           \
                for (int v = 0; v < V; v++) X[v] = (REALT)0;                           \
                oracle_pfdr_quadratic_d1_l1_##S(V, E, n, X, Y, A, Eu, Ev, La,          \
                    l1 ? L1 : NULL, pos, mode == 1 ? 1 : 0, mode == 1 ? L : NULL,      \
                    (REALT)1.5, (REALT)1e-2, (REALT)1e-1, (REALT)1e-6, itMax, &it, Obj, Dif); \
            }                                                                          \
        const REALT inf = (REALT)HUGE_VAL;                                             \
        const REALT lo[4] = {(REALT)0.1, (REALT)0.1, -inf, -inf};                      \
        const REALT hi[4] = {(REALT)0.7, inf, (REALT)0.7, inf};                        \
        for (int b = 0; b < 4; b++) {                                                  \
            for (int v = 0; v < V; v++) X[v] = (REALT)0;                               \
            oracle_pfdr_quadratic_d1_bounds_##S(V, E, n, X, Y, A, Eu, Ev, La, lo[b], hi[b], \
                0, NULL, (REALT)1.5, (REALT)1e-2, (REALT)1e-1, (REALT)0, itMax, &it, Obj, \
                b & 1 ? NULL : Dif);                                                   \
        }                                                                              \
    }                                                                                  \
    free(X); free(Y); free(La); free(L1); free(Ad); free(Adir); free(AtA); free(L);    \
    free(Obj); free(Dif);                                                              \
}                                                                                      \
                                                                                       \
static void run_simplex_##S(int V, int E, const int *Eu, const int *Ev)               \
{                                                                                      \
    const int K = 4, itMax = 30;                                                       \
    REALT *P = malloc(sizeof(REALT) * K * V), *Q = malloc(sizeof(REALT) * K * V);      \
    REALT *Laf = malloc(sizeof(REALT) * V), *La = malloc(sizeof(REALT) * (E + 1));     \
    REALT *Obj = malloc(sizeof(REALT) * (itMax + 1)), *Dif = malloc(sizeof(REALT) * itMax); \
    int it = 0;                                                                        \
    for (int v = 0; v < V; v++) {                                                      \
        REALT s = 0;                                                                   \
        for (int k = 0; k < K; k++) { Q[K * v + k] = (REALT)(0.01 + urand()); s += Q[K * v + k]; } \
        for (int k = 0; k < K; k++) Q[K * v + k] /= s;                                 \
        Laf[v] = (REALT)(0.5 + urand());                                               \
    }                                                                                  \
    for (int e = 0; e < E; e++) La[e] = (REALT)(0.05 + 0.1 * urand());                 \
    const REALT als[4] = {(REALT)0, (REALT)1, (REALT)0.1, (REALT)2};                   \
    for (int a = 0; a < 4; a++)                                                        \
        for (int f = 0; f < 2; f++) {                                                  \
            for (long i = 0; i < (long)K * V; i++) P[i] = Q[i];                        \
            oracle_pfdr_loss_d1_simplex_##S(K, V, E, als[a], f ? Laf : NULL, P, Q, Eu, Ev, La, \
                (REALT)1.5, (REALT)1e-2, (REALT)1e-1, (REALT)1e-6, itMax, &it, Obj,    \
                f ? Dif : NULL);                                                       \
        }                                                                              \
    free(P); free(Q); free(Laf); free(La); free(Obj); free(Dif);                       \
}                                                                                      \
                                                                                       \
static void run_projection_##S(void)                                                   \
{                                                                                      \
    const int D = 7, N = 9;                                                            \
    REALT X[7 * 9], M[7 * 9], Asum[9];                                                 \
    for (int i = 0; i < D * N; i++) { X[i] = (REALT)(urand() - 0.3); M[i] = (REALT)(0.5 + urand()); } \
    for (int n = 0; n < N; n++) Asum[n] = (REALT)(0.5 + urand());                      \
    oracle_proj_simplex_metric_##S(X, M, D, N, N, Asum, N);                            \
    oracle_proj_simplex_metric_##S(X, M, D, N, 2, Asum, 3);                            \
    oracle_proj_simplex_metric_##S(X, M, D, N, 1, Asum, 1);                            \
}                                                                                      \
                                                                                       \
static void run_cp_##S(int V, int E, const int *Eu, const int *Ev)                     \
{                                                                                      \
    const int N = 6, K = 3;                                                            \
    uint8_t *active = malloc(E + 1), *seg = malloc(2 * (size_t)V + 1);                 \
    int *Cv = malloc(sizeof(int) * (V + 1)), *Vc = malloc(sizeof(int) * V);            \
    int *rVc = malloc(sizeof(int) * (V + 1)), *Djv = malloc(sizeof(int) * V);          \
    int *rEu = malloc(sizeof(int) * (E + V + 1)), *rEv = malloc(sizeof(int) * (E + V + 1)); \
    REALT *La = malloc(sizeof(REALT) * (E + 1)), *L1 = malloc(sizeof(REALT) * V);      \
    REALT *rLa = malloc(sizeof(REALT) * (E + V + 1)), *rL1 = malloc(sizeof(REALT) * (V + 1)); \
    REALT *A = malloc(sizeof(REALT) * N * V), *Y = malloc(sizeof(REALT) * (N + V));    \
    REALT *R = malloc(sizeof(REALT) * N), *DfS = malloc(sizeof(REALT) * V * K);        \
    REALT *tr = malloc(sizeof(REALT) * 2 * V), *rc = malloc(sizeof(REALT) * 4 * (E + 1)); \
    REALT *rX = malloc(sizeof(REALT) * (V + 1) * K), *Q = malloc(sizeof(REALT) * V * K); \
    REALT *rA = malloc(sizeof(REALT) * N * V), *rAA = malloc(sizeof(REALT) * V * V);   \
    REALT *rY = malloc(sizeof(REALT) * (N + V)), *Leq = malloc(sizeof(REALT) * (V + 1)), *AtA = malloc(sizeof(REALT) * V * V); \
    for (int e = 0; e < E; e++) { active[e] = urand() < 0.3; La[e] = (REALT)(0.1 * urand()); } \
    for (int v = 0; v < V; v++) { L1[v] = (REALT)0.01; Y[v] = (REALT)urand(); }        \
    for (int n = 0; n < N; n++) { R[n] = (REALT)urand(); Y[V > N ? n : 0] = Y[0]; }    \
    for (long i = 0; i < (long)N * V; i++) A[i] = (REALT)(urand() - 0.5);              \
    for (long i = 0; i < (long)V * V; i++) AtA[i] = (REALT)urand();                    \
    for (long i = 0; i < (long)V * K; i++) Q[i] = (REALT)urand();                      \
    int rV = oracle_cp_components(V, E, Eu, Ev, active, Cv, Vc, rVc);                  \
    for (int r = 0; r < rV * K; r++) rX[r] = (REALT)(urand() < 0.2 ? 0 : urand());     \
    int rE = oracle_cp_reduced_graph_##S(V, E, Eu, Ev, La, L1, active, Cv, Vc, rVc, rV, \
        (REALT)1e-7, rEu, rEv, rLa, rL1);                                              \
    (void)rE;                                                                          \
    oracle_cp_reduce_##S(N, V, A, Y, rV, rVc, Vc, 0, rA, rAA, rY, Leq);              \
    oracle_cp_reduce_##S(N, V, A, Y, rV, rVc, Vc, 1, rA, rAA, rY, Leq);              \
    for (int n = 0; n <= 1; n++) {                                                     \
        oracle_cp_gradient_##S(n ? N : 0, V, E, n ? A : NULL, Y, R, Eu, Ev, La, L1, active, \
            Cv, Vc, rVc, rV, rX, DfS);                                                 \
    }                                                                                  \
    oracle_cp_gradient_##S(-V, V, E, AtA, Y, R, Eu, Ev, La, L1, active, Cv, Vc, rVc, rV, rX, DfS); \
    for (int cut = 0; cut < 3; cut++) {                                                \
        oracle_cp_capacities_##S(cut, V, E, La, L1, cut == 2, active, Cv, rX, DfS, tr, rc); \
        oracle_cp_capacities_bounds_##S(cut, V, E, La, (REALT)0.1, (REALT)0.9, active, Cv, rX, \
            DfS, tr, rc);                                                              \
    }                                                                                  \
    oracle_cp_capacities_duplex_##S(V, E, La, L1, 1, active, Cv, rX, DfS, tr, rc + 2 * (E + 1), rc); \
    for (int v = 0; v < 2 * V; v++) seg[v] = urand() < 0.5;                            \
    (void)oracle_cp_activate_duplex(V, E, Eu, Ev, seg, active);                        \
    (void)oracle_cp_activate(E, Eu, Ev, seg, active);                                  \
    (void)oracle_cp_merge_##S(E, Eu, Ev, Cv, rX, (REALT)1e-7, (REALT)1e-3, active);    \
    rV = oracle_cp_components(V, E, Eu, Ev, active, Cv, Vc, rVc);                      \
    for (int r = 0; r < rV * K; r++) rX[r] = (REALT)urand();                           \
    REALT *rQ = malloc(sizeof(REALT) * (V + 1) * K), *rLaf = malloc(sizeof(REALT) * (V + 1)); \
    int *rDi = malloc(sizeof(int) * (V + 1));                                          \
    for (int a = 0; a < 2; a++)                                                        \
        oracle_cp_simplex_reduced_##S(K, a ? (REALT)0.1 : (REALT)0, Q, Vc, rVc, rV, rX, rQ, rLaf); \
    oracle_cp_simplex_gradient_##S(K, V, E, (REALT)0.1, Q, Eu, Ev, La, active, Cv, rV, rX, \
        (REALT)1e-7, DfS, rDi);                                                        \
    for (int v = 0; v < V; v++) Djv[v] = rDi[Cv[v]];                                   \
    for (int n = 1; n < K; n++) {                                                      \
        oracle_cp_simplex_capacities_##S(K, V, E, n, Eu, Ev, La, active, Vc, rVc, rV, rDi, Djv, \
            DfS, tr, rc);                                                              \
        for (int v = 0; v < V; v++) seg[v] = urand() < 0.5;                            \
        oracle_cp_simplex_expand(V, n, seg, Djv);                                      \
    }                                                                                  \
    (void)oracle_cp_simplex_activate(E, Eu, Ev, Djv, active);                          \
    (void)oracle_cp_simplex_merge_##S(K, E, Eu, Ev, Cv, rX, (REALT)1e-7, active);      \
    free(active); free(seg); free(Cv); free(Vc); free(rVc); free(Djv); free(rEu); free(rEv); \
    free(La); free(L1); free(rLa); free(rL1); free(A); free(Y); free(R); free(DfS);    \
    free(tr); free(rc); free(rX); free(Q); free(rA); free(rAA); free(rY); free(AtA);   \
    free(rQ); free(rLaf); free(rDi); free(Leq);                                                   \
}

DEFINE_RUNS(float, f32)
DEFINE_RUNS(double, f64)

int main(void)
{
    int Eu[4096], Ev[4096];
    const int shapes[][2] = {{9, 7}, {1, 1}, {16, 1}, {5, 5}};
    for (unsigned s = 0; s < sizeof(shapes) / sizeof(shapes[0]); s++) {
        const int nx = shapes[s][0], ny = shapes[s][1], V = nx * ny;
        int E = grid(nx, ny, Eu, Ev);
        if (s == 3) {  /* a self-loop, a duplicate edge and an isolated vertex's neighbourhood */
            Eu[E] = 3; Ev[E] = 3; E++;
            Eu[E] = Eu[0]; Ev[E] = Ev[0]; E++;
        }
        run_quadratic_f32(V, E, Eu, Ev);
        run_quadratic_f64(V, E, Eu, Ev);
        run_simplex_f32(V, E, Eu, Ev);
        run_simplex_f64(V, E, Eu, Ev);
        if (s != 3) {  /* the CP graph steps take the maxflow's inputs: no self-loops */
            run_cp_f32(V, E, Eu, Ev);
            run_cp_f64(V, E, Eu, Ev);
        }
        printf("graph %dx%d (V=%d, E=%d): solvers, CP steps ok\n", nx, ny, V, E);
    }
    run_projection_f32();
    run_projection_f64();
    printf("projection ok\n");
    return 0;
}
