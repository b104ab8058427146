/* TEST INFRASTRUCTURE ONLY — restatement of the cut-pursuit graph steps
 * around each reduced PFDR solve, from
 * reference src/CP_PFDR_graph_quadratic_d1_l1.cpp, single-threaded:
 *
 *   oracle_cp_components      connected components of the graph minus its
 *                             active edges, DFS-queue order          :566-597
 *   oracle_cp_reduced_graph   reduced edges, TV weights, l1 weights  :599-661
 *   oracle_cp_merge           deactivate edges between components with
 *                             (relatively) equal values              :863-886
 *   oracle_cp_gradient        gradient of the smooth part at the current
 *                             piecewise-constant iterate, plus the d1 and
 *                             l1 directional terms                   :339-400
 *   oracle_cp_capacities      source/sink and edge capacities of the single
 *                             (differentiable) or first/second cut   :402-535
 *   oracle_cp_activate        activate the (inactive) edges a cut separates
 *                                                          :430-440, :521-556
 *
 * The maxflow graph's adjacency (reference include/graph.hpp:395-416,
 * add_edge): edge e owns arcs 2e (from Eu[e], head Ev[e]) and 2e+1 (from
 * Ev[e], head Eu[e]); each arc is PREPENDED to its origin's list, so a
 * vertex's arcs are visited newest first.  The restatement rebuilds exactly
 * those lists (cpg_lists).  Segments: 0 = SOURCE, 1 = SINK
 * (what_segment with its SINK default, include/graph.hpp:419-429).
 * Included twice by pfdr_oracle.c with REAL / SFX; the integer-only steps
 * are defined once.  Parity: pinned against the reference's own CP
 * iterations (tests/golden/make_cp_golden.py, oracle/harness/cp_step.cpp).
 */
#include <stdint.h>

#define CAT_(a, b) a##_##b
#define CAT(a, b) CAT_(a, b)
#define FN(name) CAT(name, SFX)

#ifndef ORACLE_CPG_INT_DEFINED
#define ORACLE_CPG_INT_DEFINED

/* first[V] / next[2E] arc lists of add_edge (graph.hpp:405-408); -1 ends */
static void cpg_lists(int V, int E, const int *Eu, const int *Ev, int *first, int *next)
{
    int v, e;
    for (v = 0; v < V; v++) first[v] = -1;
    for (e = 0; e < E; e++) {
        next[2 * e] = first[Eu[e]];
        first[Eu[e]] = 2 * e;
        next[2 * e + 1] = first[Ev[e]];
        first[Ev[e]] = 2 * e + 1;
    }
}

static int cpg_head(int a, const int *Eu, const int *Ev)
{
    return (a & 1) ? Eu[a >> 1] : Ev[a >> 1];
}

/* :566-597 — returns rV; Cv[V], Vc[V], rVc[rV + 1] */
int oracle_cp_components(int V, int E, const int *Eu, const int *Ev, const uint8_t *active,
                         int *Cv, int *Vc, int *rVc)
{
    int *first = (int *)malloc(sizeof(int) * (V > 0 ? V : 1));
    int *next = (int *)malloc(sizeof(int) * (2 * (size_t)E + 1));
    int u, v, w, a, rV = 0, n = 0, i = 0;
    cpg_lists(V, E, Eu, Ev, first, next);
    for (v = 0; v < V; v++) Cv[v] = -1;
    rVc[0] = 0;
    for (u = 0; u < V; u++) {
        if (Cv[u] != -1) continue;
        Cv[u] = rV;
        Vc[n++] = u;
        while (i < n) {
            v = Vc[i++];
            for (a = first[v]; a != -1; a = next[a]) {
                if (!active[a >> 1]) {
                    w = cpg_head(a, Eu, Ev);
                    if (Cv[w] != -1) continue;
                    Cv[w] = rV;
                    Vc[n++] = w;
                }
            }
        }
        rVc[++rV] = n;
    }
    free(first);
    free(next);
    return rV;
}

/* :430-440 / :521-535 / :544-556 — activate the inactive edges whose ends
 * the cut separates; returns how many */
int oracle_cp_activate(int E, const int *Eu, const int *Ev, const uint8_t *segment,
                       uint8_t *active)
{
    int e, w = 0;
    for (e = 0; e < E; e++) {
        if (segment[Eu[e]] != segment[Ev[e]] && !active[e]) {
            active[e] = 1;
            w++;
        }
    }
    return w;
}

#endif /* ORACLE_CPG_INT_DEFINED */

/* :599-661 — returns rE; outputs sized E + rV (rLa_l1: rV, when La_l1).
 * Reproduces the reference's bookkeeping exactly, including its rEc reset
 * (:645-648), which clears the end marker of an isolated component that a
 * later non-isolated component follows, so that component's eps self-loop
 * is attributed to the next non-isolated component. */
int FN(oracle_cp_reduced_graph)(int V, int E, const int *Eu, const int *Ev, const REAL *La_d1,
                                const REAL *La_l1, const uint8_t *active, const int *Cv,
                                const int *Vc, const int *rVc, int rV, REAL eps, int *rEu,
                                int *rEv, REAL *rLa_d1, REAL *rLa_l1)
{
    int *first = (int *)malloc(sizeof(int) * (V > 0 ? V : 1));
    int *next = (int *)malloc(sizeof(int) * (2 * (size_t)E + 1));
    int *rEc = (int *)malloc(sizeof(int) * (rV > 0 ? rV : 1));
    int ru, rv, re, s, t, u, a, i, rE = 0, n = 0;
    cpg_lists(V, E, Eu, Ev, first, next);
    for (rv = 0; rv < rV; rv++) rEc[rv] = -1;
    for (ru = 0; ru < rV; ru++) {
        if (La_l1) rLa_l1[ru] = (REAL)0;
        i = 1;
        for (s = rVc[ru], t = rVc[ru + 1]; s < t; s++) {
            u = Vc[s];
            if (La_l1) rLa_l1[ru] += La_l1[u];
            for (a = first[u]; a != -1; a = next[a]) {
                const int e = a >> 1;
                REAL w;
                if (!active[e]) continue;
                w = La_d1[e];
                if (w == (REAL)0) continue;
                i = 0;
                rv = Cv[cpg_head(a, Eu, Ev)];
                if (rv < ru) continue;
                re = rEc[rv];
                if (re == -1) {
                    rEv[rE] = rv;
                    rLa_d1[rE] = w;
                    rEc[rv] = rE++;
                } else {
                    rLa_d1[re] += w;
                }
            }
        }
        if (i) {
            rEv[rE] = ru;
            rLa_d1[rE++] = eps;
        } else {
            for (; n < rE; n++) rEc[rEv[n]] = -1;
        }
        rEc[ru] = rE;
    }
    re = 0;
    for (ru = 0; ru < rV; ru++) {
        while (re < rEc[ru]) rEu[re++] = ru;
    }
    free(first);
    free(next);
    free(rEc);
    return rE;
}

/* :863-886 — returns the number of deactivated edges */
int FN(oracle_cp_merge)(int E, const int *Eu, const int *Ev, const int *Cv, const REAL *rX,
                        REAL eps, REAL difTol, uint8_t *active)
{
    int e, n = 0;
    for (e = 0; e < E; e++) {
        if (active[e]) {
            REAL a = rX[Cv[Eu[e]]], b = rX[Cv[Ev[e]]], d = a - b;
            if (a < (REAL)0) a = -a;
            if (b < (REAL)0) b = -b;
            if (d < (REAL)0) d = -d;
            if (a < b) a = b;
            d = (a > eps) ? d / a : d / eps;
            if (d <= difTol) {
                active[e] = 0;
                n++;
            }
        }
    }
    return n;
}

/* :339-400 — DfS[V].  N > 0: R is the residual Y - A X of the caller;
 * N < 0: A = A^tA (V-by-V), Y = A^tY; N = 0: A diagonal or NULL. */
void FN(oracle_cp_gradient)(int N, int V, int E, const REAL *A, const REAL *Y, const REAL *R,
                            const int *Eu, const int *Ev, const REAL *La_d1, const REAL *La_l1,
                            const uint8_t *active, const int *Cv, const int *Vc, const int *rVc,
                            int rV, const REAL *rX, REAL *DfS)
{
    int *first = (int *)malloc(sizeof(int) * (V > 0 ? V : 1));
    int *next = (int *)malloc(sizeof(int) * (2 * (size_t)E + 1));
    int u, v, n, rv, s, t, a;
    cpg_lists(V, E, Eu, Ev, first, next);
    if (N > 0) {  /* :342-352 */
        for (v = 0; v < V; v++) {
            const REAL *Av = A + (size_t)N * v;
            REAL c = (REAL)0;
            for (n = 0; n < N; n++) c += Av[n] * R[n];
            DfS[v] = -c;
        }
    } else if (N < 0) {  /* :353-368 */
        for (u = 0; u < V; u++) {
            const REAL *Av = A + (size_t)V * u;
            REAL b = (REAL)0;
            for (rv = 0; rv < rV; rv++) {
                REAL c = (REAL)0;
                if (rX[rv] == (REAL)0) continue;
                for (s = rVc[rv], t = rVc[rv + 1]; s < t; s++) c += Av[Vc[s]];
                b += c * rX[rv];
            }
            DfS[u] = b - Y[u];
        }
    } else if (A) {  /* :369-373 */
        for (v = 0; v < V; v++) DfS[v] = A[v] * rX[Cv[v]] - Y[v];
    } else {  /* :374-376 */
        for (v = 0; v < V; v++) DfS[v] = rX[Cv[v]] - Y[v];
    }
    for (u = 0; u < V; u++) {  /* :379-394 d1 term, arcs newest first */
        for (a = first[u]; a != -1; a = next[a]) {
            if (active[a >> 1]) {
                const REAL d = rX[Cv[u]] - rX[Cv[cpg_head(a, Eu, Ev)]];
                if (d > (REAL)0) DfS[u] += La_d1[a >> 1];
                else if (d < (REAL)0) DfS[u] -= La_d1[a >> 1];
            }
        }
    }
    if (La_l1) {  /* :396-413 l1 term (one add per vertex) */
        for (v = 0; v < V; v++) {
            const REAL x = rX[Cv[v]];
            if (x > (REAL)0) DfS[v] += La_l1[v];
            else if (x < (REAL)0) DfS[v] -= La_l1[v];
        }
    }
    free(first);
    free(next);
}

/* :402-535 — cut 0: the only cut of the differentiable case (La_l1 NULL
 * and no positivity, :415-430); cut 1: directions +1_U (:442-476); cut 2:
 * directions -1_U (:478-518).  Edge capacities from the activity BEFORE
 * the cut's own activations (:420-429, :464-474, :519-535). */
/* the bounds driver's cuts (src/CP_PFDR_graph_quadratic_d1_bounds.cpp:386-534):
 * cut 0 (min = -inf, max = inf) tr = DfS; cut 1 (directions +1_U): +inf on
 * components at max (when max < inf), else DfS; cut 2 (-1_U): +inf on
 * components at min (when -inf < min), else -DfS; edges as above */
void FN(oracle_cp_capacities_bounds)(int cut, int V, int E, const REAL *La_d1, REAL mn, REAL mx,
                                     const uint8_t *active, const int *Cv, const REAL *rX,
                                     const REAL *DfS, REAL *tr_cap, REAL *r_cap)
{
    int v, e;
    const REAL inf = ORACLE_HUGE;
    for (v = 0; v < V; v++) {
        const REAL x = rX[Cv[v]];
        if (cut == 1) tr_cap[v] = (mx < inf && x == mx) ? inf : DfS[v];
        else if (cut == 2) tr_cap[v] = (-inf < mn && x == mn) ? inf : -DfS[v];
        else tr_cap[v] = DfS[v];
    }
    for (e = 0; e < E; e++) r_cap[e] = active[e] ? (REAL)0 : La_d1[e];
}

void FN(oracle_cp_capacities)(int cut, int V, int E, const REAL *La_d1, const REAL *La_l1,
                              int positivity, const uint8_t *active, const int *Cv,
                              const REAL *rX, const REAL *DfS, REAL *tr_cap, REAL *r_cap)
{
    int v, e;
    for (v = 0; v < V; v++) {
        const int zero = rX[Cv[v]] == (REAL)0;
        if (cut == 1 && La_l1 && zero) tr_cap[v] = DfS[v] + La_l1[v];
        else if (cut == 2 && zero) tr_cap[v] = positivity ? -ORACLE_HUGE : DfS[v] - La_l1[v];
        else tr_cap[v] = DfS[v];
    }
    for (e = 0; e < E; e++) r_cap[e] = active[e] ? (REAL)0 : La_d1[e];
}
