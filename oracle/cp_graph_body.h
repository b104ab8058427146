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

/* ------------------------------------------------------------------------
 * The simplex driver's steps (reference src/CP_PFDR_graph_loss_d1_simplex.cpp),
 * K labels, P[v*K + k] layouts, single-threaded.  al: 0 linear loss, 1
 * quadratic, 0 < al < 1 smoothed KL (al_K = al/K, al_1 = 1 - al,
 * al_K_al_1 = al_K/al_1, :208-212); eps is the driver's finite-difference
 * precision (:214-231), passed by the caller.
 * ------------------------------------------------------------------------ */

/* :733-766 (and initialize() :96-108 for the single first component):
 * per component the sums of Q over its vertices in Vc order; linear loss:
 * rQ = the sums, rP = the corner of the largest (first on ties); otherwise
 * rQ = rP = sums / size, rLa_f = size */
void FN(oracle_cp_simplex_reduced)(int K, REAL al, const REAL *Q, const int *Vc, const int *rVc,
                                   int rV, REAL *rP, REAL *rQ, REAL *rLa_f)
{
    int rv, s, k, i;
    for (rv = 0; rv < rV; rv++) {
        REAL *rPv = rP + (size_t)rv * K, *rQv = rQ + (size_t)rv * K;
        for (k = 0; k < K; k++) rPv[k] = (REAL)0;
        for (s = rVc[rv]; s < rVc[rv + 1]; s++) {
            const REAL *Qv = Q + (size_t)Vc[s] * K;
            for (k = 0; k < K; k++) rPv[k] += Qv[k];
        }
        if (al == (REAL)0) {
            REAL a = rPv[i = 0];
            for (k = 1; k < K; k++)
                if (rPv[k] > a) a = rPv[i = k];
            for (k = 0; k < K; k++) {
                rQv[k] = rPv[k];
                rPv[k] = (k == i) ? (REAL)1 : (REAL)0;
            }
        } else {
            i = rVc[rv + 1] - rVc[rv];
            for (k = 0; k < K; k++) {
                rQv[k] = rPv[k] / i;
                rPv[k] = rQv[k];
            }
            if (rLa_f) rLa_f[rv] = (REAL)i;
        }
    }
}

/* :327-376 gradient DfS[V*K] of the loss at the piecewise-constant rP plus
 * the d1 term over the active arcs in the maxflow graph's order; then
 * :525-536 rDi[rV], the most confident label of each component (first on
 * ties) */
void FN(oracle_cp_simplex_gradient)(int K, int V, int E, REAL al, const REAL *Q, const int *Eu,
                                    const int *Ev, const REAL *La_d1, const uint8_t *active,
                                    const int *Cv, int rV, const REAL *rP, REAL eps, REAL *DfS,
                                    int *rDi)
{
    int *first = (int *)malloc(sizeof(int) * (V > 0 ? V : 1));
    int *next = (int *)malloc(sizeof(int) * (2 * (size_t)E + 1));
    int v, k, a, rv, i;
    REAL al_K = (REAL)0, al_1 = (REAL)0, al_K_al_1 = (REAL)0;
    if ((REAL)0 < al && al < (REAL)1) {
        al_K = al / K;
        al_1 = (REAL)1 - al;
        al_K_al_1 = al_K / al_1;
    }
    cpg_lists(V, E, Eu, Ev, first, next);
    for (v = 0; v < V; v++) {
        REAL *D = DfS + (size_t)v * K;
        const REAL *Qv = Q + (size_t)v * K, *rPv = rP + (size_t)Cv[v] * K;
        for (k = 0; k < K; k++) {
            if (al == (REAL)0) D[k] = -Qv[k];
            else if (al == (REAL)1) D[k] = rPv[k] - Qv[k];
            else D[k] = -(al_K + al_1 * Qv[k]) / (al_K_al_1 + rPv[k]);
        }
    }
    for (v = 0; v < V; v++) {
        REAL *D = DfS + (size_t)v * K;
        const REAL *rPv = rP + (size_t)Cv[v] * K;
        for (a = first[v]; a != -1; a = next[a]) {
            if (active[a >> 1]) {
                const REAL *rPu = rP + (size_t)Cv[cpg_head(a, Eu, Ev)] * K;
                const REAL w = La_d1[a >> 1];
                for (k = 0; k < K; k++) {
                    const REAL d = rPv[k] - rPu[k];
                    if (d > eps) D[k] += w;
                    else if (d < -eps) D[k] -= w;
                }
            }
        }
    }
    for (rv = 0; rv < rV; rv++) {
        const REAL *rPv = rP + (size_t)rv * K;
        REAL m = rPv[0];
        i = 0;
        for (k = 1; k < K; k++)
            if (rPv[k] > m) m = rPv[i = k];
        rDi[rv] = i;
    }
    free(first);
    free(next);
}

/* :542-595 capacities of alpha-expansion n (1 <= n < K): source/sink per
 * vertex from its component's label i = rDi and its current alternative
 * Djv, then the d1 terms of the inactive edges in edge order (tr_cap[u] +=
 * c - a, tr_cap[v] -= c); r_cap[e] is the capacity of arc 2e (u -> v), arc
 * 2e + 1 has none */
void FN(oracle_cp_simplex_capacities)(int K, int V, int E, int n, const int *Eu, const int *Ev,
                                      const REAL *La_d1, const uint8_t *active, const int *Vc,
                                      const int *rVc, int rV, const int *rDi, const int *Djv,
                                      const REAL *DfS, REAL *tr_cap, REAL *r_cap)
{
    int rv, s, v, i, j, k, e;
    for (rv = 0; rv < rV; rv++) {
        i = rDi[rv];
        j = n > i ? n : (n - 1);
        for (s = rVc[rv]; s < rVc[rv + 1]; s++) {
            const REAL *D;
            v = Vc[s];
            D = DfS + (size_t)v * K;
            k = Djv[v];
            if (k == 0) tr_cap[v] = D[j] - D[i];
            else if (k == n) tr_cap[v] = (REAL)0;
            else if (k > i) tr_cap[v] = D[j] - D[k];
            else tr_cap[v] = D[j] - D[k - 1];
        }
    }
    for (e = 0; e < E; e++) {
        if (active[e]) {
            r_cap[e] = (REAL)0;
        } else {
            const int u = Eu[e];
            v = Ev[e];
            j = Djv[u];
            k = Djv[v];
            {
                const REAL a = (j == k) ? (REAL)0 : (REAL)2 * La_d1[e];
                const REAL b = (REAL)2 * La_d1[e], c = (REAL)2 * La_d1[e];
                tr_cap[u] += c - a;
                tr_cap[v] -= c;
                r_cap[e] = b + c - a;
            }
        }
    }
}

/* :782-803 deactivate the active edges whose components' label vectors
 * differ by at most eps in every label; returns how many */
int FN(oracle_cp_simplex_merge)(int K, int E, const int *Eu, const int *Ev, const int *Cv,
                                const REAL *rP, REAL eps, uint8_t *active)
{
    int e, k, n = 0;
    for (e = 0; e < E; e++) {
        if (active[e]) {
            const REAL *rPu = rP + (size_t)Cv[Eu[e]] * K, *rPv = rP + (size_t)Cv[Ev[e]] * K;
            REAL a = (REAL)0;
            for (k = 0; k < K; k++) {
                REAL d = rPu[k] - rPv[k];
                if (d < (REAL)0) d = -d;
                if (d > a) a = d;
            }
            if (a <= eps) {
                active[e] = 0;
                n++;
            }
        }
    }
    return n;
}

#ifndef ORACLE_CPG_SIMPLEX_INT_DEFINED
#define ORACLE_CPG_SIMPLEX_INT_DEFINED
/* :600-604 the sink side of expansion n takes alternative n */
void oracle_cp_simplex_expand(int V, int n, const uint8_t *segment, int *Djv)
{
    int v;
    for (v = 0; v < V; v++)
        if (segment[v]) Djv[v] = n;
}

/* :608-618 activate the inactive edges whose ends took different
 * alternatives; returns how many */
int oracle_cp_simplex_activate(int E, const int *Eu, const int *Ev, const int *Djv,
                               uint8_t *active)
{
    int e, s = 0;
    for (e = 0; e < E; e++) {
        if (!active[e] && Djv[Eu[e]] != Djv[Ev[e]]) {
            active[e] = 1;
            s++;
        }
    }
    return s;
}
#endif

/* ------------------------------------------------------------------------
 * The duplex driver (src/CP_PFDR_graph_quadratic_d1_l1_duplex.cpp), its
 * non-differentiable case (La_l1 or positivity): a two-layer maxflow graph,
 * node v (v1) and node V + v (v2) per vertex (:101-116).  One cut per
 * iteration (:469-545): directional derivatives up / down (:473-502), then
 * m = MAX(0, MAX(-up, down)), tr_cap[v1] = -down + m, tr_cap[v2] =
 * -(up + m), the arc v1 -> v2 of capacity m (v2 -> v1 none), and every arc
 * of an inactive edge in both layers La_d1[e] (:504-527).  With positivity
 * and no La_l1 the reference leaves up / down of the nonzero components
 * uninitialised (:470-502, malloc): they are DfS here, the evident intent.
 * Its gradient is the l1 driver's (:363-433, oracle_cp_gradient).
 * ------------------------------------------------------------------------ */
void FN(oracle_cp_capacities_duplex)(int V, int E, const REAL *La_d1, const REAL *La_l1,
                                     int positivity, const uint8_t *active, const int *Cv,
                                     const REAL *rX, const REAL *DfS, REAL *tr_cap,
                                     REAL *r_link, REAL *r_cap)
{
    int v, e;
    for (v = 0; v < V; v++) {
        const REAL x = rX[Cv[v]];
        REAL up = DfS[v], dn = DfS[v], in, m;
        if (La_l1 && x == (REAL)0) {
            up = DfS[v] + La_l1[v];
            dn = DfS[v] - La_l1[v];
        }
        if (positivity && x == (REAL)0) dn = -ORACLE_HUGE;
        in = ((-up) > (dn)) ? (-up) : (dn);
        m = (((REAL)0) > (in)) ? ((REAL)0) : (in);
        tr_cap[v] = -dn + m;
        tr_cap[V + v] = -(up + m);
        r_link[v] = m;
    }
    for (e = 0; e < E; e++) r_cap[e] = active[e] ? (REAL)0 : La_d1[e];
}

#ifndef ORACLE_CPG_DUPLEX_INT_DEFINED
#define ORACLE_CPG_DUPLEX_INT_DEFINED
/* :531-545 activate the inactive edges whose ends the cut separates in
 * either layer (segment[2V]); returns how many */
int oracle_cp_activate_duplex(int V, int E, const int *Eu, const int *Ev, const uint8_t *segment,
                              uint8_t *active)
{
    int e, w = 0;
    for (e = 0; e < E; e++) {
        if (!active[e] && (segment[Eu[e]] != segment[Ev[e]] ||
                           segment[Eu[e] + V] != segment[Ev[e] + V])) {
            active[e] = 1;
            w++;
        }
    }
    return w;
}
#endif
