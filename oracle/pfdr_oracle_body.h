/* ==========================================================================
 * TEST INFRASTRUCTURE ONLY — NOT PART OF THE PRODUCT.
 *
 * Clean-room, single-threaded C restatement of the PFDR inner solvers of
 * ai3DVision/CP_PFDR_graph_d1 (reference mounted at /root/reference).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this code, and only as the checker / CPU baseline, never as the thing
 * measured or shipped.  The product (cp_pfdr_graph_d1_amd/csrc) never links
 * or calls it.
 *
 * This body is included twice by pfdr_oracle.c with
 *     REAL = float  / SFX = f32      and      REAL = double / SFX = f64.
 * It is organised by phase, one function per GPU kernel boundary of the
 * product, NOT as a transcription of the reference loop.
 * Arithmetic is written so that each floating point operation happens in the
 * same order and with the same operands as in the reference, which makes the
 * restatement bit-exact against the reference compiled without OpenMP and
 * with -ffp-contract=off (pinned by test_oracle_vs_reference_random in
 * tests/test_oracle.py and by the golden fixtures in tests/golden/).
 *
 * Parity pinning:  tests/golden/*.npz were produced by the REAL reference
 * (oracle/_ref, compiled from /root/reference/src by oracle/Makefile) via
 * tests/golden/make_golden.py.
 * ======================================================================== */

#define CAT_(a, b) a##_##b
#define CAT(a, b) CAT_(a, b)
#define FN(name) CAT(name, SFX)

/* -------------------------------------------------------------------------
 * Quadratic data term helpers: "apply A" and "gradient".
 * ref: src/PFDR_graph_quadratic_d1_l1.cpp:355-385 (apply A),
 *      :431-445 (gradient). Identical roles in
 *      src/PFDR_graph_quadratic_d1_bounds.cpp:339-418.
 * Modes: N>0 direct (A is N-by-V column major), N<0 A^tA given (V-by-V),
 *        N==0 diagonal (A = diag of A^tA, length V) or identity (A NULL).
 * ---------------------------------------------------------------------- */
static void FN(oq_apply_A)(int V, int N, const REAL *A, const REAL *X,
                           const REAL *Y, REAL *R, REAL *P)
{
    if (N > 0){
        /* R = Y - A X, accumulated per observation n over v ascending */
        for (int n = 0; n < N; n++){
            REAL acc = (REAL) 0;
            long idx = n;
            for (int v = 0; v < V; v++, idx += N){ acc += A[idx]*X[v]; }
            R[n] = Y[n] - acc;
        }
    }else if (N < 0){
        for (int v = 0; v < V; v++){
            const REAL *col = A + (long) V*v;
            REAL acc = (REAL) 0;
            for (int u = 0; u < V; u++){ acc += col[u]*X[u]; }
            P[v] = acc;
        }
    }else if (A){
        for (int v = 0; v < V; v++){ P[v] = A[v]*X[v]; }
    }else{
        for (int v = 0; v < V; v++){ P[v] = X[v]; }
    }
}

static void FN(oq_gradient)(int V, int N, const REAL *A, const REAL *Y,
                            const REAL *R, REAL *P)
{
    if (N > 0){
        for (int v = 0; v < V; v++){
            const REAL *col = A + (long) N*v;
            REAL acc = (REAL) 0;
            for (int n = 0; n < N; n++){ acc += col[n]*R[n]; }
            P[v] = -acc;
        }
    }else{
        for (int v = 0; v < V; v++){ P[v] -= Y[v]; }
    }
}

/* data term of the objective, computed after oq_apply_A.
 * ref: src/PFDR_graph_quadratic_d1_l1.cpp:388-400 */
static REAL FN(oq_data_objective)(int V, int N, const REAL *X, const REAL *Y,
                                  const REAL *R, const REAL *P)
{
    REAL s = (REAL) 0;
    if (N > 0){
        for (int n = 0; n < N; n++){ s += R[n]*R[n]; }
        return ((REAL) 0.5)*s;
    }
    for (int v = 0; v < V; v++){ s += X[v]*(((REAL) 0.5)*P[v] - Y[v]); }
    return s;
}

/* total variation sum_e la_e |x_u - x_v|. ref: :402-410 */
static REAL FN(oq_tv_objective)(int E, const int *Eu, const int *Ev,
                                const REAL *La_d1, const REAL *X)
{
    REAL s = (REAL) 0;
    for (int e = 0; e < E; e++){
        REAL d = X[Eu[e]] - X[Ev[e]];
        if (d < (REAL) 0){ s -= La_d1[e]*d; } else { s += La_d1[e]*d; }
    }
    return s;
}

/* weighted l1 norm. ref: :411-421.  NOTE: the reference multiplies negative
 * coordinates by La_d1[e] with a stale e (out of bounds read, :417); the
 * restatement uses the intended La_l1[v].  The two agree whenever X >= 0
 * (e.g. positivity) or La_l1 == NULL; tests only compare Obj there. */
static REAL FN(oq_l1_objective)(int V, const REAL *La_l1, const REAL *X)
{
    REAL s = (REAL) 0;
    for (int v = 0; v < V; v++){
        REAL x = X[v];
        if (x < (REAL) 0){ s -= La_l1[v]*x; } else { s += La_l1[v]*x; }
    }
    return s;
}

/* -------------------------------------------------------------------------
 * Preconditioning of the quadratic solvers.
 * ref: src/PFDR_graph_quadratic_d1_l1.cpp:57-268 (l1 flavour),
 *      src/PFDR_graph_quadratic_d1_bounds.cpp:58-242 (bounds flavour:
 *      identical except that it has no l1 section).
 * XY is Y on the first call (Pgrad == NULL) and the iterate X on a
 * reconditioning call, where Pgrad holds the gradient of the smooth part and
 * Zu, Zv the current auxiliary variables.
 * La_l1 / with_l1: the l1 section (:205-219, :262-264) runs only for the l1
 * flavour with La_l1 != NULL.
 * ---------------------------------------------------------------------- */
static void FN(oq_precondition)(int V, int E, int N, const REAL *XY,
    const REAL *A, const int *Eu, const int *Ev, const REAL *La_d1,
    const REAL *La_l1, int Ltype_diag, const REAL *L, REAL *Ga,
    const REAL *Pgrad, REAL *Zu, REAL *Zv, REAL *Wu, REAL *Wv,
    REAL *W_d1u, REAL *W_d1v, REAL *Th_d1, REAL *Th_l1, REAL rho,
    REAL condMin)
{
    const REAL zero = (REAL) 0, one = (REAL) 1;
    REAL *acc = (REAL*) malloc((size_t) V*sizeof(REAL)); /* per-vertex sums */

    if (Pgrad){ /* auxiliary variables -> subgradients (:89-99) */
        for (int e = 0; e < E; e++){
            int u = Eu[e], v = Ev[e];
            Zu[e] = (Wu[e]/Ga[u])*(XY[u] - Ga[u]*Pgrad[u] - Zu[e]);
            Zv[e] = (Wv[e]/Ga[v])*(XY[v] - Ga[v]*Pgrad[v] - Zv[e]);
        }
    }

    /* diagonal of A^t A (:101-122) */
    if (N > 0){
        for (int v = 0; v < V; v++){
            const REAL *col = A + (long) N*v;
            REAL s = zero;
            for (int n = 0; n < N; n++){ s += col[n]*col[n]; }
            Ga[v] = s;
        }
    }else if (N < 0){
        for (int v = 0; v < V; v++){ Ga[v] = A[(long) (V + 1)*v]; }
    }else if (A){
        for (int v = 0; v < V; v++){ Ga[v] = A[v]; }
    }else{
        for (int v = 0; v < V; v++){ Ga[v] = one; }
    }

    /* amplitude scale c (:124-154) */
    const REAL *amp;
    if (!Pgrad){
        if (N > 0){
            for (int v = 0; v < V; v++){
                const REAL *col = A + (long) N*v;
                REAL s = zero;
                for (int n = 0; n < N; n++){ s += col[n]*XY[n]; }
                acc[v] = s/Ga[v];
            }
        }else{
            for (int v = 0; v < V; v++){
                REAL g = Ga[v];
                acc[v] = (g > zero) ? XY[v]/g : zero;
            }
        }
        amp = acc;
    }else{
        amp = XY;
    }
    REAL c = zero;
    int cnt = 0;
    for (int v = 0; v < V; v++){
        REAL a = amp[v];
        if (a > zero){ c += a; cnt++; }
        else if (a < zero){ c -= a; cnt++; }
    }
    c = (!Pgrad) ? ((REAL) cnt)/c : c/((REAL) cnt);

    /* d1 contribution to the metric and splitting weights (:156-203);
     * the per-vertex sums run in increasing edge order, u side first */
    for (int v = 0; v < V; v++){ acc[v] = zero; }
    for (int e = 0; e < E; e++){
        int u = Eu[e], v = Ev[e];
        REAL w;
        if (!Pgrad){
            w = c*La_d1[e];
        }else{
            REAL xu = XY[u], xv = XY[v], d = xu - xv;
            if (xu < zero){ xu = -xu; }
            if (xv < zero){ xv = -xv; }
            if (d < zero){ d = -d; }
            if (xu < xv){ xu = xv; }
            if (xu < c){ xu = c; }
            xu *= condMin;
            if (d < xu){ d = xu; }
            w = La_d1[e]/d;
        }
        acc[u] += w;
        acc[v] += w;
        Wu[e] = w;
        Wv[e] = w;
    }
    for (int v = 0; v < V; v++){ Ga[v] += acc[v]; }
    for (int v = 0; v < V; v++){ acc[v] = one/acc[v]; }
    for (int e = 0; e < E; e++){
        Wu[e] *= acc[Eu[e]];
        Wv[e] *= acc[Ev[e]];
    }

    if (La_l1){ /* l1 contribution (:205-219) */
        if (!Pgrad){
            for (int v = 0; v < V; v++){ Ga[v] += c*La_l1[v]; }
        }else{
            REAL cm = c*condMin;
            for (int v = 0; v < V; v++){
                REAL d = XY[v];
                if (d < zero){ d = -d; }
                if (d < cm){ d = cm; }
                Ga[v] += La_l1[v]/d;
            }
        }
    }

    /* invert the approximate Hessian, then cap it (:221-239) */
    for (int v = 0; v < V; v++){ Ga[v] = one/Ga[v]; }
    REAL cap = ((REAL) 1.9)*(((REAL) 2) - rho);
    if (!Ltype_diag || !L){
        if (L){ cap /= (*L); }
        for (int v = 0; v < V; v++){ if (Ga[v] > cap){ Ga[v] = cap; } }
    }else{
        for (int v = 0; v < V; v++){
            if (L[v] > zero){
                REAL b = cap/L[v];
                if (Ga[v] > b){ Ga[v] = b; }
            }
        }
    }

    if (Pgrad){ /* subgradients -> auxiliary variables (:241-250) */
        for (int e = 0; e < E; e++){
            int u = Eu[e], v = Ev[e];
            Zu[e] = XY[u] - Ga[u]*(Pgrad[u] + Zu[e]/Wu[e]);
            Zv[e] = XY[v] - Ga[v]*(Pgrad[v] + Zv[e]/Wv[e]);
        }
    }

    /* per-edge prox constants (:252-261) */
    for (int e = 0; e < E; e++){
        REAL wu = Wu[e]/Ga[Eu[e]];
        REAL wv = Wv[e]/Ga[Ev[e]];
        REAL s = wu + wv;
        Th_d1[e] = La_d1[e]*s/(wu*wv);
        W_d1u[e] = wu/s;
        W_d1v[e] = wv/s;
    }
    if (La_l1){
        for (int v = 0; v < V; v++){ Th_l1[v] = Ga[v]*La_l1[v]; }
    }
    free(acc);
}

/* forward step P = 2X - Ga*grad (:462-464) */
static void FN(oq_forward)(int V, const REAL *X, const REAL *Ga, REAL *P)
{
    for (int v = 0; v < V; v++){ P[v] = ((REAL) 2)*X[v] - Ga[v]*P[v]; }
}

/* backward step on the auxiliary variables: weighted average, soft
 * threshold of the difference, relaxed update (:466-489) */
static void FN(oq_edge_prox)(int E, const int *Eu, const int *Ev,
    const REAL *P, const REAL *X, REAL *Zu, REAL *Zv, const REAL *W_d1u,
    const REAL *W_d1v, const REAL *Th_d1, REAL rho)
{
    for (int e = 0; e < E; e++){
        int u = Eu[e], v = Ev[e];
        REAL wu = W_d1u[e], wv = W_d1v[e], th = Th_d1[e];
        REAL avg = wu*(P[u] - Zu[e]) + wv*(P[v] - Zv[e]);
        REAL dif = (P[u] - Zu[e]) - (P[v] - Zv[e]);
        if (dif > th){
            dif -= th;
            Zu[e] += rho*(avg + wv*dif - X[u]);
            Zv[e] += rho*(avg - wu*dif - X[v]);
        }else if (dif < -th){
            dif += th;
            Zu[e] += rho*(avg + wv*dif - X[u]);
            Zv[e] += rho*(avg - wu*dif - X[v]);
        }else{
            Zu[e] += rho*(avg - X[u]);
            Zv[e] += rho*(avg - X[v]);
        }
    }
}

/* Douglas-Rachford average X = sum_incident W*Z, increasing e (:491-497) */
static void FN(oq_average)(int V, int E, const int *Eu, const int *Ev,
    const REAL *Wu, const REAL *Zu, const REAL *Wv, const REAL *Zv, REAL *X)
{
    for (int v = 0; v < V; v++){ X[v] = (REAL) 0; }
    for (int e = 0; e < E; e++){
        X[Eu[e]] += Wu[e]*Zu[e];
        X[Ev[e]] += Wv[e]*Zv[e];
    }
}

/* relative squared evolution, also refreshes X_ (:514-529) */
static REAL FN(oq_evolution)(int V, const REAL *X, REAL *X_, REAL eps)
{
    REAL num = (REAL) 0, den = (REAL) 0;
    for (int v = 0; v < V; v++){
        REAL a = X[v], b = X_[v] - a;
        num += b*b;
        den += a*a;
        X_[v] = a;
    }
    return (den > eps) ? num/den : num/eps;
}

/* -------------------------------------------------------------------------
 * Shared driver of the two quadratic solvers.
 * ref: src/PFDR_graph_quadratic_d1_l1.cpp:270-553 and
 *      src/PFDR_graph_quadratic_d1_bounds.cpp:244-530.
 * flavour 0: l1 + positivity (La_l1, positivity);
 * flavour 1: box bounds (lo, hi; +-HUGE_VAL means no bound).
 * ---------------------------------------------------------------------- */
static void FN(oq_quadratic)(int flavour, int V, int E, int N, REAL *X,
    const REAL *Y, const REAL *A, const int *Eu, const int *Ev,
    const REAL *La_d1, const REAL *La_l1, int positivity, REAL lo, REAL hi,
    int Ltype_diag, const REAL *L, REAL rho, REAL condMin, REAL difRcd,
    REAL difTol, int itMax, int *it, REAL *Obj, REAL *Dif)
{
    const REAL zero = (REAL) 0;
    const REAL mach = ORACLE_EPS;
    const REAL eps = (zero < difTol && difTol < mach) ? difTol : mach;
    const REAL inf = ORACLE_HUGE;
    if (flavour == 1){ La_l1 = NULL; positivity = 0; }

    size_t sV = (size_t) V*sizeof(REAL), sE = (size_t) E*sizeof(REAL);
    REAL *Ga = (REAL*) malloc(sV), *P = (REAL*) malloc(sV);
    REAL *Zu = (REAL*) malloc(sE), *Zv = (REAL*) malloc(sE);
    REAL *Wu = (REAL*) malloc(sE), *Wv = (REAL*) malloc(sE);
    REAL *W_d1u = (REAL*) malloc(sE), *W_d1v = (REAL*) malloc(sE);
    REAL *Th_d1 = (REAL*) malloc(sE);
    REAL *Th_l1 = La_l1 ? (REAL*) malloc(sV) : NULL;
    REAL *R = (N > 0) ? (REAL*) malloc((size_t) N*sizeof(REAL)) : NULL;
    REAL *X_ = NULL;

    for (int e = 0; e < E; e++){ Zu[e] = X[Eu[e]]; Zv[e] = X[Ev[e]]; }
    FN(oq_precondition)(V, E, N, Y, A, Eu, Ev, La_d1, La_l1, Ltype_diag, L,
        Ga, NULL, NULL, NULL, Wu, Wv, W_d1u, W_d1v, Th_d1, Th_l1, rho,
        condMin);

    const REAL difTol2 = difTol*difTol;
    REAL difRcd2 = difRcd*difRcd;
    REAL dif = (difTol2 > difRcd2) ? difTol2 : difRcd2;
    const int track = (difTol > zero || difRcd > zero || Dif != NULL);
    if (track){
        X_ = (REAL*) malloc(sV);
        memcpy(X_, X, sV);
    }

    int k = 0;
    for (;;){
        FN(oq_apply_A)(V, N, A, X, Y, R, P);
        if (Obj){
            Obj[k] = FN(oq_data_objective)(V, N, X, Y, R, P)
                   + FN(oq_tv_objective)(E, Eu, Ev, La_d1, X);
            if (La_l1){ Obj[k] += FN(oq_l1_objective)(V, La_l1, X); }
        }
        if (k == itMax || dif < difTol2){ break; }
        FN(oq_gradient)(V, N, A, Y, R, P);
        if (dif < difRcd2){
            FN(oq_precondition)(V, E, N, X, A, Eu, Ev, La_d1, La_l1,
                Ltype_diag, L, Ga, P, Zu, Zv, Wu, Wv, W_d1u, W_d1v, Th_d1,
                Th_l1, rho, condMin);
            difRcd2 *= (REAL) 0.01;
        }
        FN(oq_forward)(V, X, Ga, P);
        FN(oq_edge_prox)(E, Eu, Ev, P, X, Zu, Zv, W_d1u, W_d1v, Th_d1, rho);
        FN(oq_average)(V, E, Eu, Ev, Wu, Zu, Wv, Zv, X);
        if (flavour == 0){ /* l1 prox + positivity (:499-512) */
            if (La_l1){
                for (int v = 0; v < V; v++){
                    REAL x = X[v], th = Th_l1[v];
                    if (x > th){ X[v] = x - th; }
                    else if (!positivity && x < -th){ X[v] = x + th; }
                    else { X[v] = zero; }
                }
            }else if (positivity){
                for (int v = 0; v < V; v++){ if (X[v] < zero){ X[v] = zero; } }
            }
        }else{ /* box projection (bounds :472-490) */
            int haslo = -inf < lo, hashi = hi < inf;
            if (haslo && hashi){
                for (int v = 0; v < V; v++){
                    if (X[v] < lo){ X[v] = lo; } else if (X[v] > hi){ X[v] = hi; }
                }
            }else if (haslo){
                for (int v = 0; v < V; v++){ if (X[v] < lo){ X[v] = lo; } }
            }else if (hashi){
                for (int v = 0; v < V; v++){ if (X[v] > hi){ X[v] = hi; } }
            }
        }
        if (track){
            dif = FN(oq_evolution)(V, X, X_, eps);
            if (Dif){ Dif[k] = dif; }
        }
        k++;
    }
    *it = k;
    free(Ga); free(P); free(Zu); free(Zv); free(Wu); free(Wv);
    free(W_d1u); free(W_d1v); free(Th_d1); free(Th_l1); free(R); free(X_);
}

void FN(oracle_pfdr_quadratic_d1_l1)(int V, int E, int N, REAL *X,
    const REAL *Y, const REAL *A, const int *Eu, const int *Ev,
    const REAL *La_d1, const REAL *La_l1, int positivity, int Ltype,
    const REAL *L, REAL rho, REAL condMin, REAL difRcd, REAL difTol,
    int itMax, int *it, REAL *Obj, REAL *Dif)
{
    FN(oq_quadratic)(0, V, E, N, X, Y, A, Eu, Ev, La_d1, La_l1, positivity,
        (REAL) 0, (REAL) 0, Ltype, L, rho, condMin, difRcd, difTol, itMax,
        it, Obj, Dif);
}

void FN(oracle_pfdr_quadratic_d1_bounds)(int V, int E, int N, REAL *X,
    const REAL *Y, const REAL *A, const int *Eu, const int *Ev,
    const REAL *La_d1, REAL lo, REAL hi, int Ltype, const REAL *L, REAL rho,
    REAL condMin, REAL difRcd, REAL difTol, int itMax, int *it, REAL *Obj,
    REAL *Dif)
{
    FN(oq_quadratic)(1, V, E, N, X, Y, A, Eu, Ev, La_d1, NULL, 0, lo, hi,
        Ltype, L, rho, condMin, difRcd, difTol, itMax, it, Obj, Dif);
}

/* -------------------------------------------------------------------------
 * Projection of each D-column onto {x >= 0, sum x = a} in metric diag(1/m),
 * by the active-set sweep of src/proj_simplex_metric.cpp:18-83.
 * ---------------------------------------------------------------------- */
void FN(oracle_proj_simplex_metric)(REAL *X, const REAL *M, int D, int N,
                                     int nm, const REAL *Asum, int na)
{
    unsigned char *active = (unsigned char*) malloc((size_t) (D > 0 ? D : 1));
    for (int n = 0; n < N; n++){
        REAL *x = X + (long) D*n;
        const REAL *m = (nm > n) ? M + (long) D*n : M + (long) D*(nm - 1);
        REAL target = (na > n) ? Asum[n] : Asum[na - 1];
        /* first pass: running threshold over the coordinates seen so far */
        REAL lam = (x[0] - target)/m[0];
        REAL msum = m[0];
        x[0] = x[0]/m[0];
        active[0] = 1;
        for (int d = 1; d < D; d++){
            x[d] = x[d]/m[d];
            if (x[d] > lam){
                active[d] = 1;
                msum += m[d];
                lam += m[d]*(x[d] - lam)/msum;
            }else{
                active[d] = 0;
            }
        }
        /* drop coordinates fallen below the threshold until stable */
        int changed = 1;
        while (changed){
            changed = 0;
            for (int d = 0; d < D; d++){
                if (active[d] && x[d] < lam){
                    active[d] = 0;
                    msum -= m[d];
                    lam += m[d]*(lam - x[d])/msum;
                    changed = 1;
                }
            }
        }
        for (int d = 0; d < D; d++){
            x[d] = active[d] ? (x[d] - lam)*m[d] : (REAL) 0;
        }
    }
    free(active);
}

/* -------------------------------------------------------------------------
 * Simplex-constrained solver.  ref: src/PFDR_graph_loss_d1_simplex.cpp.
 * loss: al == 0 linear, al == 1 quadratic (exact equality), otherwise the
 * smoothed Kullback-Leibler branch (the reference tests al == 1 and al > 0
 * exactly like this: :95, :106, :160-171, :251, :264).
 * Layouts: P, Q, Ga, GaQ are K-by-V (index v*K + k); edge state is K-by-E.
 * ---------------------------------------------------------------------- */
struct FN(os_consts) { REAL al, alK, al1, alKal1; int K; };

/* ref: :64-370 */
static void FN(os_precondition)(const struct FN(os_consts) *cst, int V, int E,
    const REAL *La_f, const REAL *P, const REAL *Q, const int *Eu,
    const int *Ev, const REAL *La_d1, REAL *Ga, REAL *GaQ, REAL *Zu,
    REAL *Zv, REAL *Wu, REAL *Wv, REAL *W_d1u, REAL *W_d1v, REAL *Th_d1,
    REAL rho, REAL condMin)
{
    const int K = cst->K;
    const REAL al = cst->al, alK = cst->alK, al1 = cst->al1;
    const REAL alKal1 = cst->alKal1;
    const REAL zero = (REAL) 0, one = (REAL) 1;
    const long VK = (long) V*K, EK = (long) E*K;
    const int recond = (Zu != NULL);

    if (recond){
        /* recover the metric before its per-vertex normalisation (:92-135) */
        if (al == one){
            if (!La_f){
                for (long i = 0; i < VK; i++){ Ga[i] = GaQ[i]; }
            }else{
                for (int v = 0; v < V; v++){
                    REAL s = one/La_f[v];
                    for (int k = 0; k < K; k++){ Ga[v*K+k] = s*GaQ[v*K+k]; }
                }
            }
        }else if (al > zero){
            if (!La_f){
                for (long i = 0; i < VK; i++){ Ga[i] = GaQ[i]/(alK + al1*Q[i]); }
            }else{
                for (int v = 0; v < V; v++){
                    REAL s = one/La_f[v];
                    for (int k = 0; k < K; k++){
                        long i = (long) v*K + k;
                        Ga[i] = s*GaQ[i]/(alK + al1*Q[i]);
                    }
                }
            }
        }else{
            for (int v = 0; v < V; v++){
                long b = (long) v*K;
                int imax = 0;
                REAL qmax = Q[b];
                for (int k = 1; k < K; k++){
                    if (qmax < Q[b+k]){ qmax = Q[b+k]; imax = k; }
                }
                REAL s = GaQ[b+imax]/qmax/Ga[b+imax];
                for (int k = 0; k < K; k++){ Ga[b+k] *= s; }
            }
        }
        /* auxiliary variables -> subgradients (:136-156) */
        for (int e = 0; e < E; e++){
            long u = (long) Eu[e]*K, v = (long) Ev[e]*K, i = (long) e*K;
            for (int k = 0; k < K; k++, u++, v++, i++){
                if (al == zero){
                    Zu[i] = (Wu[i]/Ga[u])*(P[u] + GaQ[u] - Zu[i]);
                    Zv[i] = (Wv[i]/Ga[v])*(P[v] + GaQ[v] - Zv[i]);
                }else if (al == one){
                    Zu[i] = (Wu[i]/Ga[u])*(P[u] - GaQ[u]*(P[u] - Q[u]) - Zu[i]);
                    Zv[i] = (Wv[i]/Ga[v])*(P[v] - GaQ[v]*(P[v] - Q[v]) - Zv[i]);
                }else{
                    Zu[i] = (Wu[i]/Ga[u])*(P[u] + GaQ[u]/(alKal1 + P[u]) - Zu[i]);
                    Zv[i] = (Wv[i]/Ga[v])*(P[v] + GaQ[v]/(alKal1 + P[v]) - Zv[i]);
                }
            }
        }
    }

    /* Hessian of the loss (:159-190) */
    if (al == zero){
        for (long i = 0; i < VK; i++){ Ga[i] = zero; }
    }else if (al == one){
        if (!La_f){
            for (long i = 0; i < VK; i++){ Ga[i] = one; }
        }else{
            for (int v = 0; v < V; v++){
                for (int k = 0; k < K; k++){ Ga[(long) v*K+k] = La_f[v]; }
            }
        }
    }else{
        for (int v = 0; v < V; v++){
            REAL lf = La_f ? La_f[v] : one;
            for (int k = 0; k < K; k++){
                long i = (long) v*K + k;
                REAL t = alKal1 + P[i];
                if (La_f){ Ga[i] = lf*(alK + al1*Q[i])/(t*t); }
                else { Ga[i] = (alK + al1*Q[i])/(t*t); }
            }
        }
    }

    /* d1 contribution and splitting weights (:192-241); per (vertex,k)
     * sums in increasing edge order, u side first */
    REAL *acc;
    if (al == zero){ acc = Ga; }
    else {
        for (long i = 0; i < VK; i++){ GaQ[i] = zero; }
        acc = GaQ;
    }
    for (int e = 0; e < E; e++){
        long u = (long) Eu[e]*K, v = (long) Ev[e]*K, i = (long) e*K;
        for (int k = 0; k < K; k++, u++, v++, i++){
            REAL w;
            if (!recond){
                w = La_d1[e];
            }else{
                REAL d = P[u] - P[v];
                if (d < zero){ d = -d; }
                if (d < condMin){ d = condMin; }
                w = La_d1[e]/d;
            }
            acc[u] += w;
            acc[v] += w;
            Wu[i] = w;
            Wv[i] = w;
        }
    }
    if (al > zero){ for (long i = 0; i < VK; i++){ Ga[i] += acc[i]; } }
    for (long i = 0; i < VK; i++){ acc[i] = one/acc[i]; }
    for (int e = 0; e < E; e++){
        long u = (long) Eu[e]*K, v = (long) Ev[e]*K, i = (long) e*K;
        for (int k = 0; k < K; k++, u++, v++, i++){
            Wu[i] *= acc[u];
            Wv[i] *= acc[v];
        }
    }
    if (al > zero){ for (long i = 0; i < VK; i++){ Ga[i] = one/Ga[i]; } }

    /* cap by the Lipschitz constant of the loss (:249-285) */
    REAL cap = ((REAL) 1.9)*(((REAL) 2) - rho);
    if (al == one){
        if (La_f){
            for (int v = 0; v < V; v++){
                REAL cv = cap/La_f[v];
                for (int k = 0; k < K; k++){
                    long i = (long) v*K + k;
                    if (Ga[i] > cv){ Ga[i] = cv; }
                }
            }
        }else if (cap < one){
            for (long i = 0; i < VK; i++){ if (Ga[i] > cap){ Ga[i] = cap; } }
        }
    }else if (al > zero){
        if (!La_f){
            REAL b = one/(alKal1*alKal1);
            for (long i = 0; i < VK; i++){
                REAL cv = cap/((alK + al1*Q[i])*b);
                if (Ga[i] > cv){ Ga[i] = cv; }
            }
        }else{
            for (int v = 0; v < V; v++){
                REAL b = La_f[v]*one/(alKal1*alKal1);
                for (int k = 0; k < K; k++){
                    long i = (long) v*K + k;
                    REAL cv = cap/((alK + al1*Q[i])*b);
                    if (Ga[i] > cv){ Ga[i] = cv; }
                }
            }
        }
    }

    /* prox weights and thresholds (:287-306) */
    if (al > zero){
        for (int e = 0; e < E; e++){
            long u = (long) Eu[e]*K, v = (long) Ev[e]*K, i = (long) e*K;
            REAL la = La_d1[e];
            for (int k = 0; k < K; k++, u++, v++, i++){
                REAL wu = Wu[i]/Ga[u], wv = Wv[i]/Ga[v], s = wu + wv;
                Th_d1[i] = la*s/(wu*wv);
                W_d1u[i] = wu/s;
                W_d1v[i] = wv/s;
            }
        }
    }
    /* metric times first-order information (:307-335) */
    if (al == zero){
        for (long i = 0; i < VK; i++){ GaQ[i] = Ga[i]*Q[i]; }
    }else if (al == one){
        if (!La_f){
            for (long i = 0; i < VK; i++){ GaQ[i] = Ga[i]; }
        }else{
            for (int v = 0; v < V; v++){
                for (int k = 0; k < K; k++){
                    long i = (long) v*K + k;
                    GaQ[i] = La_f[v]*Ga[i];
                }
            }
        }
    }else{
        for (int v = 0; v < V; v++){
            for (int k = 0; k < K; k++){
                long i = (long) v*K + k;
                if (La_f){ GaQ[i] = La_f[v]*Ga[i]*(alK + al1*Q[i]); }
                else { GaQ[i] = Ga[i]*(alK + al1*Q[i]); }
            }
        }
    }
    if (recond){ /* subgradients -> auxiliary variables (:337-358) */
        for (int e = 0; e < E; e++){
            long u = (long) Eu[e]*K, v = (long) Ev[e]*K, i = (long) e*K;
            for (int k = 0; k < K; k++, u++, v++, i++){
                if (al == zero){
                    Zu[i] = P[u] + GaQ[u] - (Ga[u]/Wu[i])*Zu[i];
                    Zv[i] = P[v] + GaQ[v] - (Ga[v]/Wv[i])*Zv[i];
                }else if (al == one){
                    Zu[i] = P[u] - GaQ[u]*(P[u] - Q[u] + Zu[i]/Wu[i]);
                    Zv[i] = P[v] - GaQ[v]*(P[v] - Q[v] + Zv[i]/Wv[i]);
                }else{
                    Zu[i] = P[u] + GaQ[u]/(alKal1 + P[u]) - (Ga[u]/Wu[i])*Zu[i];
                    Zv[i] = P[v] + GaQ[v]/(alKal1 + P[v]) - (Ga[v]/Wv[i])*Zv[i];
                }
            }
        }
    }
    /* normalise the metric of each vertex by its maximum (:360-369) */
    for (int v = 0; v < V; v++){
        long b = (long) v*K;
        REAL mx = Ga[b];
        for (int k = 1; k < K; k++){ if (Ga[b+k] > mx){ mx = Ga[b+k]; } }
        for (int k = 0; k < K; k++){ Ga[b+k] /= mx; }
    }
}

/* objective (:476-544) */
static REAL FN(os_objective)(const struct FN(os_consts) *cst, int V, int E,
    const REAL *La_f, const REAL *P, const REAL *Q, const int *Eu,
    const int *Ev, const REAL *La_d1)
{
    const int K = cst->K;
    const REAL al = cst->al, zero = (REAL) 0;
    const long VK = (long) V*K;
    REAL s = zero;
    if (al == zero){
        for (long i = 0; i < VK; i++){ s -= P[i]*Q[i]; }
    }else if (al == (REAL) 1){
        if (!La_f){
            for (long i = 0; i < VK; i++){ REAL d = P[i] - Q[i]; s += d*d; }
        }else{
            for (int v = 0; v < V; v++){
                REAL b = zero;
                for (int k = 0; k < K; k++){
                    REAL d = P[(long) v*K+k] - Q[(long) v*K+k];
                    b += d*d;
                }
                s += La_f[v]*b;
            }
        }
        s *= (REAL) 0.5;
    }else{
        if (!La_f){
            for (long i = 0; i < VK; i++){
                REAL c = cst->alK + cst->al1*Q[i];
                s += c*ORACLE_LOG(c/(cst->alK + cst->al1*P[i]));
            }
        }else{
            for (int v = 0; v < V; v++){
                REAL b = zero;
                for (int k = 0; k < K; k++){
                    long i = (long) v*K + k;
                    REAL c = cst->alK + cst->al1*Q[i];
                    b += c*ORACLE_LOG(c/(cst->alK + cst->al1*P[i]));
                }
                s += La_f[v]*b;
            }
        }
    }
    REAL tv = zero;
    for (int e = 0; e < E; e++){
        long u = (long) Eu[e]*K, v = (long) Ev[e]*K;
        REAL b = zero;
        for (int k = 0; k < K; k++){
            REAL d = P[u+k] - P[v+k];
            if (d < zero){ b -= d; } else { b += d; }
        }
        tv += La_d1[e]*b;
    }
    return s + tv;
}

/* ref: :372-715 */
void FN(oracle_pfdr_loss_d1_simplex)(int K, int V, int E, REAL al,
    const REAL *La_f, REAL *P, const REAL *Q, const int *Eu, const int *Ev,
    const REAL *La_d1, REAL rho, REAL condMin, REAL difRcd, REAL difTol,
    int itMax, int *it, REAL *Obj, REAL *Dif)
{
    const REAL zero = (REAL) 0, one = (REAL) 1, two = (REAL) 2;
    const REAL half = (REAL) 0.5;
    struct FN(os_consts) cst;
    cst.K = K; cst.al = al;
    cst.alK = cst.al1 = cst.alKal1 = zero;
    if (zero < al && al < one){
        cst.alK = al/K;
        cst.al1 = one - al;
        cst.alKal1 = cst.alK/cst.al1;
    }
    const long VK = (long) V*K, EK = (long) E*K;
    size_t sVK = (size_t) VK*sizeof(REAL), sEK = (size_t) EK*sizeof(REAL);
    REAL *Ga = (REAL*) malloc(sVK), *GaQ = (REAL*) malloc(sVK);
    REAL *FP = (REAL*) malloc(sVK);
    REAL *Zu = (REAL*) malloc(sEK), *Zv = (REAL*) malloc(sEK);
    REAL *Wu = (REAL*) malloc(sEK), *Wv = (REAL*) malloc(sEK);
    REAL *W_d1u = NULL, *W_d1v = NULL, *Th_d1 = NULL;
    if (al > zero){
        W_d1u = (REAL*) malloc(sEK); W_d1v = (REAL*) malloc(sEK);
        Th_d1 = (REAL*) malloc(sEK);
    }
    for (int e = 0; e < E; e++){
        for (int k = 0; k < K; k++){
            Zu[(long) e*K+k] = P[(long) Eu[e]*K+k];
            Zv[(long) e*K+k] = P[(long) Ev[e]*K+k];
        }
    }
    FN(os_precondition)(&cst, V, E, La_f, P, Q, Eu, Ev, La_d1, Ga, GaQ,
        NULL, NULL, Wu, Wv, W_d1u, W_d1v, Th_d1, rho, condMin);

    REAL dif = (difTol > difRcd) ? difTol : difRcd;
    const int track = (difTol > zero || difRcd > zero || Dif != NULL);
    const int labels = (difTol >= one);
    REAL *P_ = NULL;
    if (track){
        if (labels){
            P_ = (REAL*) malloc((size_t) V*sizeof(REAL));
            for (int v = 0; v < V; v++){
                long b = (long) v*K;
                REAL mx = P[b];
                P_[v] = zero;
                for (int k = 1; k < K; k++){
                    if (P[b+k] > mx){ mx = P[b+k]; P_[v] = (REAL) k; }
                }
            }
        }else{
            P_ = (REAL*) malloc(sVK);
            memcpy(P_, P, sVK);
        }
    }
    const REAL unit = one;
    int k_it = 0;
    for (;;){
        if (Obj){
            Obj[k_it] = FN(os_objective)(&cst, V, E, La_f, P, Q, Eu, Ev, La_d1);
        }
        if (k_it == itMax || dif < difTol){ break; }
        if (dif < difRcd){
            FN(os_precondition)(&cst, V, E, La_f, P, Q, Eu, Ev, La_d1, Ga,
                GaQ, Zu, Zv, Wu, Wv, W_d1u, W_d1v, Th_d1, rho, condMin);
            difRcd *= (REAL) 0.1;
        }
        /* explicit step (:567-587) */
        for (long i = 0; i < VK; i++){
            if (al == zero){ FP[i] = two*P[i] + GaQ[i]; }
            else if (al == one){ FP[i] = two*P[i] - GaQ[i]*(P[i] - Q[i]); }
            else { FP[i] = two*P[i] + GaQ[i]/(cst.alKal1 + P[i]); }
        }
        /* implicit d1 step on the auxiliary variables (:589-634) */
        for (int e = 0; e < E; e++){
            long u = (long) Eu[e]*K, v = (long) Ev[e]*K, i = (long) e*K;
            for (int k = 0; k < K; k++, u++, v++, i++){
                REAL a = FP[u] - Zu[i];
                REAL b = FP[v] - Zv[i];
                if (al == zero){
                    REAL avg = half*(a + b);
                    REAL d = a - b;
                    if (d > two){
                        d = half*(d - two);
                        Zu[i] += rho*(avg + d - P[u]);
                        Zv[i] += rho*(avg - d - P[v]);
                    }else if (d < -two){
                        d = half*(d + two);
                        Zu[i] += rho*(avg + d - P[u]);
                        Zv[i] += rho*(avg - d - P[v]);
                    }else{
                        Zu[i] += rho*(avg - P[u]);
                        Zv[i] += rho*(avg - P[v]);
                    }
                }else{
                    REAL avg = W_d1u[i]*a + W_d1v[i]*b;
                    REAL d = a - b, th = Th_d1[i];
                    if (d > th){
                        d -= th;
                        Zu[i] += rho*(avg + W_d1v[i]*d - P[u]);
                        Zv[i] += rho*(avg - W_d1u[i]*d - P[v]);
                    }else if (d < -th){
                        d += th;
                        Zu[i] += rho*(avg + W_d1v[i]*d - P[u]);
                        Zv[i] += rho*(avg - W_d1u[i]*d - P[v]);
                    }else{
                        Zu[i] += rho*(avg - P[u]);
                        Zv[i] += rho*(avg - P[v]);
                    }
                }
            }
        }
        /* average, per label in increasing edge order (:636-648) */
        for (long i = 0; i < VK; i++){ P[i] = zero; }
        for (int e = 0; e < E; e++){
            for (int k = 0; k < K; k++){
                long i = (long) e*K + k;
                P[(long) Eu[e]*K+k] += Wu[i]*Zu[i];
                P[(long) Ev[e]*K+k] += Wv[i]*Zv[i];
            }
        }
        FN(oracle_proj_simplex_metric)(P, Ga, K, V, V, &unit, 1);
        if (track){ /* (:653-691) */
            dif = zero;
            if (labels){
                for (int v = 0; v < V; v++){
                    long b = (long) v*K;
                    REAL mx = P[b];
                    int lab = 0;
                    for (int k = 1; k < K; k++){
                        if (P[b+k] > mx){ mx = P[b+k]; lab = k; }
                    }
                    REAL fl = (REAL) lab;
                    if (fl != P_[v]){ dif += one; P_[v] = fl; }
                }
            }else{
                for (long i = 0; i < VK; i++){
                    REAL d = P_[i] - P[i];
                    if (d < zero){ d = -d; }
                    dif += d;
                    P_[i] = P[i];
                }
                dif /= V;
            }
            if (Dif){ Dif[k_it] = dif; }
        }
        k_it++;
    }
    *it = k_it;
    free(Ga); free(GaQ); free(FP); free(Zu); free(Zv); free(Wu); free(Wv);
    free(W_d1u); free(W_d1v); free(Th_d1); free(P_);
}

#undef FN
#undef CAT
#undef CAT_
