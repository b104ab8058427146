/* TEST INFRASTRUCTURE ONLY — restatement of the cut-pursuit reduced-problem
 * builder (reference src/CP_PFDR_graph_quadratic_d1_l1.cpp:663-841),
 * single-threaded, without its operator-norm call (time-seeded in the
 * reference, :792/:822): the equilibration factors are returned instead and
 * the caller multiplies by a norm of its choice.  Included twice by
 * pfdr_oracle.c with REAL / SFX.  Parity: this restates the reference lines
 * (cited per block) and is checked against the GPU build and against a
 * float64 numpy statement of the same algebra; the reference computes these
 * arrays inside CP and never exposes them, so no reference output pins
 * them directly ("parity pinned to the restatement").
 *
 *   N > 0: rA (N x rV) = component column sums of A (:676-687); when preAt,
 *          rAA = rA^t rA (upper triangle, then mirrored :689-702, :754-763)
 *          and rY = rA^t Y (:704-711); equilibration around the norm
 *          (:772-818) is applied to rAA (preAt) or rA and reverted, the
 *          reverted arrays are returned as the reference leaves them;
 *          Leq[rv] = the equilibration factor (sqrt of the diagonal / of the
 *          column norm).
 *   N < 0: rY = component sums of Y (= A^tY) (:715-723), rAA[ru][rv] =
 *          double component sums of A^tA (:724-741), same equilibration.
 *   N = 0: rY as above, rAA[rv] = component sums of the diagonal A (or the
 *          component sizes for the identity) (:744-759); Leq unused.
 *   rVc[rV + 1] = component offsets into Vc[V] (the CP's connected
 *   components, :571-597). */
#define CAT_(a, b) a##_##b
#define CAT(a, b) CAT_(a, b)
#define FN(name) CAT(name, SFX)

void FN(oracle_cp_reduce)(int N, int V, const REAL *A, const REAL *Y, int rV, const int *rVc,
                          const int *Vc, int preAt, REAL *rA, REAL *rAA, REAL *rY, REAL *Leq)
{
    int rv, ru, n, s, t, u, v, i;
    if (N > 0) {
        for (rv = 0; rv < rV; rv++) {  /* :676-687 */
            REAL *rAv = rA + (size_t)N * rv;
            for (n = 0; n < N; n++) rAv[n] = (REAL)0;
            for (s = rVc[rv], t = rVc[rv + 1]; s < t; s++) {
                const REAL *Av = A + (size_t)N * Vc[s];
                for (n = 0; n < N; n++) rAv[n] += Av[n];
            }
        }
        if (preAt) {
            for (ru = 0; ru < rV; ru++) {  /* :689-702 upper triangle */
                const REAL *Av = rA + (size_t)N * ru;
                REAL *rAv = rAA + (size_t)rV * ru;
                i = 0;
                for (rv = 0; rv <= ru; rv++) {
                    REAL a = (REAL)0;
                    for (n = 0; n < N; n++) a += rA[i++] * Av[n];
                    rAv[rv] = a;
                }
            }
            for (rv = 0; rv < rV; rv++) {  /* :704-711 */
                const REAL *rAv = rA + (size_t)N * rv;
                REAL a = (REAL)0;
                for (n = 0; n < N; n++) a += rAv[n] * Y[n];
                rY[rv] = a;
            }
        }
    } else {
        for (rv = 0; rv < rV; rv++) {  /* :715-723 */
            REAL a = (REAL)0;
            for (s = rVc[rv], t = rVc[rv + 1]; s < t; s++) a += Y[Vc[s]];
            rY[rv] = a;
        }
        if (N < 0) {  /* :724-741 upper triangle, u outer, v inner */
            for (ru = 0; ru < rV; ru++) {
                REAL *rAv = rAA + (size_t)rV * ru;
                for (rv = 0; rv <= ru; rv++) {
                    REAL a = (REAL)0;
                    for (s = rVc[ru], t = rVc[ru + 1]; s < t; s++) {
                        const REAL *Av = A + (size_t)V * Vc[s];
                        int q, r;
                        for (q = rVc[rv], r = rVc[rv + 1]; q < r; q++) a += Av[Vc[q]];
                    }
                    rAv[rv] = a;
                }
            }
        } else {  /* :744-759 */
            for (rv = 0; rv < rV; rv++) {
                if (A) {
                    REAL a = (REAL)0;
                    for (s = rVc[rv], t = rVc[rv + 1]; s < t; s++) a += A[Vc[s]];
                    rAA[rv] = a;
                } else {
                    rAA[rv] = (REAL)(rVc[rv + 1] - rVc[rv]);
                }
            }
        }
    }
    if ((preAt || N < 0) && N != 0) {  /* :761-770 lower triangle */
        for (ru = 0; ru < rV - 1; ru++) {
            REAL *rAv = rAA + (size_t)rV * ru;
            i = rV + (rV + 1) * ru;
            for (rv = ru + 1; rv < rV; rv++) { rAv[rv] = rAA[i]; i += rV; }
        }
    }
    if (N == 0) return;
    if (preAt || N < 0) {  /* :776-800 Jacobi equilibration of rAA, reverted */
        for (rv = 0; rv < rV; rv++) Leq[rv] = (REAL)sqrt(rAA[(size_t)rv * (rV + 1)]);
        for (ru = 0; ru < rV; ru++) {
            REAL *rAv = rAA + (size_t)rV * ru;
            const REAL a = Leq[ru];
            for (rv = 0; rv < rV; rv++) rAv[rv] /= (a * Leq[rv]);
        }
        for (ru = 0; ru < rV; ru++) {
            REAL *rAv = rAA + (size_t)rV * ru;
            const REAL a = Leq[ru];
            for (rv = 0; rv < rV; rv++) rAv[rv] *= (a * Leq[rv]);
        }
    } else {  /* :801-825 on rA */
        for (rv = 0; rv < rV; rv++) {
            const REAL *rAv = rA + (size_t)N * rv;
            REAL a = (REAL)0;
            for (n = 0; n < N; n++) { const REAL b = rAv[n]; a += b * b; }
            Leq[rv] = (REAL)sqrt(a);
        }
        for (rv = 0; rv < rV; rv++) {
            REAL *rAv = rA + (size_t)N * rv;
            const REAL a = Leq[rv];
            for (n = 0; n < N; n++) rAv[n] /= a;
        }
        for (rv = 0; rv < rV; rv++) {
            REAL *rAv = rA + (size_t)N * rv;
            const REAL a = Leq[rv];
            for (n = 0; n < N; n++) rAv[n] *= a;
        }
    }
    (void)u; (void)v;
}

#undef FN
#undef CAT
#undef CAT_
