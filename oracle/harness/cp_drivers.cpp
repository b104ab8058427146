/* TEST INFRASTRUCTURE ONLY.  A command-line driver of the REFERENCE's four
 * cut-pursuit solvers, compiled from the reference sources by
 * oracle/Makefile once per CP source and per PFDR provider:
 *   _ref/cp_<kind>_ref     CP + the reference PFDR objects (CPU)
 *   _ref/cp_<kind>_mi355x  CP + libpfdr_mi355x.so (the drop-in, GPU)
 * with <kind> = l1 (src/CP_PFDR_graph_quadratic_d1_l1.cpp, -DCP_KIND=0),
 * duplex (src/CP_PFDR_graph_quadratic_d1_l1_duplex.cpp, 1), bounds
 * (src/CP_PFDR_graph_quadratic_d1_bounds.cpp, 2) and simplex
 * (src/CP_PFDR_graph_loss_d1_simplex.cpp, 3).  The CP object code is the
 * same in both binaries of a kind: the "CP callers link unchanged" check.
 *
 * Declarations follow include/CP_PFDR_graph_quadratic_d1_l1.hpp:52-61 and
 * :133-142, include/CP_PFDR_graph_quadratic_d1_bounds.hpp:55-63,
 * include/CP_PFDR_graph_loss_d1_simplex.hpp:40-47.
 *
 * Determinism: the reference's operator_norm_matrix seeds its power method
 * with time(NULL) + thread (src/operator_norm_matrix.cpp:182), so two CP runs
 * with N != 0 would start the power method differently.  This harness
 * defines time() to return a constant, so both binaries of a kind (run on
 * the same host, same thread count) compute the same Lipschitz constants
 * and differ only through PFDR.
 *
 * usage: cp_<kind> in.bin out.bin
 *   in : int32  kind, V, E, N, K, dtype (0 f32, 1 f64), CP_itMax, PFDR_itMax,
 *               positivity, flags (1: A given, 2: La_l1 given)
 *        float64 CP_difTol, PFDR_difTol, rho, condMin, PFDR_difRcd, min, max, al
 *        real Y[len] (simplex: Q[K V]; N > 0: Y[N]; else A^t Y [V])
 *        real A[...] if flags & 1 (N > 0: N V; N < 0: V V; N = 0: V)
 *        int32 Eu[E], Ev[E]; real La_d1[E]; real La_l1[V] if flags & 2
 *   out: int32 rV, CP_it; int32 Cv[V]; real rX[rV] (simplex: rP[K rV])
 * stderr: cp_time_s=... rV=... CP_it=... */
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <vector>

#ifndef CP_KIND
#define CP_KIND 0
#endif
#if CP_KIND == 0 || CP_KIND == 1
#include "CP_PFDR_graph_quadratic_d1_l1.hpp"
#elif CP_KIND == 2
#include "CP_PFDR_graph_quadratic_d1_bounds.hpp"
#else
#include "CP_PFDR_graph_loss_d1_simplex.hpp"
#endif

extern "C" time_t time(time_t *t) {
    if (t) *t = (time_t)1;
    return (time_t)1;
}

template <typename T>
static std::vector<T> rd(FILE *f, size_t n) {
    std::vector<T> v(n);
    if (n && fread(v.data(), sizeof(T), n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
    return v;
}

template <typename real>
static int run(FILE *f, FILE *o, const int *h, const double *d) {
    const int kind = h[0], V = h[1], E = h[2], N = h[3], K = h[4];
    const int CP_itMax = h[6], PFDR_itMax = h[7], pos = h[8], flags = h[9];
    if (kind != CP_KIND) { fprintf(stderr, "problem kind %d, driver kind %d\n", kind, CP_KIND); return 2; }
    const size_t ny = kind == 3 ? (size_t)K * V : (N > 0 ? (size_t)N : (size_t)V);
    const size_t na = N > 0 ? (size_t)N * V : (N < 0 ? (size_t)V * V : (size_t)V);
    std::vector<real> Y = rd<real>(f, ny);
    std::vector<real> A = (flags & 1) ? rd<real>(f, na) : std::vector<real>();
    std::vector<int> Eu = rd<int>(f, E), Ev = rd<int>(f, E);
    std::vector<real> Ld = rd<real>(f, E);
    std::vector<real> Ll = (flags & 2) ? rd<real>(f, V) : std::vector<real>();
    const real *Ap = (flags & 1) ? A.data() : NULL;
    const real *Llp = (flags & 2) ? Ll.data() : NULL;
    (void)Ap; (void)Llp; (void)pos;
    int rV = 0, CP_it = 0;
    std::vector<int> Cv(V);
    real *rX = NULL;
    const real CP_difTol = (real)d[0], PFDR_difTol = (real)d[1], rho = (real)d[2];
    const real condMin = (real)d[3], difRcd = (real)d[4];
    const auto t0 = std::chrono::steady_clock::now();
#if CP_KIND == 0
    CP_PFDR_graph_quadratic_d1_l1<real>(V, E, N, &rV, Cv.data(), &rX, Y.data(), Ap,
        Eu.data(), Ev.data(), Ld.data(), Llp, pos, CP_difTol, CP_itMax, &CP_it,
        rho, condMin, difRcd, PFDR_difTol, PFDR_itMax, NULL, NULL, NULL, 0, NULL);
#elif CP_KIND == 1
    CP_PFDR_graph_quadratic_d1_l1_duplex<real>(V, E, N, &rV, Cv.data(), &rX, Y.data(), Ap,
        Eu.data(), Ev.data(), Ld.data(), Llp, pos, CP_difTol, CP_itMax, &CP_it,
        rho, condMin, difRcd, PFDR_difTol, PFDR_itMax, NULL, NULL, NULL, 0, NULL);
#elif CP_KIND == 2
    const real lo = std::isinf(d[5]) ? (d[5] < 0 ? -(real)HUGE_VAL : (real)HUGE_VAL) : (real)d[5];
    const real hi = std::isinf(d[6]) ? (d[6] < 0 ? -(real)HUGE_VAL : (real)HUGE_VAL) : (real)d[6];
    CP_PFDR_graph_quadratic_d1_bounds<real>(V, E, N, &rV, Cv.data(), &rX, Y.data(), Ap,
        Eu.data(), Ev.data(), Ld.data(), lo, hi, CP_difTol, CP_itMax, &CP_it,
        rho, condMin, difRcd, PFDR_difTol, PFDR_itMax, NULL, NULL, NULL, 0, NULL);
#else
    CP_PFDR_graph_loss_d1_simplex<real>(K, V, E, (real)d[7], &rV, Cv.data(), &rX, Y.data(),
        Eu.data(), Ev.data(), Ld.data(), CP_difTol, CP_itMax, &CP_it,
        rho, condMin, difRcd, PFDR_difTol, PFDR_itMax, NULL, NULL, NULL, 0, NULL);
#endif
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr, "cp_time_s=%.6f rV=%d CP_it=%d\n", el, rV, CP_it);
    fwrite(&rV, 4, 1, o);
    fwrite(&CP_it, 4, 1, o);
    fwrite(Cv.data(), 4, V, o);
    fwrite(rX, sizeof(real), (size_t)rV * (kind == 3 ? K : 1), o);
    free(rX);
    return 0;
}

int main(int argc, char **argv) {
    if (argc != 3) { fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb"), *o = fopen(argv[2], "wb");
    if (!f || !o) { perror("open"); return 2; }
    std::vector<int> h = rd<int>(f, 10);
    std::vector<double> d = rd<double>(f, 8);
    int r = h[5] ? run<double>(f, o, h.data(), d.data()) : run<float>(f, o, h.data(), d.data());
    fclose(f);
    fclose(o);
    return r;
}
