/* TEST INFRASTRUCTURE ONLY.  A command-line driver of the REFERENCE's
 * cut-pursuit solver CP_PFDR_graph_quadratic_d1_l1<real>
 * (include/CP_PFDR_graph_quadratic_d1_l1.hpp:52-61), compiled from the
 * reference sources by oracle/Makefile twice:
 *   _ref/cp_driver_ref     CP + the reference PFDR objects (CPU, OpenMP)
 *   _ref/cp_driver_mi355x  CP + libpfdr_mi355x.so (the drop-in, GPU)
 * The CP sources are the same object code in both: this is the "CP callers
 * link unchanged" demonstration.
 * usage: cp_driver in.bin out.bin
 *   in : int32 V, E, dtype (0 f32, 1 f64), CP_itMax, PFDR_itMax, positivity,
 *        float64 CP_difTol, PFDR_difTol, rho, condMin,
 *        real Y[V], real A[V] (diagonal of A^tA), int32 Eu[E], Ev[E],
 *        real La_d1[E], real La_l1[V]
 *   out: int32 rV, CP_it, int32 Cv[V], real rX[rV]
 * stderr: the wall time of the CP call (cp_time_s=...) */
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "CP_PFDR_graph_quadratic_d1_l1.hpp"

template <typename T>
static std::vector<T> rd(FILE *f, size_t n) {
    std::vector<T> v(n);
    if (n && fread(v.data(), sizeof(T), n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
    return v;
}

template <typename real>
static int run(FILE *f, FILE *o, const int *h, const double *d) {
    const int V = h[0], E = h[1], CP_itMax = h[3], PFDR_itMax = h[4], pos = h[5];
    std::vector<real> Y = rd<real>(f, V), A = rd<real>(f, V);
    std::vector<int> Eu = rd<int>(f, E), Ev = rd<int>(f, E);
    std::vector<real> Ld = rd<real>(f, E), Ll = rd<real>(f, V);
    int rV = 0, CP_it = 0;
    std::vector<int> Cv(V);
    real *rX = NULL;
    const auto t0 = std::chrono::steady_clock::now();
    CP_PFDR_graph_quadratic_d1_l1<real>(V, E, 0, &rV, Cv.data(), &rX, Y.data(), A.data(),
        Eu.data(), Ev.data(), Ld.data(), Ll.data(), pos, (real)d[0], CP_itMax, &CP_it,
        (real)d[2], (real)d[3], (real)0, (real)d[1], PFDR_itMax, NULL, NULL, NULL, 0, NULL);
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr, "cp_time_s=%.6f rV=%d CP_it=%d\n", el, rV, CP_it);
    fwrite(&rV, 4, 1, o);
    fwrite(&CP_it, 4, 1, o);
    fwrite(Cv.data(), 4, V, o);
    fwrite(rX, sizeof(real), rV, o);
    free(rX);
    return 0;
}

int main(int argc, char **argv) {
    if (argc != 3) { fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb"), *o = fopen(argv[2], "wb");
    if (!f || !o) { perror("open"); return 2; }
    std::vector<int> h = rd<int>(f, 6);
    std::vector<double> d = rd<double>(f, 4);
    int r = h[2] ? run<double>(f, o, h.data(), d.data()) : run<float>(f, o, h.data(), d.data());
    fclose(f);
    fclose(o);
    return r;
}
