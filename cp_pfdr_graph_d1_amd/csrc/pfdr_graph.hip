// Graph-side setup of the MI355X PFDR library:
//
//  * the vertex -> incidence CSR that turns the reference's serial
//    Douglas-Rachford scatter (src/PFDR_graph_quadratic_d1_l1.cpp:491-497,
//    bounds :464-470, simplex src/PFDR_graph_loss_d1_simplex.cpp:636-648)
//    and the serial preconditioning scatter (:156-192) into an atomic-free,
//    deterministic segmented gather.  Incidence slot s = 2e + side
//    (side 0 = Eu end, 1 = Ev end).  Per vertex the slots are sorted by
//    (e, side): exactly the order in which the reference adds them, so each
//    per-vertex sum rounds identically to the reference.  Built with a
//    stable LSD radix sort (rocPRIM) keyed by vertex.
//  * deterministic host-side synthetic generators (splitmix64), the native
//    twins of cp_pfdr_graph_d1_amd/graphs.py.

#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <stdexcept>
#include <vector>

#include "pfdr_graph.hpp"
#include "pfdr_sort.hpp"

namespace pfdr {

// min / max of the endpoints (validated before any gather kernel runs)
__global__ void k_endpoint_range(const int *__restrict__ Eu,
                                 const int *__restrict__ Ev, long E,
                                 int *__restrict__ mm) {
    __shared__ int lo[kBlock / kWave], hi[kBlock / kWave];
    long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    int a = 0x7fffffff, b = -0x7fffffff - 1;
    for (; e < E; e += (long)gridDim.x * blockDim.x) {
        const int u = Eu[e], v = Ev[e];
        a = min(a, min(u, v));
        b = max(b, max(u, v));
    }
    for (int o = 32; o > 0; o >>= 1) {
        a = min(a, __shfl_xor(a, o, 64));
        b = max(b, __shfl_xor(b, o, 64));
    }
    if ((threadIdx.x & 63) == 0) { lo[threadIdx.x >> 6] = a; hi[threadIdx.x >> 6] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < kBlock / kWave; i++) { a = min(a, lo[i]); b = max(b, hi[i]); }
        atomicMin(&mm[0], a);
        atomicMax(&mm[1], b);
    }
}

void check_endpoints(const int *dEu, const int *dEv, long E, int V, hipStream_t s) {
    if (E <= 0) return;
    DevBuf<int> mm(2);
    int init[2] = {0x7fffffff, -0x7fffffff - 1};
    PFDR_HIP(hipMemcpyAsync(mm.p, init, sizeof init, hipMemcpyHostToDevice, s));
    const int g = std::min(grid_for(E), 2048);
    k_endpoint_range<<<g, kBlock, 0, s>>>(dEu, dEv, E, mm.p);
    PFDR_HIP(hipGetLastError());
    int h[2];
    PFDR_HIP(hipMemcpyAsync(h, mm.p, sizeof h, hipMemcpyDeviceToHost, s));
    PFDR_HIP(hipStreamSynchronize(s));
    if (h[0] < 0 || h[1] >= V) {
        char msg[160];
        snprintf(msg, sizeof msg, "edge endpoints must lie in [0, %d): found [%d, %d]", V, h[0], h[1]);
        throw std::runtime_error(msg);
    }
}

// key[s] = endpoint of slot s, val[s] = s
__global__ void k_incidence_keys(const int *__restrict__ Eu,
                                 const int *__restrict__ Ev, long E,
                                 unsigned *__restrict__ key,
                                 unsigned *__restrict__ val) {
    long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    key[2 * e] = (unsigned)Eu[e];
    key[2 * e + 1] = (unsigned)Ev[e];
    val[2 * e] = (unsigned)(2 * e);
    val[2 * e + 1] = (unsigned)(2 * e + 1);
}

// ptr[v] = first sorted position whose key is >= v, ptr[V] = n: position i
// starts every vertex in (key[i-1], key[i]] (key[-1] = -1, key[n] = V)
__global__ void k_incidence_ptr(const unsigned *__restrict__ skey, long n,
                                int V, int *__restrict__ ptr) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    long kp = (i == 0) ? -1 : (long)skey[i - 1];
    long kc = (i == n) ? (long)V : (long)skey[i];
    for (long v = kp + 1; v <= kc; v++) ptr[v] = (int)i;
}

void build_incidence(const int *dEu, const int *dEv, int V, long E,
                     Incidence &inc, hipStream_t s) {
    const long n = 2 * E;
    inc.V = V;
    inc.n = n;
    inc.ptr.alloc((size_t)V + 1);
    inc.idx.alloc((size_t)(n > 0 ? n : 1));
    if (n == 0) {
        PFDR_HIP(hipMemsetAsync(inc.ptr.p, 0, sizeof(int) * (V + 1), s));
        return;
    }
    check_endpoints(dEu, dEv, E, V, s);
    DevBuf<unsigned> key(n), val(n), skey(n);
    k_incidence_keys<<<grid_for(E), kBlock, 0, s>>>(dEu, dEv, E, key.p, val.p);
    PFDR_HIP(hipGetLastError());
    unsigned bits = 1;
    while (bits < 32 && ((1ull << bits) < (unsigned long long)V)) bits++;
    radix_sort_pairs_stable<unsigned>(key.p, skey.p, val.p, inc.idx.p, n, (int)bits, s);
    k_incidence_ptr<<<grid_for(n + 1), kBlock, 0, s>>>(skey.p, n, V,
                                                       inc.ptr.p);
    PFDR_HIP(hipGetLastError());
    // temporaries freed at scope exit: dev_free reuses them only once the
    // stream is idle (or synchronises before a real hipFree)
}

// CSR from rows listed in the wanted order within each row: stable radix
// sort over the row bits (rows >= V were set to V and sort last)
void build_incidence_rows(const unsigned *rows, unsigned *srows, const unsigned *vals, long n,
                          int V, Incidence &inc, hipStream_t s) {
    inc.V = V;
    inc.n = n;
    inc.ptr.alloc((size_t)V + 1);
    inc.idx.alloc((size_t)(n > 0 ? n : 1));
    unsigned bits = 1;
    while (bits < 32 && ((1ull << bits) <= (unsigned long long)V)) bits++;
    radix_sort_pairs_stable<unsigned>(rows, srows, vals, inc.idx.p, n, (int)bits, s);
    k_incidence_ptr<<<grid_for(n + 1), kBlock, 0, s>>>(srows, n, V, inc.ptr.p);
    PFDR_HIP(hipGetLastError());  // temporaries: see build_incidence
}

// Keyed CSR: entry i has key = (row << 32) | order and value = address of
// its contribution.  Rows >= V (non-owned slots, key ~0) sort last and are
// ignored.  ptr[v] = first sorted position of row v.
__global__ void k_keyed_ptr(const unsigned long long *__restrict__ skey, long n, int V,
                            int *__restrict__ ptr) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    long kp = (i == 0) ? -1 : (long)min((unsigned long long)V, skey[i - 1] >> 32);
    long kc = (i == n) ? (long)V : (long)min((unsigned long long)V, skey[i] >> 32);
    for (long v = kp + 1; v <= kc; v++) ptr[v] = (int)i;
}

void keyed_rows(const unsigned long long *skey, long n, int V, int *ptr, hipStream_t s) {
    k_keyed_ptr<<<grid_for(n + 1), kBlock, 0, s>>>(skey, n, V, ptr);
    PFDR_HIP(hipGetLastError());
}

void build_incidence_keyed(unsigned long long *keys, unsigned *vals, long n, int V,
                           Incidence &inc, hipStream_t s) {
    inc.V = V;
    inc.n = n;
    inc.ptr.alloc((size_t)V + 1);
    inc.idx.alloc((size_t)(n > 0 ? n : 1));
    if (n == 0) {
        PFDR_HIP(hipMemsetAsync(inc.ptr.p, 0, sizeof(int) * (V + 1), s));
        return;
    }
    unsigned vbits = 1;
    while (vbits < 31 && ((1ull << vbits) <= (unsigned long long)V)) vbits++;
    DevBuf<unsigned long long> skey(n);
    radix_sort_pairs_stable<unsigned long long>(keys, skey.p, vals, inc.idx.p, n,
                                                (int)(32 + vbits + 1), s);
    k_keyed_ptr<<<grid_for(n + 1), kBlock, 0, s>>>(skey.p, n, V, inc.ptr.p);
    PFDR_HIP(hipGetLastError());  // temporaries: see build_incidence
}

}  // namespace pfdr

// ===================================================================== //
//                      host-side synthetic generators                   //
// ===================================================================== //
namespace {

inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// U[0,1) for counter i of stream seed (graphs.py: uniform)
inline double uniform(uint64_t seed, uint64_t i) {
    uint64_t x = seed * 0xD1B54A32D192ED03ull + i;
    return (double)(splitmix64(x) >> 11) * 0x1.0p-53;
}

struct Pt { double x, y, z; };

// static-schedule parallel for over [b, e) on the host's cores
template <typename F>
void host_parallel_for(int64_t b, int64_t e, F f) {
    const int64_t n = e - b;
    int nt = (int)std::min<int64_t>(std::max(1u, std::thread::hardware_concurrency()), 64);
    if (n < 4096) nt = 1;
    nt = (int)std::min<int64_t>(nt, std::max<int64_t>(n, 1));
    std::vector<std::thread> th;
    const int64_t per = (n + nt - 1) / nt;
    for (int t = 0; t < nt; t++) {
        const int64_t lo = b + t * per, hi = std::min(e, lo + per);
        if (lo >= hi) break;
        th.emplace_back([=] { for (int64_t v = lo; v < hi; v++) f(v); });
    }
    for (auto &x : th) x.join();
}

inline Pt jitter_point(uint64_t seed, double jit, int64_t v, int64_t x,
                       int64_t y, int64_t z) {
    uint64_t b = 3ull * (uint64_t)v;
    return {x + (2.0 * uniform(seed, b) - 1.0) * jit,
            y + (2.0 * uniform(seed, b + 1) - 1.0) * jit,
            z + (2.0 * uniform(seed, b + 2) - 1.0) * jit};
}

}  // namespace

extern "C" int64_t pfdr_gen_knn_jitter_grid(int nx, int ny, int nz, int k,
                                            uint64_t seed, double jitter,
                                            int64_t v_begin, int64_t v_end,
                                            int *Eu, int *Ev) {
    if (k < 1 || k > 26 || nx < 1 || ny < 1 || nz < 1) return -1;
    const int64_t V = (int64_t)nx * ny * nz;
    if (v_begin < 0 || v_end > V || v_begin > v_end) return -1;
    // neighbour enumeration order dz, dy, dx ascending (graphs.py: _nbr26)
    int off[26][3];
    int m = 0;
    for (int dz = -1; dz <= 1; dz++)
        for (int dy = -1; dy <= 1; dy++)
            for (int dx = -1; dx <= 1; dx++)
                if (dx || dy || dz) { off[m][0] = dx; off[m][1] = dy; off[m][2] = dz; m++; }
    host_parallel_for(v_begin, v_end, [&](int64_t v) {
        int64_t x = v % nx, y = (v / nx) % ny, z = v / ((int64_t)nx * ny);
        Pt p = jitter_point(seed, jitter, v, x, y, z);
        double d[26];
        int64_t w[26];
        for (int j = 0; j < 26; j++) {
            int64_t xx = x + off[j][0], yy = y + off[j][1], zz = z + off[j][2];
            bool ok = xx >= 0 && xx < nx && yy >= 0 && yy < ny && zz >= 0 && zz < nz;
            w[j] = xx + nx * (yy + (int64_t)ny * zz);
            if (ok) {
                Pt q = jitter_point(seed, jitter, w[j], xx, yy, zz);
                d[j] = (p.x - q.x) * (p.x - q.x) + (p.y - q.y) * (p.y - q.y) +
                       (p.z - q.z) * (p.z - q.z);
            } else {
                d[j] = HUGE_VAL;
            }
        }
        // stable selection of the k smallest (ties: enumeration order)
        int order[26];
        for (int j = 0; j < 26; j++) order[j] = j;
        for (int i = 1; i < 26; i++) {  // stable insertion sort
            int oj = order[i];
            int t = i - 1;
            while (t >= 0 && d[order[t]] > d[oj]) { order[t + 1] = order[t]; t--; }
            order[t + 1] = oj;
        }
        int64_t base = (v - v_begin) * k;
        for (int j = 0; j < k; j++) {
            Eu[base + j] = (int)v;
            Ev[base + j] = (int)w[order[j]];
        }
    });
    return (v_end - v_begin) * (int64_t)k;
}

extern "C" int64_t pfdr_gen_grid_edges(int nx, int ny, int nz, int conn,
                                       int64_t v_begin, int64_t v_end,
                                       int *Eu, int *Ev) {
    // same enumeration as graphs.py: _offsets / grid_graph
    int off[13][3];
    int m = 0;
    const bool is3d = nz > 1 || conn == 6 || conn == 26;
    if (!is3d && conn == 4) {
        int o[2][3] = {{1, 0, 0}, {0, 1, 0}};
        m = 2; memcpy(off, o, sizeof(o));
    } else if (!is3d && conn == 8) {
        int o[4][3] = {{1, 0, 0}, {0, 1, 0}, {1, 1, 0}, {-1, 1, 0}};
        m = 4; memcpy(off, o, sizeof(o));
    } else if (is3d && conn == 6) {
        int o[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
        m = 3; memcpy(off, o, sizeof(o));
    } else if (is3d && conn == 26) {
        for (int dz = -1; dz <= 1; dz++)
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    bool pos = dz > 0 || (dz == 0 && (dy > 0 || (dy == 0 && dx > 0)));
                    if (pos) { off[m][0] = dx; off[m][1] = dy; off[m][2] = dz; m++; }
                }
    } else {
        return -1;
    }
    int64_t cnt = 0;
    for (int64_t v = v_begin; v < v_end; v++) {
        int64_t x = v % nx, y = (v / nx) % ny, z = v / ((int64_t)nx * ny);
        for (int j = 0; j < m; j++) {
            int64_t xx = x + off[j][0], yy = y + off[j][1], zz = z + off[j][2];
            if (xx < 0 || xx >= nx || yy < 0 || yy >= ny || zz < 0 || zz >= nz)
                continue;
            if (Eu) {
                Eu[cnt] = (int)v;
                Ev[cnt] = (int)(xx + nx * (yy + (int64_t)ny * zz));
            }
            cnt++;
        }
    }
    return cnt;
}

template <typename T>
static int gen_piecewise(int nx, uint64_t seed, double noise, int64_t v0,
                         int64_t v1, T *Y) {
    host_parallel_for(v0, v1, [&](int64_t v) {
        double base = ((v % nx) < nx / 2) ? 1.0 : -0.5;
        Y[v - v0] = (T)(base + (2.0 * uniform(seed, (uint64_t)v) - 1.0) * noise);
    });
    return 0;
}

extern "C" int pfdr_gen_piecewise_f32(int nx, uint64_t seed, double noise,
                                      int64_t v0, int64_t v1, float *Y) {
    return gen_piecewise(nx, seed, noise, v0, v1, Y);
}
extern "C" int pfdr_gen_piecewise_f64(int nx, uint64_t seed, double noise,
                                      int64_t v0, int64_t v1, double *Y) {
    return gen_piecewise(nx, seed, noise, v0, v1, Y);
}

// out[i] = lo + (hi - lo) * U(seed, i0 + i), rounded once from double:
// the dense matrices of C3 (A ~ U(-h, h)) reproducible on any host
template <typename T>
static int gen_uniform(uint64_t seed, int64_t i0, int64_t n, double lo, double hi, T *out) {
    if (n < 0 || !out) return -1;
    host_parallel_for(0, n, [&](int64_t i) {
        out[i] = (T)(lo + (hi - lo) * uniform(seed, (uint64_t)(i0 + i)));
    });
    return 0;
}
extern "C" int pfdr_gen_uniform_f32(uint64_t seed, int64_t i0, int64_t n, double lo,
                                    double hi, float *out) {
    return gen_uniform(seed, i0, n, lo, hi, out);
}
extern "C" int pfdr_gen_uniform_f64(uint64_t seed, int64_t i0, int64_t n, double lo,
                                    double hi, double *out) {
    return gen_uniform(seed, i0, n, lo, hi, out);
}

// y[n] = sum_v A[n + N v] x[v] for the column-major N-by-V matrix A, each
// row accumulated in double in increasing v (so the result does not depend
// on the thread count or the host), rounded once: the observations Y = A x0
// of C3.  Threads own row ranges and walk v outermost (contiguous columns).
template <typename T>
static int gen_matvec(int64_t N, int64_t V, const T *A, const T *x, T *y) {
    if (N <= 0 || V < 0 || !A || !x || !y) return -1;
    const int64_t rows = 64;
    const int64_t nb = (N + rows - 1) / rows;
    host_parallel_for(0, nb, [&](int64_t b) {
        const int64_t n0 = b * rows, n1 = std::min(N, n0 + rows);
        double acc[rows];
        for (int64_t n = n0; n < n1; n++) acc[n - n0] = 0.0;
        for (int64_t v = 0; v < V; v++) {
            const T *a = A + N * v;
            const double xv = (double)x[v];
            for (int64_t n = n0; n < n1; n++) acc[n - n0] += (double)a[n] * xv;
        }
        for (int64_t n = n0; n < n1; n++) y[n] = (T)acc[n - n0];
    });
    return 0;
}
extern "C" int pfdr_gen_matvec_f32(int64_t N, int64_t V, const float *A, const float *x,
                                   float *y) {
    return gen_matvec(N, V, A, x, y);
}
extern "C" int pfdr_gen_matvec_f64(int64_t N, int64_t V, const double *A, const double *x,
                                   double *y) {
    return gen_matvec(N, V, A, x, y);
}

// symmetric, diagonally dominant V-by-V matrix (an A^tA stand-in that any
// host reproduces bit for bit): off-diagonal (u, v) = s (2 U(seed, min V +
// max) - 1), diagonal d.  Column-major = row-major (symmetric).
template <typename T>
static int gen_symmetric(int64_t V, uint64_t seed, double s, double d, T *G) {
    if (V < 0 || !G) return -1;
    host_parallel_for(0, V, [&](int64_t v) {
        for (int64_t u = 0; u < V; u++) {
            const int64_t a = std::min(u, v), b = std::max(u, v);
            G[u + V * v] = u == v ? (T)d
                                  : (T)(s * (2.0 * uniform(seed, (uint64_t)(a * V + b)) - 1.0));
        }
    });
    return 0;
}
extern "C" int pfdr_gen_symmetric_f32(int64_t V, uint64_t seed, double s, double d, float *G) {
    return gen_symmetric(V, seed, s, d, G);
}
extern "C" int pfdr_gen_symmetric_f64(int64_t V, uint64_t seed, double s, double d, double *G) {
    return gen_symmetric(V, seed, s, d, G);
}
