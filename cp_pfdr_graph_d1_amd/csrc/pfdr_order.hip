// Locality reordering of a graph's vertices (randomly
// labelled k-NN graphs).  The reference iterates in the caller's labels;
// with random labels every gather of the edge and vertex sweeps misses the
// caches (headline graph shuffled: 4.8 ms/iteration instead of 0.9).  The
// session therefore relabels internally, when the labels are scattered, by a
// breadth-first order: a vertex's neighbours lie within one BFS level of it,
// so its gathers stay inside a window of about two levels.
//
// The order is deterministic: within a level, vertices are sorted by the
// smallest position of a discovering vertex, then by label (atomics only
// compute minima; candidates are sorted).  Nothing numerical depends on it
// — the session keeps the reference's per-vertex summation order (original
// edge ids in the incidence keys) and sums the amplitude in original vertex
// order — so results are bit-identical with and without reordering.
#include <climits>
#include <cstring>
#include <vector>
#include <rocprim/rocprim.hpp>

#include "pfdr_order.hpp"

namespace pfdr {

__global__ void k_far_edges(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                            long thr, unsigned long long *cnt) {
    __shared__ unsigned long long red[kBlock / kWave];
    unsigned long long c = 0;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < E;
         e += (long)gridDim.x * blockDim.x) {
        const long d = (long)Eu[e] - (long)Ev[e];
        c += (d > thr || d < -thr) ? 1 : 0;
    }
    c = block_sum(c, red);
    if (threadIdx.x == 0) atomicAdd(cnt, c);
}

bool labels_scattered(const int *Eu, const int *Ev, long E, int V, hipStream_t s) {
    if (V < (1 << 20) || E < V) return false;
    DevBuf<unsigned long long> cnt(1);
    PFDR_HIP(hipMemsetAsync(cnt.p, 0, 8, s));
    k_far_edges<<<1024, kBlock, 0, s>>>(E, Eu, Ev, V / 64, cnt.p);
    PFDR_HIP(hipGetLastError());
    unsigned long long h = 0;
    PFDR_HIP(hipMemcpyAsync(&h, cnt.p, 8, hipMemcpyDeviceToHost, s));
    PFDR_HIP(hipStreamSynchronize(s));
    return h > (unsigned long long)E / 4;  // a quarter of the edges span > V/64
}

// neighbour incidence: value a < E is the u end of edge a (neighbour Ev[a]),
// a >= E the v end of edge a - E (neighbour Eu[a - E])
__global__ void k_nbr_keys(long E, const int *__restrict__ Eu, const int *__restrict__ Ev,
                           unsigned long long *__restrict__ keys, unsigned *__restrict__ vals) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    keys[e] = ((unsigned long long)Eu[e] << 32) | (unsigned)e;
    keys[E + e] = ((unsigned long long)Ev[e] << 32) | (unsigned)e;
    vals[e] = (unsigned)Ev[e];
    vals[E + e] = (unsigned)Eu[e];
}

__global__ void k_bfs_init(int V, int *lvl, unsigned *pmin) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    lvl[v] = -1;
    pmin[v] = 0xffffffffu;
}

__global__ void k_bfs_root(int root, int pos, int L, int *lvl, int *order, int *where) {
    lvl[root] = L;
    order[pos] = root;
    where[root] = pos;
}

// expand the frontier order[f0, f1) (level L) into candidates of level L+1
__global__ void k_bfs_expand(int f0, int f1, const int *__restrict__ order,
                             const int *__restrict__ ptr, const unsigned *__restrict__ nbr,
                             int *lvl, int L, unsigned *pmin, int *cand, int *ncand) {
    const int q = f0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= f1) return;
    const int u = order[q];
    for (int j = ptr[u], j1 = ptr[u + 1]; j < j1; j++) {
        const int w = (int)nbr[j];
        const int lv = __hip_atomic_load(lvl + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lv != -1 && lv != L + 1) continue;
        atomicMin(pmin + w, (unsigned)q);
        if (lv == -1 && atomicCAS(lvl + w, -1, L + 1) == -1) cand[atomicAdd(ncand, 1)] = w;
    }
}

__global__ void k_cand_keys(int n, const int *__restrict__ cand, const unsigned *__restrict__ pmin,
                            unsigned long long *__restrict__ keys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int w = cand[i];
    keys[i] = ((unsigned long long)pmin[w] << 32) | (unsigned)w;
}

__global__ void k_place(int n, int base, const unsigned long long *__restrict__ keys,
                        int *order, int *where) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int w = (int)(keys[i] & 0xffffffffu);
    order[base + i] = w;
    where[w] = base + i;
}

__global__ void k_min_unvisited(int V, const int *__restrict__ lvl, int *out) {
    int m = INT_MAX;
    for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < V; v += gridDim.x * blockDim.x)
        if (lvl[v] == -1) { m = v; break; }  // first in this lane's stride
    if (m != INT_MAX) atomicMin(out, m);
}

__global__ void k_collect_unvisited(int V, const int *__restrict__ lvl, int *cand, int *ncand) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < V && lvl[v] == -1) cand[atomicAdd(ncand, 1)] = v;
}

__global__ void k_unvisited_keys(int n, const int *__restrict__ cand,
                                 unsigned long long *__restrict__ keys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keys[i] = (unsigned long long)(unsigned)cand[i];
}

bool bfs_order(const int *Eu, const int *Ev, long E, int V, DevBuf<int> &order,
               DevBuf<int> &where, hipStream_t s, int max_levels) {
    // symmetric neighbour CSR (rows sorted by vertex, then edge id)
    DevBuf<int> ptr(V + 1);
    DevBuf<unsigned> nbr(2 * E);
    {
        DevBuf<unsigned long long> keys(2 * E), skeys(2 * E);
        DevBuf<unsigned> vals(2 * E);
        k_nbr_keys<<<grid_for(E), kBlock, 0, s>>>(E, Eu, Ev, keys.p, vals.p);
        PFDR_HIP(hipGetLastError());
        unsigned vbits = 1;
        while (vbits < 31 && ((1ull << vbits) <= (unsigned long long)V)) vbits++;
        size_t tb = 0;
        PFDR_HIP(rocprim::radix_sort_pairs(nullptr, tb, keys.p, skeys.p, vals.p, nbr.p,
                                           (size_t)(2 * E), 0, 32 + vbits, s));
        DevBuf<char> tmp(tb ? tb : 1);
        PFDR_HIP(rocprim::radix_sort_pairs((void *)tmp.p, tb, keys.p, skeys.p, vals.p, nbr.p,
                                           (size_t)(2 * E), 0, 32 + vbits, s));
        keyed_rows(skeys.p, 2 * E, V, ptr.p, s);
    }
    order.alloc(V);
    where.alloc(V);
    DevBuf<int> lvl(V), cand(V), dev_int(2);
    DevBuf<unsigned> pmin(V);
    DevBuf<unsigned long long> ck(V), cks(V);
    size_t tb = 0;
    PFDR_HIP(rocprim::radix_sort_keys(nullptr, tb, ck.p, cks.p, (size_t)V, 0, 64, s));
    DevBuf<char> tmp(tb ? tb : 1);
    k_bfs_init<<<grid_for(V), kBlock, 0, s>>>(V, lvl.p, pmin.p);
    PFDR_HIP(hipGetLastError());
    int *h = static_cast<int *>(pinned_small_get());  // pinned: [count, root]
    struct Free {
        int *h;
        hipStream_t s;
        ~Free() { (void)hipStreamSynchronize(s); pinned_small_put(h); }
    } fr{h, s};
    int placed = 0, L = 0, roots = 0, levels = 0;
    auto sort_place = [&](int n, int base) {
        size_t b = tb;
        PFDR_HIP(rocprim::radix_sort_keys((void *)tmp.p, b, ck.p, cks.p, (size_t)n, 0, 64, s));
        k_place<<<grid_for(n), kBlock, 0, s>>>(n, base, cks.p, order.p, where.p);
        PFDR_HIP(hipGetLastError());
    };
    while (placed < V) {
        if (roots < 64) {  // BFS from the smallest unvisited label
            h[1] = INT_MAX;
            PFDR_HIP(hipMemcpyAsync(dev_int.p + 1, h + 1, sizeof(int), hipMemcpyHostToDevice, s));
            k_min_unvisited<<<1024, kBlock, 0, s>>>(V, lvl.p, dev_int.p + 1);
            PFDR_HIP(hipMemcpyAsync(h + 1, dev_int.p + 1, sizeof(int), hipMemcpyDeviceToHost, s));
            PFDR_HIP(hipStreamSynchronize(s));
            const int root = h[1];
            if (root == INT_MAX) break;
            k_bfs_root<<<1, 1, 0, s>>>(root, placed, L, lvl.p, order.p, where.p);
            int f0 = placed, f1 = placed + 1;
            placed++;
            roots++;
            for (;;) {
                PFDR_HIP(hipMemsetAsync(dev_int.p, 0, sizeof(int), s));
                k_bfs_expand<<<grid_for(f1 - f0), kBlock, 0, s>>>(f0, f1, order.p, ptr.p, nbr.p,
                                                                   lvl.p, L, pmin.p, cand.p,
                                                                   dev_int.p);
                PFDR_HIP(hipGetLastError());
                PFDR_HIP(hipMemcpyAsync(h, dev_int.p, sizeof(int), hipMemcpyDeviceToHost, s));
                PFDR_HIP(hipStreamSynchronize(s));
                const int n = h[0];
                L++;
                if (n == 0) break;
                if (++levels > max_levels) return false;  // path-like: not worth it
                k_cand_keys<<<grid_for(n), kBlock, 0, s>>>(n, cand.p, pmin.p, ck.p);
                sort_place(n, f1);
                f0 = f1;
                f1 += n;
                placed += n;
            }
        } else {  // many components: the rest in label order
            PFDR_HIP(hipMemsetAsync(dev_int.p, 0, sizeof(int), s));
            k_collect_unvisited<<<grid_for(V), kBlock, 0, s>>>(V, lvl.p, cand.p, dev_int.p);
            PFDR_HIP(hipMemcpyAsync(h, dev_int.p, sizeof(int), hipMemcpyDeviceToHost, s));
            PFDR_HIP(hipStreamSynchronize(s));
            const int n = h[0];
            k_unvisited_keys<<<grid_for(n), kBlock, 0, s>>>(n, cand.p, ck.p);
            sort_place(n, placed);
            placed += n;
        }
    }
    PFDR_HIP(hipStreamSynchronize(s));
    return placed == V;
}

}  // namespace pfdr

extern "C" int pfdr_locality_order(int V, int64_t E, const int *Eu, const int *Ev, int mem,
                                   int *order_out, int *applied) {
    using namespace pfdr;
    if (V <= 0 || E < 0 || (E > 0 && (!Eu || !Ev)) || !order_out)
        return report_error("pfdr_locality_order", "invalid arguments");
    try {
        hipStream_t s = lib_stream();
        DevBuf<int> du(E ? E : 1), dv(E ? E : 1), order, where;
        const auto kind = mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
        if (E) {
            PFDR_HIP(hipMemcpyAsync(du.p, Eu, E * sizeof(int), kind, s));
            PFDR_HIP(hipMemcpyAsync(dv.p, Ev, E * sizeof(int), kind, s));
        }
        check_endpoints(du.p, dv.p, E, V, s);
        const bool ok = E > 0 && bfs_order(du.p, dv.p, E, V, order, where, s);
        if (!ok) {
            std::vector<int> id(V);
            for (int v = 0; v < V; v++) id[v] = v;
            PFDR_HIP(hipMemcpyAsync(order_out, id.data(), V * sizeof(int),
                                    mem == PFDR_MEM_DEVICE ? hipMemcpyHostToDevice
                                                           : hipMemcpyHostToHost, s));
        } else {
            PFDR_HIP(hipMemcpyAsync(order_out, order.p, V * sizeof(int),
                                    mem == PFDR_MEM_DEVICE ? hipMemcpyDeviceToDevice
                                                           : hipMemcpyDeviceToHost, s));
        }
        PFDR_HIP(hipStreamSynchronize(s));
        if (applied) *applied = ok ? 1 : 0;
    } catch (const HipError &h) {
        return report_error("pfdr_locality_order", h);
    } catch (const std::exception &ex) {
        return report_error("pfdr_locality_order", ex.what());
    }
    return PFDR_OK;
}
