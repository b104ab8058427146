// Vertex -> incidence CSR (see pfdr_graph.hip).
#pragma once
#include "pfdr_dev.hpp"

namespace pfdr {

struct Incidence {
    int V = 0;          // vertices with a row
    long n = 0;         // incidence slots (2E, plus received halo slots)
    DevBuf<int> ptr;    // V + 1 row offsets
    DevBuf<unsigned> idx;  // slot ids, sorted by (vertex, e, side)
};

// Throws std::runtime_error unless every endpoint lies in [0, V).
void check_endpoints(const int *dEu, const int *dEv, long E, int V, hipStream_t s);

// Build the CSR (validates the endpoints first) of the 2E slots of edges (Eu, Ev) over vertices [0, V).
void build_incidence(const int *dEu, const int *dEv, int V, long E,
                     Incidence &inc, hipStream_t s);

// Keyed CSR (quadratic solvers): n entries, key = (row << 32) | order
// (order = 2 e_global + side, the reference's summation order), value =
// address of the entry's contribution; rows >= V are dropped.  keys/vals
// are consumed (sorted out of place, then may be freed).
void build_incidence_keyed(unsigned long long *keys, unsigned *vals, long n, int V,
                           Incidence &inc, hipStream_t s);

// Same CSR when the n entries are already listed in summation order:
// rows[i] (rows >= V set to V, dropped) stably sorted into srows.
void build_incidence_rows(const unsigned *rows, unsigned *srows, const unsigned *vals, long n,
                          int V, Incidence &inc, hipStream_t s);

// Row offsets ptr[0..V] of n keys sorted by row (row = key >> 32).
void keyed_rows(const unsigned long long *skey, long n, int V, int *ptr, hipStream_t s);

// out[g] = ((0 + x[off[g]]) + x[off[g] + 1]) + ... over [off[g], off[g+1]),
// x[i] = val[idx[i]] (idx may be null: val[i]), each sum in that exact
// order (pfdr_cpgraph.hip: one lane per short segment, one LDS-staged
// workgroup per long one).  Synchronises the stream.
template <typename real>
void ordered_segment_sums(int G, const int *off, const int *idx, const real *val, real *out,
                          hipStream_t s);

}  // namespace pfdr
