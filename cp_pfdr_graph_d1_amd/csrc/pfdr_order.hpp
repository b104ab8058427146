// Locality reordering of scattered vertex labels (pfdr_order.hip).
#pragma once
#include "pfdr_graph.hpp"

namespace pfdr {

// True when the labels look random: V >= 2^20 and more than a quarter of
// the edges join labels more than V/64 apart.
bool labels_scattered(const int *Eu, const int *Ev, long E, int V, hipStream_t s);

// Deterministic breadth-first order of the vertices (level by level from
// the smallest unvisited label; within a level by the first discovering
// position, then label).  order[new] = old, where[old] = new.  Returns
// false (no order) for path-like graphs with more than max_levels levels.
bool bfs_order(const int *Eu, const int *Ev, long E, int V, DevBuf<int> &order,
               DevBuf<int> &where, hipStream_t s, int max_levels = 20000);

}  // namespace pfdr
