// Stable LSD radix sort of (key, value) pairs on the GPU: unsigned 32- or
// 64-bit keys, 32-bit values, the low `bits` bits of the key.
//
// Why not rocPRIM: its device radix sort instantiates ~300 kernels per key /
// value type pair (onesweep variants, block sorts, merge-sort fallbacks), so
// the translation unit that builds the incidence CSR carried ~880 kernels,
// and loading that code object cost ~45 ms of every process's first call
// (profiles/r2/r2s_first_call.md).  This sort is three small kernels per
// type.  Each pass sorts one 8-bit digit:
//   k_rs_hist     per tile of 4096 keys, the count of every digit
//                 (LDS atomics), written digit-major: hist[d * ntiles + t];
//   scan          exclusive scan of the counts: the first output position of
//                 digit d of tile t (every tile's keys of a digit land after
//                 the same digit's keys of earlier tiles: stability);
//   k_rs_scatter  each tile re-reads its keys in order (round j: elements
//                 j * 256 + lane), ranks every key among the equal digits
//                 before it in the tile -- within a wave by a match mask of 8
//                 ballots, across the 4 waves through LDS counts -- and
//                 writes key and value to their final positions.
// Keys beyond n belong to no digit.  Deterministic and stable, so the
// incidence lists come out in the order the reference adds them.
#pragma once

#include "pfdr_dev.hpp"

namespace pfdr {

// kin / vin are not modified; kout / vout receive the sorted pairs; n < 2^31.
template <typename K>
void radix_sort_pairs_stable(const K *kin, K *kout, const unsigned *vin, unsigned *vout, long n,
                             int bits, hipStream_t s);

}  // namespace pfdr
