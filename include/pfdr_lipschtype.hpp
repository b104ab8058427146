/* Lipschitz information type of the quadratic PFDR solvers.  Same spelling
 * as the reference (include/PFDR_graph_quadratic_d1_l1.hpp:34): a
 * typedef-named anonymous enum, so that it mangles as `10Lipschtype` and the
 * drop-in symbols match the reference's exactly.  Guarded once here, so the
 * l1 and bounds declarations can share a translation unit (the reference
 * headers cannot: both define it). */
#ifndef PFDR_LIPSCHTYPE_HPP
#define PFDR_LIPSCHTYPE_HPP
typedef enum {SCAL, DIAG} Lipschtype;
#endif
