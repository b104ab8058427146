/* ==========================================================================
 * TEST INFRASTRUCTURE ONLY — CPU oracle for the MI355X PFDR build.
 *
 * Plain C (gcc) restatement of the reference PFDR solvers
 * (ai3DVision/CP_PFDR_graph_d1 src/PFDR_graph_quadratic_d1_l1.cpp,
 *  src/PFDR_graph_quadratic_d1_bounds.cpp, src/PFDR_graph_loss_d1_simplex.cpp,
 *  src/proj_simplex_metric.cpp), single-threaded, instantiated for float and
 * double.  Built by oracle/Makefile into oracle/liboracle_pfdr.so and loaded
 * by oracle/oracle.py.  Exported entry points:
 *     oracle_pfdr_quadratic_d1_l1_{f32,f64}
 *     oracle_pfdr_quadratic_d1_bounds_{f32,f64}
 *     oracle_pfdr_loss_d1_simplex_{f32,f64}
 *     oracle_proj_simplex_metric_{f32,f64}
 *     oracle_cp_reduce_{f32,f64}   (cp_reduce_body.h: the CP reduced-problem
 *                                   builder)
 *     oracle_cp_components, oracle_cp_activate, oracle_cp_reduced_graph_*,
 *     oracle_cp_merge_*, oracle_cp_gradient_*, oracle_cp_capacities_*
 *                                  (cp_graph_body.h: the CP graph steps,
 *                                   SURVEY.md §8(f) ranks 2-3)
 * Argument lists follow the reference functions (Lipschtype passed as int,
 * no verbose flag).  Parity pinned against the reference itself: see the
 * header of pfdr_oracle_body.h.
 * ======================================================================== */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define REAL float
#define SFX f32
#define ORACLE_EPS FLT_EPSILON
#define ORACLE_HUGE HUGE_VALF
/* the reference calls the C double log() on float operands (global ::log
 * from <cmath>), so the float objective accumulates a double product */
#define ORACLE_LOG log
#include "pfdr_oracle_body.h"
#include "cp_reduce_body.h"
#include "cp_graph_body.h"
#undef REAL
#undef SFX
#undef ORACLE_EPS
#undef ORACLE_HUGE
#undef ORACLE_LOG

#define REAL double
#define SFX f64
#define ORACLE_EPS DBL_EPSILON
#define ORACLE_HUGE HUGE_VAL
#define ORACLE_LOG log
#include "pfdr_oracle_body.h"
#include "cp_reduce_body.h"
#include "cp_graph_body.h"
#undef REAL
#undef SFX
#undef ORACLE_EPS
#undef ORACLE_HUGE
#undef ORACLE_LOG
