/* ==========================================================================
 * pfdr_mi355x.h — C ABI of the MI355X-native PFDR solvers (libpfdr_mi355x.so)
 *
 * Plain C, fixed-width scalars, plain pointers and sizes; no C++ or torch
 * types.  Two layers:
 *
 *  1. Drop-in entry points.  Same argument list and meaning as the reference
 *     C++ templates they replace, host pointers, synchronous (device work is
 *     finished and every output copied back before return), status return
 *     instead of void.  The C++ drop-in symbols
 *     (include/PFDR_graph_quadratic_d1_l1.hpp etc.) forward to these.
 *       pfdr_quadratic_d1_l1_{f32,f64}
 *           replaces PFDR_graph_quadratic_d1_l1<real>
 *           (reference include/PFDR_graph_quadratic_d1_l1.hpp:36-42,
 *            src/PFDR_graph_quadratic_d1_l1.cpp:270-553)
 *       pfdr_quadratic_d1_bounds_{f32,f64}
 *           replaces PFDR_graph_quadratic_d1_bounds<real>
 *           (reference include/PFDR_graph_quadratic_d1_bounds.hpp:34-40,
 *            src/PFDR_graph_quadratic_d1_bounds.cpp:244-530)
 *       pfdr_loss_d1_simplex_{f32,f64}
 *           replaces PFDR_graph_loss_d1_simplex<real>
 *           (reference include/PFDR_graph_loss_d1_simplex.hpp:24-30,
 *            src/PFDR_graph_loss_d1_simplex.cpp:372-715)
 *       pfdr_proj_simplex_metric_{f32,f64}
 *           replaces proj_simplex_metric<real>
 *           (reference include/proj_simplex.hpp:33-35,
 *            src/proj_simplex_metric.cpp:18-83)
 *
 *  2. Sessions: the same solvers with inputs that may already live in HBM,
 *     setup separated from iterations (benchmarks, repeated solves) and the
 *     1-D vertex-range partition across GPUs (RCCL halo exchange).
 *
 * Every entry returns PFDR_OK (0) or an error code; pfdr_last_error() gives
 * the message of the calling thread's last failure.  There is no CPU
 * fallback: without a usable gfx950 device every compute entry fails.
 * ======================================================================== */
#ifndef PFDR_MI355X_H
#define PFDR_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PFDR_OK 0
#define PFDR_ERR_ARG 1    /* invalid argument */
#define PFDR_ERR_HIP 2    /* HIP runtime failure (no device, OOM, fault) */
#define PFDR_ERR_RCCL 3   /* collective failure */
#define PFDR_ERR_STATE 4  /* session used out of order */

/* Lipschitz information type, same values as the reference's
 * typedef enum {SCAL, DIAG} Lipschtype (include/PFDR_graph_quadratic_d1_l1.hpp:34) */
#define PFDR_LIPSCHITZ_SCAL 0
#define PFDR_LIPSCHITZ_DIAG 1

const char *pfdr_last_error(void);
int pfdr_abi_version(void);          /* 4 (pfdr_problem.spec added) */
int pfdr_device_count(void);         /* visible HIP devices, <0 on error */

/* ------------------------------------------------------------------ l1 -- */
int pfdr_quadratic_d1_l1_f32(int V, int E, int N, float *X, const float *Y,
    const float *A, const int *Eu, const int *Ev, const float *La_d1,
    const float *La_l1, int positivity, int Ltype, const float *L,
    float rho, float condMin, float difRcd, float difTol, int itMax,
    int *it, float *Obj, float *Dif, int verbose);
int pfdr_quadratic_d1_l1_f64(int V, int E, int N, double *X, const double *Y,
    const double *A, const int *Eu, const int *Ev, const double *La_d1,
    const double *La_l1, int positivity, int Ltype, const double *L,
    double rho, double condMin, double difRcd, double difTol, int itMax,
    int *it, double *Obj, double *Dif, int verbose);

/* -------------------------------------------------------------- bounds -- */
int pfdr_quadratic_d1_bounds_f32(int V, int E, int N, float *X,
    const float *Y, const float *A, const int *Eu, const int *Ev,
    const float *La_d1, float min, float max, int Ltype, const float *L,
    float rho, float condMin, float difRcd, float difTol, int itMax,
    int *it, float *Obj, float *Dif, int verbose);
int pfdr_quadratic_d1_bounds_f64(int V, int E, int N, double *X,
    const double *Y, const double *A, const int *Eu, const int *Ev,
    const double *La_d1, double min, double max, int Ltype, const double *L,
    double rho, double condMin, double difRcd, double difTol, int itMax,
    int *it, double *Obj, double *Dif, int verbose);

/* ------------------------------------------------------------- simplex -- */
int pfdr_loss_d1_simplex_f32(int K, int V, int E, float al,
    const float *La_f, float *P, const float *Q, const int *Eu,
    const int *Ev, const float *La_d1, float rho, float condMin,
    float difRcd, float difTol, int itMax, int *it, float *Obj, float *Dif,
    int verbose);
int pfdr_loss_d1_simplex_f64(int K, int V, int E, double al,
    const double *La_f, double *P, const double *Q, const int *Eu,
    const int *Ev, const double *La_d1, double rho, double condMin,
    double difRcd, double difTol, int itMax, int *it, double *Obj,
    double *Dif, int verbose);

int pfdr_proj_simplex_metric_f32(float *X, const float *M, int D, int N,
    int nm, const float *A, int na);
int pfdr_proj_simplex_metric_f64(double *X, const double *M, int D, int N,
    int nm, const double *A, int na);

/* ------------------------------------------------------------ sessions -- */
#define PFDR_KIND_L1 0
#define PFDR_KIND_BOUNDS 1
#define PFDR_KIND_SIMPLEX 2

#define PFDR_F32 0
#define PFDR_F64 1

#define PFDR_MEM_HOST 0    /* pointers are host memory (copied in) */
#define PFDR_MEM_DEVICE 1  /* pointers are device memory of the current device */
/* Ordering of device inputs: the library reads (and, for the session's
 * lifetime, keeps reading nothing but its own copies of) the caller's
 * device arrays on its own non-blocking stream, which does not wait for the
 * caller's streams.  Every write into those arrays must be complete before
 * the call (e.g. synchronise the producing stream; the Python front-end
 * synchronises torch's current stream).  Outputs are complete on return. */

/* Internal vertex relabelling for cache locality (breadth-first order,
 * pfdr_order.hip): AUTO applies it when the labels look random (V >= 2^20 and
 * over a quarter of the edges span more than V/64 labels).  Inputs and
 * outputs stay in the caller's labels; the reference's summation orders are
 * kept, so results do not change. */
#define PFDR_REORDER_AUTO 0
#define PFDR_REORDER_ON 1
#define PFDR_REORDER_OFF 2

/* Iterate-evolution statistic (the stopping / reconditioning test and Dif;
 * reference src/PFDR_graph_quadratic_d1_l1.cpp:514-529, simplex
 * src/PFDR_graph_loss_d1_simplex.cpp:653-691).  The reference adds its terms
 * one by one in `real`, and over millions of f32 terms that sum drifts by
 * percents from the exact value -- enough to move the stopping iteration.
 * SEQUENTIAL reproduces that rounding exactly (parallel binade scan,
 * pfdr_monosum.hpp): Dif, the stopping iteration and the iterate are then
 * the reference's bit for bit.  TREE sums in a fixed tree (faster; the
 * decision may land an iteration or so away on huge f32 problems).  AUTO:
 * SEQUENTIAL on one GPU for sums of at least 2^17 terms, except on the
 * small-graph paths that decide inside a sweep (quadratic: identity /
 * diagonal A, no objective record, <= 1,024 vertex blocks of 256; both
 * solvers' one-workgroup paths), which keep TREE.  A partitioned session
 * applies the same rule to its global term count: SEQUENTIAL sums the terms
 * rank to rank in the caller's order (ChainSum, pfdr_halo.hpp; a relabelled
 * split first routes every term to the rank owning that caller-order
 * slice), bit-identical to one GPU; the simplex's label counts (0 / 1 terms,
 * exact in any order) keep TREE there.  SEQUENTIAL forced on a small graph
 * takes the multi-launch loop instead of those paths. */
#define PFDR_EVOLUTION_AUTO 0
#define PFDR_EVOLUTION_SEQUENTIAL 1
#define PFDR_EVOLUTION_TREE 2
/* speculative decisions (pfdr_problem.spec; env PFDR_SPEC = auto | serial |
 * off overrides): sessions with a sequential evolution statistic, difRcd = 0
 * and no objective record decide on iteration t while t + 1 sweeps.
 *   AUTO   the evolution sums and the decision run on a second stream; a
 *          partition runs them over a communicator split from its own
 *          (ncclCommSplit) beside the next iteration's halo exchanges --
 *          concurrent operations on two communicators, which NCCL/RCCL do
 *          not guarantee to co-schedule;
 *   SERIAL the same buffers and decisions on the session stream over the one
 *          communicator: no split, no second stream, no concurrency; results
 *          identical bit for bit, the decision no longer overlapped;
 *   OFF    the plain sequential loop (identical results). */
#define PFDR_SPEC_AUTO 0
#define PFDR_SPEC_SERIAL 1
#define PFDR_SPEC_OFF 2

typedef struct pfdr_problem {
    int kind;             /* PFDR_KIND_* */
    int dtype;            /* PFDR_F32 / PFDR_F64: type of every real array */
    int mem;              /* PFDR_MEM_*: location of every array below */
    int V, E, N, K;       /* as the reference (K only for simplex) */
    void *X;              /* X (quadratic) or P (simplex), initial value */
    const void *Y;        /* Y / A^tY (quadratic) or Q (simplex) */
    const void *A;        /* quadratic only, NULL for identity */
    const int *Eu, *Ev;   /* endpoints (global vertex ids when distributed) */
    const void *La_d1;    /* length E */
    const void *La_l1;    /* l1 weights (V) or La_f (simplex, V); may be NULL */
    int positivity;       /* l1 only */
    double min, max;      /* bounds only (+-HUGE_VAL for none) */
    double al;            /* simplex only */
    int Ltype;            /* PFDR_LIPSCHITZ_* */
    const void *L;        /* NULL, scalar or length V */
    double rho, condMin, difRcd, difTol;
    int itMax;
    int verbose;
    int record_obj;       /* keep Obj[0..itMax] on the device */
    int record_dif;       /* keep Dif[0..itMax-1] on the device */
    /* --- 1-D vertex-range partition (leave zero for one GPU) ------------ */
    int nranks, rank;     /* rank r owns global vertices [vtx_begin, vtx_begin+V) */
    void *comm;           /* ncclComm_t (pfdr_comm_init) or loopback hub */
    int comm_kind;        /* PFDR_COMM_RCCL or PFDR_COMM_LOOPBACK */
    int64_t vtx_begin;    /* first owned global vertex */
    int64_t V_global;     /* total vertices over all ranks */
    const int64_t *e_global; /* global id of each local edge; NULL: e_offset + e */
    int64_t e_offset;
    /* --- internal locality reordering (quadratic solvers, one GPU) -------- */
    int reorder;          /* PFDR_REORDER_*; results are identical either way */
    /* --- iterate-evolution statistic -------------------------------------- */
    int evolution;        /* PFDR_EVOLUTION_* */
    /* --- relabelled partition (pfdr_locality_order) ----------------------- */
    const int64_t *vtx_label; /* caller's label of each owned vertex (V of them,
                             host or device per mem); NULL: vtx_begin + v.  Set
                             when the ranks own ranges of a RELABELLED graph:
                             the preconditioner's amplitude sum then runs in
                             the caller's label order (all-reduced, then summed
                             in that order on every rank), as the reference's
                             one-thread loop does (quadratic solvers). */
    /* --- speculative decisions ---------------------------------------------- */
    int spec;             /* PFDR_SPEC_* (0: AUTO) */
} pfdr_problem;

typedef struct pfdr_session pfdr_session;

/* Locality order of a graph's vertices for a vertex-range partition
 * (randomly labelled k-NN graphs must be reordered before
 * partitioning, or every edge becomes a halo edge): the deterministic
 * breadth-first order of pfdr_order.hip, computed on the current device.
 * order_out[new] = old label (V entries, host or device per mem).  *applied
 * = 0 when the graph is path-like (too many levels) and the identity was
 * returned.  Use: rank r owns new labels [off[r], off[r+1]), its edges are
 * those whose relabelled Eu it owns (original edge ids as e_global), and
 * vtx_label = order_out[off[r] .. off[r+1]) (see partition.py). */
int pfdr_locality_order(int V, int64_t E, const int *Eu, const int *Ev, int mem,
                        int *order_out, int *applied);

int pfdr_session_create(pfdr_session **out, const pfdr_problem *p);
/* Run up to `iters` more iterations (stopping early on difTol / itMax as the
 * reference does).  *it_total receives the total iteration count so far. */
int pfdr_session_run(pfdr_session *s, int iters, int *it_total);
/* Capture now the hipGraphs that a later pfdr_session_run(s, iters) replays
 * (chunks of 32 iterations and the run's tail), so that the run itself
 * instantiates nothing; no iteration runs.  A no-op where the session
 * launches directly (small one-workgroup graphs, objective record, loopback
 * partitions). */
int pfdr_session_prepare(pfdr_session *s, int iters);
/* Copy X (or P) back to host memory, and the iteration count; Obj/Dif copy
 * it+1 / it values when recorded (may be NULL). */
int pfdr_session_result(pfdr_session *s, void *X_host, int *it, void *Obj_host,
                        void *Dif_host);
/* Device pointer of the current iterate (valid until destroy). */
void *pfdr_session_device_x(pfdr_session *s);
/* Kernel timing: when enabled, HIP events bracket the launches of the named
 * kernels on the session stream; stats give timed launches and mean
 * duration.  on = 0 off, 1 every launch, P >= 2 every P-th launch of each
 * kernel (an event pair costs ~6-9 us of GPU time: sampling keeps it out of
 * short iterations).  The filter restricts timing to a comma-separated list
 * of kernel names (NULL or "" = all). */
int pfdr_session_set_profiling(pfdr_session *s, int on);
int pfdr_session_profile_filter(pfdr_session *s, const char *names);
int pfdr_session_kernel_stats(pfdr_session *s, const char *kernel,
                              int *launches, double *mean_ms);
/* Synchronise the session stream. */
int pfdr_session_sync(pfdr_session *s);
/* Bytes of device memory held by the session. */
int64_t pfdr_session_device_bytes(pfdr_session *s);
/* Session facts by name: "reordered" (1 when the internal locality
 * relabelling is active), "device_bytes", "split_blocks", "ustaged",
 * "symv", "tiny", "coop" (workgroups of the persistent mid-size-graph
 * launch, 0 when off), "fused" (1: the loop decision of a small graph is
 * taken inside the next edge sweep, two launches per iteration), "padded"
 * (1: such a graph's contributions are stored in per-vertex-block lists, so
 * its vertex sweep stages them without dependent address loads),
 * "dense_exact" (1: the dense products run in the reference's sequential
 * order, bit-exact; small single-GPU problems), "tiled_blocks" (vertex
 * blocks staging tile-ordered contributions) and "record_blocks" (of those,
 * the blocks whose runs fit one per-block record), "slot_patterns" (distinct
 * slot sequences of those records' runs, 0: per-entry slots), "speculative"
 * (1: the evolution sums run beside the next iteration's sweeps on a second
 * stream, 2: after them on the session stream), "edge_ratio" (1: the tiled
 * edge sweep reads each end's (c La_d1 / Aux) / Ga formed once per vertex;
 * until the first reconditioning), "vertex_pair" (> 0: the vertex sweep takes
 * two record blocks per workgroup, the value the largest block's entries). */
int pfdr_session_query(pfdr_session *s, const char *what, int64_t *value);
void pfdr_session_destroy(pfdr_session *s);

/* ------------------------------------------- dense matrices (CP builder) -- */
/* Gram matrix on the matrix cores (exact-f32 / f64 MFMA, fixed-order
 * reductions): which = 0 -> G = A^t A (N-by-N), 1 -> G = A A^t (M-by-M); A
 * is M-by-N column major; mem = PFDR_MEM_HOST or _DEVICE for A and G.
 * *ms (may be NULL) receives the kernel time.  Replaces the reference's
 * symmetrisation loops (src/operator_norm_matrix.cpp:112-165,
 * src/CP_PFDR_graph_quadratic_d1_l1.cpp:688-702). */
int pfdr_gram_f32(int which, int M, int N, const float *A, int mem, float *G, double *ms);
int pfdr_gram_f64(int which, int M, int N, const double *A, int mem, double *G, double *ms);
/* Strictly sequential sum seed + a[0] + ... + a[n-1] of NONNEGATIVE terms,
 * rounded exactly as the one-thread loop: the preconditioner's amplitude sum
 * (src/PFDR_graph_quadratic_d1_l1.cpp:146-152, _bounds.cpp:143-149).  method 0:
 * workgroup binade scan (what the solvers use), 1: one-lane loop.  mem =
 * PFDR_MEM_HOST / _DEVICE for a; *ms (may be NULL) receives the kernel time.
 * Negative terms give an unspecified result. */
int pfdr_sequential_sum_f32(int64_t n, const float *a, int mem, float seed, int method,
                            float *out, double *ms);
int pfdr_sequential_sum_f64(int64_t n, const double *a, int mem, double seed, int method,
                            double *out, double *ms);
/* The stable LSD radix sort the library builds its incidence lists with
 * (pairs sorted by the low `bits` bits of the key, equal keys in input
 * order), on host arrays, in place; *ms (may be NULL) receives the sort's
 * GPU time.  n < 2^31.  Exposed for its tests. */
int pfdr_radix_sort_pairs_u32(int64_t n, uint32_t *keys, uint32_t *vals, int bits, double *ms);
int pfdr_radix_sort_pairs_u64(int64_t n, uint64_t *keys, uint32_t *vals, int bits, double *ms);
/* Squared operator norm ||A||^2 by the power method (reference
 * operator_norm_matrix<real>, include/operator_norm_matrix.hpp:12-14, same
 * argument meaning; deterministic starts).  *gram_ms (may be NULL): time of
 * the Gram step when the matrix was symmetrised first. */
int pfdr_operator_norm_f32(int M, int N, const float *A, int mem, float nTol, int itMax,
                           int nbInit, int verbose, float *norm2, double *gram_ms);
int pfdr_operator_norm_f64(int M, int N, const double *A, int mem, double nTol, int itMax,
                           int nbInit, int verbose, double *norm2, double *gram_ms);

/* Cut-pursuit reduced-problem builder (reference
 * src/CP_PFDR_graph_quadratic_d1_l1.cpp:663-841).
 * Components: rVc[rV + 1] offsets into the vertex list Vc[V].  A, Y as the
 * CP caller's (N > 0: A N-by-V, Y length N; N = -V: A = A^tA, Y = A^tY;
 * N = 0: A diagonal or NULL).  preAt (N > 0): also form rAA = rA^t rA and
 * rY = rA^t Y (forced for N <= 0).  Outputs (host or device per mem): rA
 * (N-by-rV, N > 0), rAA (rV-by-rV, or rV for N = 0), rY (rV; not formed
 * for N > 0 without preAt: CP then passes the whole Y), L (rV: the
 * Lipschitz metric l^2 c after Jacobi equilibration, c = squared norm of
 * the equilibrated matrix by the power method with normTol / normItMax /
 * normNbInit — CP uses 1e-3, 100, 10), Leq (rV, may be NULL: l).  All sums
 * sequential in the reference's order (bit-identical to the restatement);
 * only c depends on the (deterministic) starts. */
int pfdr_cp_reduce_f32(int N, int V, const float *A, const float *Y, int rV, const int *rVc,
                       const int *Vc, int preAt, int mem, float normTol, int normItMax,
                       int normNbInit, float *rA, float *rAA, float *rY, float *L, float *Leq);
int pfdr_cp_reduce_f64(int N, int V, const double *A, const double *Y, int rV, const int *rVc,
                       const int *Vc, int preAt, int mem, double normTol, int normItMax,
                       int normNbInit, double *rA, double *rAA, double *rY, double *L,
                       double *Leq);

/* ------------------------------------------- cut-pursuit graph steps -- */
/* The full-graph work of every cut-pursuit iteration around the reduced
 * PFDR solve, on a device-resident graph
 * (reference src/CP_PFDR_graph_quadratic_d1_l1.cpp; the maxflow stays with
 * the caller: capacities out, segments 0 = SOURCE / 1 = SINK back).  The
 * graph holds the endpoints, TV weights La_d1[E], l1 weights La_l1[V] (or
 * NULL), the activity of every edge (CP's is_active, initially none), the
 * components (Cv[V], Vc[V], rVc[rV + 1], initially one) and the component
 * values rX[rV].  Every result equals the reference's, including its
 * orders (queue order of Vc, visiting order of the reduced edges) and its
 * floating sums.  dtype PFDR_F32 / PFDR_F64 fixes the real type of every
 * void* below; mem = PFDR_MEM_HOST / _DEVICE for the caller's arrays. */
typedef struct pfdr_cpgraph pfdr_cpgraph;
int pfdr_cpgraph_create(pfdr_cpgraph **out, int dtype, int V, int E,
    const int *Eu, const int *Ev, const void *La_d1, const void *La_l1, int mem);
void pfdr_cpgraph_destroy(pfdr_cpgraph *g);
int pfdr_cpgraph_set_active(pfdr_cpgraph *g, const uint8_t *active, int mem);
int pfdr_cpgraph_get_active(pfdr_cpgraph *g, uint8_t *active, int mem);
int pfdr_cpgraph_set_components(pfdr_cpgraph *g, int rV, const int *Cv,
    const int *Vc, const int *rVc, int mem);
/* any output may be NULL */
int pfdr_cpgraph_get_components(pfdr_cpgraph *g, int *rV, int *Cv, int *Vc,
    int *rVc, int mem);
/* rX[rV]: the values of the current components */
int pfdr_cpgraph_set_values(pfdr_cpgraph *g, const void *rX, int mem);
/* connected components of the graph minus its active edges (:566-597) */
int pfdr_cpgraph_components(pfdr_cpgraph *g, int *rV);
/* reduced edges and weights of the current components (:599-661); eps is
 * CP's (:236-251), the weight of an isolated component's self-loop */
int pfdr_cpgraph_reduced_graph(pfdr_cpgraph *g, double eps, int *rE);
/* rEu, rEv, rLa_d1 [rE], rLa_l1 [rV] (when La_l1); any may be NULL */
int pfdr_cpgraph_get_reduced(pfdr_cpgraph *g, int *rEu, int *rEv,
    void *rLa_d1, void *rLa_l1, int mem);
/* deactivate the active edges whose components' values differ by at most
 * CP_difTol relatively (:863-886) */
int pfdr_cpgraph_merge(pfdr_cpgraph *g, double eps, double CP_difTol, int *deactivated);
/* DfS[V] (kept on the device; copied out when DfS != NULL) at the current
 * values (:339-413): N > 0: A N-by-V, R[N] the residual Y - A X; N = -V:
 * A = A^tA, Y = A^tY; N = 0: A diagonal or NULL, Y = A^tY */
int pfdr_cpgraph_gradient(pfdr_cpgraph *g, int N, const void *A, const void *Y,
    const void *R, int mem, void *DfS);
/* cut 0: the single cut of the differentiable case (La_l1 NULL, no
 * positivity); 1 / 2: directions +1_U / -1_U (:402-535).  tr_cap[V]
 * (source > 0 / sink < 0), r_cap[E] (both arcs of an edge), from the
 * activity BEFORE this cut's activations; either may be NULL */
int pfdr_cpgraph_capacities(pfdr_cpgraph *g, int cut, int positivity,
    void *tr_cap, void *r_cap, int mem);
/* the same for CP_PFDR_graph_quadratic_d1_bounds (graph created without
 * La_l1): cut 0 when min = -inf and max = inf; cut 1 (+1_U): +inf on the
 * components at max, else DfS; cut 2 (-1_U): +inf on the components at min,
 * else -DfS (src/CP_PFDR_graph_quadratic_d1_bounds.cpp:386-534) */
int pfdr_cpgraph_capacities_bounds(pfdr_cpgraph *g, int cut, double min, double max,
    void *tr_cap, void *r_cap, int mem);
/* activate the inactive edges whose ends lie in different segments[V] */
int pfdr_cpgraph_activate(pfdr_cpgraph *g, const uint8_t *segment, int mem,
    int *activated);

/* The duplex driver, CP_PFDR_graph_quadratic_d1_l1_duplex, in its
 * non-differentiable case (graph created with La_l1; positivity optional):
 * one cut per iteration on a two-layer maxflow graph, node v (v1) and node
 * V + v (v2) per vertex (src/CP_PFDR_graph_quadratic_d1_l1_duplex.cpp:101-116).
 * The gradient is pfdr_cpgraph_gradient's.  tr_cap[2V] (v1 nodes, then v2),
 * r_link[V] (arc v1 -> v2; v2 -> v1 has none), r_cap[E] (every arc of edge
 * e, both layers) from the activity before the cut (:469-527); any may be
 * NULL.  Activation: edges separated in either layer, segment[2V]
 * (:531-545).  The components, reduced graph and merge are the l1 driver's.
 * (Its differentiable case indexes La_d1 as if its one-layer graph had four
 * arcs per edge, :407 / :628 -- not reproduced.) */
int pfdr_cpgraph_capacities_duplex(pfdr_cpgraph *g, int positivity, void *tr_cap,
    void *r_link, void *r_cap, int mem);
int pfdr_cpgraph_activate_duplex(pfdr_cpgraph *g, const uint8_t *segment, int mem,
    int *activated);

/* The simplex driver, CP_PFDR_graph_loss_d1_simplex (graph created
 * without La_l1): K >= 2 labels, Q[V*K] and the component label vectors
 * rP[rV*K] vertex-major like the reference (P[v*K + k]); al = 0 linear,
 * 1 quadratic, (0, 1) smoothed-KL loss.  One CP iteration: gradient ->
 * for n = 1 .. K-1 { capacities(n) -> caller's maxflow -> expand(n,
 * segments) } -> activate -> pfdr_cpgraph_components -> reduced_graph ->
 * observations (the reduced problem's rQ, rLa_f and warm start rP) ->
 * PFDR_graph_loss_d1_simplex -> set_values -> merge.  eps: the driver's
 * finite-difference precision (src/CP_PFDR_graph_loss_d1_simplex.cpp:214-231).
 * Replaces :327-376 (gradient), :525-536 (most confident labels),
 * :542-604 (alpha-expansion capacities and labels), :608-618 (activation),
 * :733-766 (reduced observations) and :782-803 (merge). */
int pfdr_cpgraph_simplex_setup(pfdr_cpgraph *g, int K, double al, const void *Q, int mem);
/* per component the sums of Q in Vc order; linear: rQ = sums, rP = corner
 * of the first largest; else rQ = rP = sums / size, rLa_f[rV] = size.  The
 * component values become rP.  Any output may be NULL; also gives the
 * initial values of the one-component state (:96-108) */
int pfdr_cpgraph_simplex_observations(pfdr_cpgraph *g, void *rP, void *rQ, void *rLa_f,
    int mem);
/* rP[rV*K]: the label vectors of the current components (PFDR's output) */
int pfdr_cpgraph_simplex_set_values(pfdr_cpgraph *g, const void *rP, int mem);
/* DfS[V*K] and rDi[rV] (most confident label per component), kept on the
 * device (copied out when not NULL); resets every vertex's alternative */
int pfdr_cpgraph_simplex_gradient(pfdr_cpgraph *g, double eps, void *DfS, int *rDi, int mem);
/* alpha-expansion n in [1, K): tr_cap[V] and r_cap[E], the capacity of arc
 * 2e (Eu -> Ev); arc 2e + 1 has none (:563-595) */
int pfdr_cpgraph_simplex_capacities(pfdr_cpgraph *g, int n, void *tr_cap, void *r_cap,
    int mem);
/* the SINK side of expansion n's maxflow takes alternative n (:600-604) */
int pfdr_cpgraph_simplex_expand(pfdr_cpgraph *g, int n, const uint8_t *segment, int mem);
int pfdr_cpgraph_simplex_activate(pfdr_cpgraph *g, int *activated);
/* deactivate the active edges whose components' label vectors differ by
 * at most eps in every label */
int pfdr_cpgraph_simplex_merge(pfdr_cpgraph *g, double eps, int *deactivated);
/* Djv[V]: every vertex's alternative after the expansions so far */
int pfdr_cpgraph_simplex_labels(pfdr_cpgraph *g, int *Djv, int mem);

/* ------------------------------------------------------ multi-GPU comm -- */
/* Partitioned sessions (quadratic solvers, identity or diagonal A): every
 * rank passes its owned vertices (V of them, global ids [vtx_begin,
 * vtx_begin + V), ranks in vertex order) and its edges (global endpoint ids,
 * global edge ids e_global or e_offset + e).  Creation and every run() are
 * collective.  The result equals the unpartitioned solve bit for bit. */
#define PFDR_COMM_RCCL 0      /* one process per GPU, ncclComm_t */
#define PFDR_COMM_LOOPBACK 1  /* k ranks as k threads of one process, one GPU */
#define PFDR_COMM_ID_BYTES 128
/* rank 0 creates the id, the caller broadcasts it, every rank inits */
int pfdr_comm_unique_id(void *id_out /* PFDR_COMM_ID_BYTES */);
int pfdr_comm_init(void **comm_out, int nranks, int rank, const void *id);
int pfdr_comm_destroy(void *comm);
int pfdr_comm_allreduce_max_f64(void *comm, double *value);
int pfdr_loopback_create(void **hub_out, int nranks);
/* a failing rank wakes the others: their pending and later exchanges fail */
int pfdr_loopback_abort(void *hub, const char *reason);
int pfdr_loopback_destroy(void *hub);
/* Watchdog: a rank whose collective does not complete within
 * PFDR_COMM_TIMEOUT seconds (default 120) prints
 * "[pfdr watchdog] ... rank r of n, <phase>, iteration i, last collective:
 * <op, peers, bytes>" to stderr, aborts the communicator (RCCL) or the hub
 * (loopback) and fails the call with that message (no retry). */

/* Several GPUs behind the drop-in entry points (one synchronous call, one
 * host thread per device, RCCL communicators from ncclCommInitAll, created
 * once and cached across calls): the drop-in calls of this process with at
 * least min_vertices vertices (< 0: the default 2^20) are vertex-range
 * partitioned across devices[0 .. n) -- bit-identical to the one-GPU solve.
 * n = 0 returns to one GPU.  The devices must be all distinct (RCCL), or one
 * device repeated, which runs the ranks as threads on it (loopback transport;
 * for tests); a mixed list is refused and leaves the configuration as it was.
 * Without this call the PFDR_DEVICES environment variable (N or "all")
 * selects devices 0 .. N-1. */
int pfdr_set_devices(int n, const int *devices, int64_t min_vertices);

/* Host-only partition planner (what the partitioned session runs at setup;
 * exposed so the partition logic can be driven by any transport, e.g. the
 * CPU tests).  Rank `rank` owns global vertices [offsets[rank],
 * offsets[rank+1]); its E edges have global endpoints Eu/Ev and global ids
 * e_global (or e_offset + e).  Flow: create -> get PULL_REQUEST/PUSH_ITEMS
 * for every peer -> send them -> set_incoming what every peer sent ->
 * finish -> get the results.  pfdr_plan_get returns the element count and
 * copies the elements when out != NULL. */
typedef struct pfdr_plan pfdr_plan;
#define PFDR_PLAN_GHOSTS 0          /* int64 global ids of the ghost vertices */
#define PFDR_PLAN_EU_LOCAL 1        /* int32 local endpoint ids (ghosts >= V) */
#define PFDR_PLAN_EV_LOCAL 2
#define PFDR_PLAN_PULL_REQUEST 3    /* int64 ghost ids owned by `peer` */
#define PFDR_PLAN_PUSH_ITEMS 4      /* int64 (vertex, 2 e_global + side) pairs for `peer` */
#define PFDR_PLAN_PUSH_ADDR 5       /* uint32 contribution address of every item sent */
#define PFDR_PLAN_PULL_INDEX 6      /* int32 owned local ids to send, per peer */
#define PFDR_PLAN_RECV_KEYS 7       /* uint64 (local vertex << 32 | order) of items received */
#define PFDR_PLAN_GHOST_OFFSETS 8   /* int32 nranks + 1 */
#define PFDR_PLAN_PULL_OFFSETS 9    /* int32 nranks + 1, into PULL_INDEX */
#define PFDR_PLAN_PUSH_OFFSETS 10   /* int32 nranks + 1, into PUSH_ADDR */
#define PFDR_PLAN_RECV_OFFSETS 11   /* int32 nranks + 1, into RECV_KEYS */
int pfdr_plan_create(pfdr_plan **out, int nranks, int rank,
    const int64_t *offsets, int E, const int *Eu, const int *Ev,
    const int64_t *e_global, int64_t e_offset);
int64_t pfdr_plan_get(pfdr_plan *plan, int what, int peer, void *out);
int pfdr_plan_set_incoming(pfdr_plan *plan, int peer, int what, int64_t n,
    const int64_t *data);
int pfdr_plan_finish(pfdr_plan *plan);
void pfdr_plan_destroy(pfdr_plan *plan);

/* ---------------------------------------------------------- test hooks -- */
/* The per-edge-block records of the tiled edge sweep (k_edge_sweep_tl), built
 * on the device from host endpoint arrays already in tile order: blocks
 * [blk_begin, blk_begin + blk_count) of 1,024 (f32) / 512 (f64) edges are
 * written, every other record of rec (rec_ints = blocks * ints per record)
 * keeps what the caller put there -- so a test can check that building one
 * block's record touches nothing else.  Layout: pfdr_debug_erec_layout. */
int pfdr_debug_tile_erec(int64_t E, int dtype, const int *Eu, const int *Ev,
    int blk_begin, int blk_count, int *rec, int64_t rec_ints);
int pfdr_debug_erec_layout(int *ints, int *runs, int *nostage);

/* -------------------------------------------------- synthetic inputs -- */
/* Host-side deterministic generators (no device needed), identical laws to
 * cp_pfdr_graph_d1_amd/graphs.py.  Edges are written for emitters
 * [v_begin, v_end); the k-NN graph writes exactly k*(v_end-v_begin). */
int64_t pfdr_gen_knn_jitter_grid(int nx, int ny, int nz, int k, uint64_t seed,
    double jitter, int64_t v_begin, int64_t v_end, int *Eu, int *Ev);
int64_t pfdr_gen_grid_edges(int nx, int ny, int nz, int conn,
    int64_t v_begin, int64_t v_end, int *Eu, int *Ev);
int pfdr_gen_piecewise_f32(int nx, uint64_t seed, double noise,
    int64_t v_begin, int64_t v_end, float *Y);
int pfdr_gen_piecewise_f64(int nx, uint64_t seed, double noise,
    int64_t v_begin, int64_t v_end, double *Y);
/* Dense inputs (C3): out[i] = lo + (hi-lo) U(seed, i0+i); y = A x with each
 * row accumulated in double in increasing column order (host- and
 * thread-count independent); a symmetric diagonally dominant V-by-V matrix
 * (off-diagonal s (2U - 1), diagonal d). */
int pfdr_gen_uniform_f32(uint64_t seed, int64_t i0, int64_t n, double lo, double hi,
    float *out);
int pfdr_gen_uniform_f64(uint64_t seed, int64_t i0, int64_t n, double lo, double hi,
    double *out);
int pfdr_gen_matvec_f32(int64_t N, int64_t V, const float *A, const float *x, float *y);
int pfdr_gen_matvec_f64(int64_t N, int64_t V, const double *A, const double *x, double *y);
int pfdr_gen_symmetric_f32(int64_t V, uint64_t seed, double s, double d, float *G);
int pfdr_gen_symmetric_f64(int64_t V, uint64_t seed, double s, double d, double *G);

#ifdef __cplusplus
}
#endif
#endif /* PFDR_MI355X_H */
