"""Python host side of the MI355X PFDR solvers (ctypes over libpfdr_mi355x.so).

Two layers, both calling the C ABI of ``include/pfdr_mi355x.h``:

* ``Lib`` — one method per C entry point, same argument order as the
  reference C++ templates (include/PFDR_graph_quadratic_d1_l1.hpp:36-42 and
  friends) minus the outputs, numpy in / numpy out.
* MEX-style front-ends mirroring the reference's Octave wrappers
  (octave/mex/PFDR_*_mex.cpp): ``PFDR_graph_quadratic_d1_l1``,
  ``PFDR_graph_l22_d1_l1``, ``PFDR_graph_quadratic_d1_l1_AtA`` and the bounds
  and simplex counterparts, returning ``(X, it, Obj, Dif)`` like
  ``[X, it, Obj, Dif] = PFDR_..._mex(...)``.

There is no CPU fallback: if the shared library is missing, or the HIP device
is unusable, every call raises ``PFDRError``.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpfdr_mi355x.so")

PFDR_F32, PFDR_F64 = 0, 1
PFDR_MEM_HOST, PFDR_MEM_DEVICE = 0, 1
PFDR_KIND_L1, PFDR_KIND_BOUNDS, PFDR_KIND_SIMPLEX = 0, 1, 2
SCAL, DIAG = 0, 1
REORDER_AUTO, REORDER_ON, REORDER_OFF = 0, 1, 2
# iterate-evolution statistic (include/pfdr_mi355x.h PFDR_EVOLUTION_*)
EVOLUTION_AUTO, EVOLUTION_SEQUENTIAL, EVOLUTION_TREE = 0, 1, 2
# speculative decisions (PFDR_SPEC_*): own stream / split communicator,
# serial on the session stream over one communicator, or none
SPEC_AUTO, SPEC_SERIAL, SPEC_OFF = 0, 1, 2
ABI_VERSION = 4  # pfdr_abi_version() of the matching library

# every C entry point of include/pfdr_mi355x.h
EXPORTED = (
    "pfdr_last_error", "pfdr_abi_version", "pfdr_device_count",
    "pfdr_quadratic_d1_l1_f32", "pfdr_quadratic_d1_l1_f64",
    "pfdr_quadratic_d1_bounds_f32", "pfdr_quadratic_d1_bounds_f64",
    "pfdr_loss_d1_simplex_f32", "pfdr_loss_d1_simplex_f64",
    "pfdr_proj_simplex_metric_f32", "pfdr_proj_simplex_metric_f64",
    "pfdr_gram_f32", "pfdr_gram_f64", "pfdr_operator_norm_f32", "pfdr_operator_norm_f64",
    "pfdr_sequential_sum_f32", "pfdr_sequential_sum_f64",
    "pfdr_radix_sort_pairs_u32", "pfdr_radix_sort_pairs_u64",
    "pfdr_cp_reduce_f32", "pfdr_cp_reduce_f64",
    "pfdr_cpgraph_create", "pfdr_cpgraph_destroy", "pfdr_cpgraph_set_active",
    "pfdr_cpgraph_get_active", "pfdr_cpgraph_set_components", "pfdr_cpgraph_get_components",
    "pfdr_cpgraph_set_values", "pfdr_cpgraph_components", "pfdr_cpgraph_reduced_graph",
    "pfdr_cpgraph_get_reduced", "pfdr_cpgraph_merge", "pfdr_cpgraph_gradient",
    "pfdr_cpgraph_capacities", "pfdr_cpgraph_capacities_bounds", "pfdr_cpgraph_activate",
    "pfdr_cpgraph_simplex_setup", "pfdr_cpgraph_simplex_observations",
    "pfdr_cpgraph_simplex_set_values", "pfdr_cpgraph_simplex_gradient",
    "pfdr_cpgraph_simplex_capacities", "pfdr_cpgraph_simplex_expand",
    "pfdr_cpgraph_simplex_activate", "pfdr_cpgraph_simplex_merge", "pfdr_cpgraph_simplex_labels",
    "pfdr_cpgraph_capacities_duplex", "pfdr_cpgraph_activate_duplex",
    "pfdr_session_create", "pfdr_session_run", "pfdr_session_prepare", "pfdr_session_result",
    "pfdr_session_device_x", "pfdr_session_set_profiling", "pfdr_session_profile_filter",
    "pfdr_session_kernel_stats", "pfdr_session_sync",
    "pfdr_session_device_bytes", "pfdr_session_query", "pfdr_session_destroy",
    "pfdr_comm_unique_id", "pfdr_comm_init", "pfdr_comm_destroy",
    "pfdr_comm_allreduce_max_f64", "pfdr_loopback_create", "pfdr_loopback_abort",
    "pfdr_loopback_destroy", "pfdr_plan_create", "pfdr_plan_get",
    "pfdr_plan_set_incoming", "pfdr_plan_finish", "pfdr_plan_destroy",
    "pfdr_set_devices", "pfdr_debug_tile_erec", "pfdr_debug_erec_layout",
    "pfdr_gen_knn_jitter_grid", "pfdr_gen_grid_edges",
    "pfdr_gen_piecewise_f32", "pfdr_gen_piecewise_f64",
    "pfdr_gen_uniform_f32", "pfdr_gen_uniform_f64", "pfdr_gen_matvec_f32",
    "pfdr_gen_matvec_f64", "pfdr_gen_symmetric_f32", "pfdr_gen_symmetric_f64",
    "pfdr_locality_order",
)


class PFDRError(RuntimeError):
    pass


class Problem(C.Structure):
    """Mirror of ``pfdr_problem`` (include/pfdr_mi355x.h)."""
    _fields_ = [
        ("kind", C.c_int), ("dtype", C.c_int), ("mem", C.c_int),
        ("V", C.c_int), ("E", C.c_int), ("N", C.c_int), ("K", C.c_int),
        ("X", C.c_void_p), ("Y", C.c_void_p), ("A", C.c_void_p),
        ("Eu", C.c_void_p), ("Ev", C.c_void_p),
        ("La_d1", C.c_void_p), ("La_l1", C.c_void_p),
        ("positivity", C.c_int), ("min", C.c_double), ("max", C.c_double),
        ("al", C.c_double), ("Ltype", C.c_int), ("L", C.c_void_p),
        ("rho", C.c_double), ("condMin", C.c_double),
        ("difRcd", C.c_double), ("difTol", C.c_double),
        ("itMax", C.c_int), ("verbose", C.c_int),
        ("record_obj", C.c_int), ("record_dif", C.c_int),
        ("nranks", C.c_int), ("rank", C.c_int), ("comm", C.c_void_p),
        ("comm_kind", C.c_int),
        ("vtx_begin", C.c_int64), ("V_global", C.c_int64),
        ("e_global", C.c_void_p), ("e_offset", C.c_int64),
        ("reorder", C.c_int),
        ("evolution", C.c_int),
        ("vtx_label", C.c_void_p),
        ("spec", C.c_int),
    ]


_LIB = None


def load():
    """Load libpfdr_mi355x.so (built by __graft_entry__.build() / make)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise PFDRError("%s is missing: build it with "
                            "`make -C cp_pfdr_graph_d1_amd/csrc`" % LIB_PATH)
        # torch (when installed) first: its bundled HIP runtime is then the one
        # the library binds to, and torch.cuda keeps working in this process
        # (loaded the other way round, torch finds no GPU: INTEGRATION.md)
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        # PFDR_LIB_PATH: A/B of compile-time variants of the same library
        lib = C.CDLL(os.environ.get("PFDR_LIB_PATH") or LIB_PATH)
        lib.pfdr_last_error.restype = C.c_char_p
        lib.pfdr_session_device_x.restype = C.c_void_p
        lib.pfdr_session_device_bytes.restype = C.c_int64
        lib.pfdr_gen_knn_jitter_grid.restype = C.c_int64
        lib.pfdr_gen_grid_edges.restype = C.c_int64
        lib.pfdr_gen_knn_jitter_grid.argtypes = [
            C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_double,
            C.c_int64, C.c_int64, C.c_void_p, C.c_void_p]
        lib.pfdr_gen_grid_edges.argtypes = [
            C.c_int, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int64,
            C.c_void_p, C.c_void_p]
        for nm, ct in (("pfdr_gen_piecewise_f32", C.c_float),
                       ("pfdr_gen_piecewise_f64", C.c_double)):
            getattr(lib, nm).argtypes = [C.c_int, C.c_uint64, C.c_double,
                                         C.c_int64, C.c_int64, C.c_void_p]
        lib.pfdr_comm_allreduce_max_f64.argtypes = [C.c_void_p,
                                                    C.POINTER(C.c_double)]
        lib.pfdr_comm_init.argtypes = [C.POINTER(C.c_void_p), C.c_int,
                                       C.c_int, C.c_void_p]
        lib.pfdr_comm_destroy.argtypes = [C.c_void_p]
        # (PFDR_LIB_PATH: an A/B against a build of the previous ABI, 3, which
        # reads the problem without its trailing `spec` field)
        old_ok = bool(os.environ.get("PFDR_LIB_PATH")) and lib.pfdr_abi_version() == 3
        if lib.pfdr_abi_version() != ABI_VERSION and not old_ok:
            raise PFDRError("%s has ABI %d, this module expects %d: rebuild it" % (
                LIB_PATH, lib.pfdr_abi_version(), ABI_VERSION))
        _LIB = lib
    return _LIB


def _check(status, what):
    if status != 0:
        raise PFDRError("%s failed (%d): %s" % (
            what, status, load().pfdr_last_error().decode()))


def _real(dtype):
    dtype = np.dtype(dtype)
    if dtype == np.float32:
        return C.c_float, "f32", PFDR_F32
    if dtype == np.float64:
        return C.c_double, "f64", PFDR_F64
    raise TypeError("PFDR supports float32 and float64, got %s" % dtype)


def _arr(a, dtype):
    if a is None:
        return None
    return np.ascontiguousarray(a, dtype=dtype)


def _ptr(a, ct):
    return None if a is None else a.ctypes.data_as(C.POINTER(ct))


class Lib:
    """Raw C-ABI calls (host pointers, synchronous)."""

    def __init__(self):
        self.lib = load()

    def quadratic_d1_l1(self, X0, Y, A, N, Eu, Ev, La_d1, La_l1=None,
                        positivity=0, Ltype=SCAL, L=None, rho=1.5,
                        condMin=1e-3, difRcd=0.0, difTol=1e-5, itMax=1000,
                        obj=False, dif=False, verbose=0):
        X = np.array(X0, copy=True)
        ct, sfx, _ = _real(X.dtype)
        dt = X.dtype
        Y, A, La_d1, La_l1, L = (_arr(a, dt) for a in (Y, A, La_d1, La_l1, L))
        Eu, Ev = _arr(Eu, np.int32), _arr(Ev, np.int32)
        Obj = np.zeros(itMax + 1, dt) if obj else None
        Dif = np.zeros(max(itMax, 1), dt) if dif else None
        it = C.c_int(0)
        fn = getattr(self.lib, "pfdr_quadratic_d1_l1_" + sfx)
        _check(fn(C.c_int(X.size), C.c_int(Eu.size), C.c_int(N), _ptr(X, ct),
                  _ptr(Y, ct), _ptr(A, ct), _ptr(Eu, C.c_int),
                  _ptr(Ev, C.c_int), _ptr(La_d1, ct), _ptr(La_l1, ct),
                  C.c_int(positivity), C.c_int(Ltype), _ptr(L, ct), ct(rho),
                  ct(condMin), ct(difRcd), ct(difTol), C.c_int(itMax),
                  C.byref(it), _ptr(Obj, ct), _ptr(Dif, ct),
                  C.c_int(verbose)), "pfdr_quadratic_d1_l1_" + sfx)
        return X, it.value, Obj, Dif

    def quadratic_d1_bounds(self, X0, Y, A, N, Eu, Ev, La_d1, lo=-np.inf,
                            hi=np.inf, Ltype=SCAL, L=None, rho=1.5,
                            condMin=1e-3, difRcd=0.0, difTol=1e-5,
                            itMax=1000, obj=False, dif=False, verbose=0):
        X = np.array(X0, copy=True)
        ct, sfx, _ = _real(X.dtype)
        dt = X.dtype
        Y, A, La_d1, L = (_arr(a, dt) for a in (Y, A, La_d1, L))
        Eu, Ev = _arr(Eu, np.int32), _arr(Ev, np.int32)
        Obj = np.zeros(itMax + 1, dt) if obj else None
        Dif = np.zeros(max(itMax, 1), dt) if dif else None
        it = C.c_int(0)
        fn = getattr(self.lib, "pfdr_quadratic_d1_bounds_" + sfx)
        _check(fn(C.c_int(X.size), C.c_int(Eu.size), C.c_int(N), _ptr(X, ct),
                  _ptr(Y, ct), _ptr(A, ct), _ptr(Eu, C.c_int),
                  _ptr(Ev, C.c_int), _ptr(La_d1, ct), ct(lo), ct(hi),
                  C.c_int(Ltype), _ptr(L, ct), ct(rho), ct(condMin),
                  ct(difRcd), ct(difTol), C.c_int(itMax), C.byref(it),
                  _ptr(Obj, ct), _ptr(Dif, ct), C.c_int(verbose)),
               "pfdr_quadratic_d1_bounds_" + sfx)
        return X, it.value, Obj, Dif

    def loss_d1_simplex(self, P0, Q, K, Eu, Ev, La_d1, al=0.1, La_f=None,
                        rho=1.0, condMin=0.1, difRcd=0.0, difTol=1e-4,
                        itMax=1000, obj=False, dif=False, verbose=0):
        P = np.array(P0, copy=True)
        ct, sfx, _ = _real(P.dtype)
        dt = P.dtype
        Q, La_d1, La_f = (_arr(a, dt) for a in (Q, La_d1, La_f))
        Eu, Ev = _arr(Eu, np.int32), _arr(Ev, np.int32)
        Obj = np.zeros(itMax + 1, dt) if obj else None
        Dif = np.zeros(max(itMax, 1), dt) if dif else None
        it = C.c_int(0)
        fn = getattr(self.lib, "pfdr_loss_d1_simplex_" + sfx)
        _check(fn(C.c_int(K), C.c_int(P.size // K), C.c_int(Eu.size), ct(al),
                  _ptr(La_f, ct), _ptr(P, ct), _ptr(Q, ct), _ptr(Eu, C.c_int),
                  _ptr(Ev, C.c_int), _ptr(La_d1, ct), ct(rho), ct(condMin),
                  ct(difRcd), ct(difTol), C.c_int(itMax), C.byref(it),
                  _ptr(Obj, ct), _ptr(Dif, ct), C.c_int(verbose)),
               "pfdr_loss_d1_simplex_" + sfx)
        return P, it.value, Obj, Dif

    def proj_simplex_metric(self, X0, M, D, N, nm, A, na):
        X = np.array(X0, copy=True)
        ct, sfx, _ = _real(X.dtype)
        M, A = _arr(M, X.dtype), _arr(A, X.dtype)
        fn = getattr(self.lib, "pfdr_proj_simplex_metric_" + sfx)
        _check(fn(_ptr(X, ct), _ptr(M, ct), C.c_int(D), C.c_int(N),
                  C.c_int(nm), _ptr(A, ct), C.c_int(na)),
               "pfdr_proj_simplex_metric_" + sfx)
        return X


# ------------------------------------------------------ MEX-style API -----
def _edges(Eu, Ev):
    # the Python binding reinterprets uint32 edge arrays as int
    # (reference python/CP_quadratic_l1_py.cpp:228-258); accept any integer
    return (np.ascontiguousarray(Eu).astype(np.int32, copy=False),
            np.ascontiguousarray(Ev).astype(np.int32, copy=False))


def _scal_or_vec(x, n, dt):
    """MEX wrappers pass scalars for 'none' (numel == 1 -> NULL)."""
    if x is None:
        return None
    a = np.asarray(x, dt).ravel()
    return None if a.size <= 1 else a


def PFDR_graph_quadratic_d1_l1(Y, A, Eu, Ev, La_d1, La_l1, positivity, L,
                               rho, condMin, difRcd, difTol, itMax,
                               verbose=0, obj=False, dif=False):
    """[X, it, Obj, Dif] = PFDR_graph_quadratic_d1_l1_mex(Y, A, Eu, Ev, La_d1,
    La_l1, positivity, L, rho, condMin, difRcd, difTol, itMax, verbose)
    (octave/mex/PFDR_graph_quadratic_d1_l1_mex.cpp): A is N-by-V."""
    A = np.asarray(A)
    dt = np.result_type(Y, np.float32)
    N, V = A.shape
    L = np.asarray(L, dt).ravel()
    Ltype = SCAL if L.size == 1 else DIAG
    Eu, Ev = _edges(Eu, Ev)
    return Lib().quadratic_d1_l1(
        np.zeros(V, dt), np.asarray(Y, dt), np.asfortranarray(A, dt).ravel(order="F"),
        N, Eu, Ev, np.asarray(La_d1, dt), _scal_or_vec(La_l1, V, dt),
        positivity, Ltype, L, rho, condMin, difRcd, difTol, itMax, obj, dif,
        verbose)


def PFDR_graph_quadratic_d1_l1_AtA(AtY, AtA, Eu, Ev, La_d1, La_l1, positivity,
                                   L, rho, condMin, difRcd, difTol, itMax,
                                   verbose=0, obj=False, dif=False):
    """octave/mex/PFDR_graph_quadratic_d1_l1_AtA_mex.cpp: N = -V."""
    dt = np.result_type(AtY, np.float32)
    V = np.asarray(AtY).size
    L = np.asarray(L, dt).ravel()
    Eu, Ev = _edges(Eu, Ev)
    return Lib().quadratic_d1_l1(
        np.zeros(V, dt), np.asarray(AtY, dt),
        np.asfortranarray(AtA, dt).ravel(order="F"), -V, Eu, Ev,
        np.asarray(La_d1, dt), _scal_or_vec(La_l1, V, dt), positivity,
        SCAL if L.size == 1 else DIAG, L, rho, condMin, difRcd, difTol, itMax,
        obj, dif, verbose)


def PFDR_graph_l22_d1_l1(Y, La_l2, Eu, Ev, La_d1, La_l1, positivity, rho,
                         condMin, difRcd, difTol, itMax, verbose=0,
                         obj=False, dif=False):
    """octave/mex/PFDR_graph_l22_d1_l1_mex.cpp:54-83: Y <- La_l2*Y, N = 0,
    A = La_l2 (diagonal), Ltype DIAG, L = La_l2; Obj += 1/2 ||y||^2_La_l2."""
    Y = np.asarray(Y)
    dt = np.result_type(Y, np.float32)
    V = Y.size
    La_l2 = _scal_or_vec(La_l2, V, dt)
    Yw = (La_l2 * Y).astype(dt) if La_l2 is not None else Y.astype(dt)
    Eu, Ev = _edges(Eu, Ev)
    X, it, Obj, Dif = Lib().quadratic_d1_l1(
        np.zeros(V, dt), Yw, La_l2, 0, Eu, Ev, np.asarray(La_d1, dt),
        _scal_or_vec(La_l1, V, dt), positivity, DIAG, La_l2, rho, condMin,
        difRcd, difTol, itMax, obj, dif, verbose)
    if Obj is not None:
        y = Y.astype(dt)
        w = La_l2 if La_l2 is not None else np.ones(V, dt)
        y2 = float(np.sum(w.astype(np.float64) * y * y)) / 2.0
        Obj[: it + 1] += y2
    return X, it, Obj, Dif


def PFDR_graph_quadratic_d1_bounds(Y, A, Eu, Ev, La_d1, Bnd, L, rho, condMin,
                                   difRcd, difTol, itMax, verbose=0,
                                   obj=False, dif=False):
    """octave/mex/PFDR_graph_quadratic_d1_bounds_mex.cpp (Bnd = [min, max])."""
    A = np.asarray(A)
    dt = np.result_type(Y, np.float32)
    N, V = A.shape
    L = np.asarray(L, dt).ravel()
    Eu, Ev = _edges(Eu, Ev)
    return Lib().quadratic_d1_bounds(
        np.zeros(V, dt), np.asarray(Y, dt), np.asfortranarray(A, dt).ravel(order="F"),
        N, Eu, Ev, np.asarray(La_d1, dt), Bnd[0], Bnd[1],
        SCAL if L.size == 1 else DIAG, L, rho, condMin, difRcd, difTol, itMax,
        obj, dif, verbose)


def PFDR_graph_l22_d1_bounds(Y, La_l2, Eu, Ev, La_d1, Bnd, rho, condMin,
                             difRcd, difTol, itMax, verbose=0, obj=False,
                             dif=False):
    """octave/mex/PFDR_graph_l22_d1_bounds_mex.cpp."""
    Y = np.asarray(Y)
    dt = np.result_type(Y, np.float32)
    V = Y.size
    La_l2 = _scal_or_vec(La_l2, V, dt)
    Yw = (La_l2 * Y).astype(dt) if La_l2 is not None else Y.astype(dt)
    Eu, Ev = _edges(Eu, Ev)
    X, it, Obj, Dif = Lib().quadratic_d1_bounds(
        np.zeros(V, dt), Yw, La_l2, 0, Eu, Ev, np.asarray(La_d1, dt), Bnd[0],
        Bnd[1], DIAG, La_l2, rho, condMin, difRcd, difTol, itMax, obj, dif,
        verbose)
    if Obj is not None:
        y = Y.astype(dt)
        w = La_l2 if La_l2 is not None else np.ones(V, dt)
        Obj[: it + 1] += float(np.sum(w.astype(np.float64) * y * y)) / 2.0
    return X, it, Obj, Dif


def PFDR_graph_loss_d1_simplex(Q, al, Eu, Ev, La_d1, rho, condMin, difRcd,
                               difTol, itMax, verbose=0, obj=False,
                               dif=False, La_f=None, P0=None):
    """octave/mex/PFDR_graph_loss_d1_simplex_mex.cpp: Q is K-by-V (column v
    = Q[:, v]); P starts at Q (:33) and La_f is NULL (:46) unless given."""
    Q = np.asarray(Q)
    dt = np.result_type(Q, np.float32)
    K = Q.shape[0]
    q = np.asfortranarray(Q, dt).ravel(order="F")
    p0 = q if P0 is None else np.asfortranarray(P0, dt).ravel(order="F")
    Eu, Ev = _edges(Eu, Ev)
    P, it, Obj, Dif = Lib().loss_d1_simplex(
        p0, q, K, Eu, Ev, np.asarray(La_d1, dt), al, La_f, rho, condMin,
        difRcd, difTol, itMax, obj, dif, verbose)
    return P.reshape(Q.shape, order="F"), it, Obj, Dif


def PFDR_quadratic_l1(obs, source, target, edge_weight, A, l1_weight, positivity=0,
                      PFDR_rho=1.0, PFDR_condMin=1e-3, PFDR_difRcd=0.0, PFDR_difTol=1e-4,
                      PFDR_itMax=10000, verbose=0):
    """PFDR front-end with the conventions of the reference's Python binding
    (python/CP_quadratic_l1_py.cpp:7-56, 130-258, which wraps CP; this
    entry solves the same functional F(x) = 1/2 ||A x - obs||^2 + sum_e
    edge_weight |x_u - x_v| + sum_v l1_weight |x_v| directly with PFDR):
      * A scalar -> identity (its value discarded); A of shape (N,) ->
        diagonal, obs and A pre-multiplied (obs*A, A*A) as the binding does
        (:121-132); A of shape (N, V) -> the design matrix;
      * edge_weight / l1_weight: array, or scalar broadcast to every edge /
        vertex (the binding's broadcast loops run to V for both, :134-145,
        an out-of-range write for the edge weights when E > V; here each
        fills its own length);
      * source / target: any integer dtype (the binding reinterprets uint32
        as int32, :228-258);
      * defaults from :64-72 (PFDR_rho 1, condMin 1e-3, difRcd 0, difTol
        1e-4, itMax 1e4).
    Returns (x, iterations)."""
    obs = np.asarray(obs)
    if obs.dtype not in (np.float32, np.float64):
        raise TypeError("Type unknown, must be float32, float64, f4, or f8.")
    dt = obs.dtype
    A = np.asarray(A, dt)
    N = obs.size
    Eu, Ev = _edges(source, target)
    E = Eu.size
    if A.ndim == 0 or A.size == 1 and A.ndim <= 1 and N != 1:
        V, mode = N, "identity"
    elif A.ndim == 1:
        if A.size != N:
            raise ValueError("A should be either a scalar, vector of size N, or a N-by-V matrix ")
        V, mode = N, "diagonal"
    elif A.ndim == 2:
        if A.shape[0] != N:
            raise ValueError("A should be either a scalar, a vector of size N, or a N-by-V matrix ")
        V, mode = A.shape[1], "matrix"
    else:
        raise ValueError("A should be either a scalar, a vector of size N, or a N-by-V matrix ")
    ew = np.asarray(edge_weight, dt).ravel()
    ew = np.full(E, ew[0], dt) if ew.size == 1 else ew
    lw = np.asarray(l1_weight, dt).ravel()
    lw = np.full(V, lw[0], dt) if lw.size == 1 else lw
    lib = Lib()
    X0 = np.zeros(V, dt)
    if mode == "identity":
        X, it, _, _ = lib.quadratic_d1_l1(X0, obs, None, 0, Eu, Ev, ew, lw, positivity, SCAL,
                                          None, PFDR_rho, PFDR_condMin, PFDR_difRcd,
                                          PFDR_difTol, PFDR_itMax, verbose=verbose)
    elif mode == "diagonal":
        Yd = (obs * A).astype(dt)
        Ad = (A * A).astype(dt)
        X, it, _, _ = lib.quadratic_d1_l1(X0, Yd, Ad, 0, Eu, Ev, ew, lw, positivity, DIAG, Ad,
                                          PFDR_rho, PFDR_condMin, PFDR_difRcd, PFDR_difTol,
                                          PFDR_itMax, verbose=verbose)
    else:
        Af = np.asfortranarray(A)
        L = np.array([operator_norm(Af)[0]], dt)
        X, it, _, _ = lib.quadratic_d1_l1(X0, obs, Af.ravel(order="F"), N, Eu, Ev, ew, lw,
                                          positivity, SCAL, L, PFDR_rho, PFDR_condMin,
                                          PFDR_difRcd, PFDR_difTol, PFDR_itMax, verbose=verbose)
    return X, it


def proj_simplex_metric(X, M, A):
    """Column-wise metric simplex projection of the D-by-N array X
    (include/proj_simplex.hpp:33-35); M is D-by-nm, A has na entries."""
    X = np.asarray(X)
    dt = np.result_type(X, np.float32)
    D = X.shape[0]
    N = X.shape[1] if X.ndim > 1 else 1
    M = np.asarray(M, dt)
    nm = M.shape[1] if M.ndim > 1 else 1
    A = np.atleast_1d(np.asarray(A, dt))
    out = Lib().proj_simplex_metric(np.asfortranarray(X, dt).ravel(order="F"),
                                    np.asfortranarray(M, dt).ravel(order="F"),
                                    D, N, nm, A, A.size)
    return out.reshape(X.shape, order="F")


def _producers_done():
    """Device inputs are read on the library's own stream, which does not
    wait for torch's: finish the kernels torch has queued (the producers of
    the tensors handed over) before the library reads them
    (include/pfdr_mi355x.h, PFDR_MEM_DEVICE)."""
    import torch
    torch.cuda.current_stream().synchronize()


# ------------------------------------------------------------- sessions ---
class Session:
    """Device-resident solve: setup once, iterate in steps (benchmarks,
    repeated solves).  Arrays may be numpy (host) or torch CUDA tensors
    (device pointers, mem = PFDR_MEM_DEVICE)."""

    def __init__(self, kind, dtype, V, E, Eu, Ev, La_d1, X0, Y, N=0, A=None,
                 La_l1=None, positivity=0, lo=-np.inf, hi=np.inf, K=0,
                 al=0.0, Ltype=SCAL, L=None, rho=1.5, condMin=1e-3,
                 difRcd=0.0, difTol=0.0, itMax=1000, record_obj=False,
                 record_dif=False, verbose=0, device=False, nranks=0, rank=0,
                 comm=None, comm_kind=0, vtx_begin=0, V_global=0, e_global=None,
                 e_offset=0, reorder=REORDER_AUTO, evolution=EVOLUTION_AUTO,
                 vtx_label=None, spec=SPEC_AUTO):
        self.lib = load()
        ct, _, dcode = _real(dtype)
        self._keep = []
        if device:
            _producers_done()

        def addr(a, is_int=False):
            if a is None:
                return None
            if device:
                return C.c_void_p(a.data_ptr())
            a = np.ascontiguousarray(a, np.int32 if is_int else dtype)
            self._keep.append(a)
            return C.c_void_p(a.ctypes.data)

        p = Problem()
        p.kind, p.dtype = kind, dcode
        p.mem = PFDR_MEM_DEVICE if device else PFDR_MEM_HOST
        p.V, p.E, p.N, p.K = V, E, N, K
        p.X, p.Y, p.A = addr(X0), addr(Y), addr(A)
        p.Eu, p.Ev = addr(Eu, True), addr(Ev, True)
        p.La_d1, p.La_l1, p.L = addr(La_d1), addr(La_l1), addr(L)
        p.positivity, p.min, p.max, p.al = positivity, lo, hi, al
        p.Ltype = Ltype
        p.rho, p.condMin, p.difRcd, p.difTol = rho, condMin, difRcd, difTol
        p.itMax, p.verbose = itMax, verbose
        p.record_obj, p.record_dif = int(record_obj), int(record_dif)
        # 1-D vertex-range partition (see partition.py)
        p.nranks, p.rank = nranks, rank
        p.comm = comm
        p.comm_kind = comm_kind
        p.vtx_begin, p.V_global, p.e_offset = vtx_begin, V_global, e_offset
        p.reorder = reorder
        p.evolution = evolution
        p.spec = spec
        if vtx_label is not None:
            vl = np.ascontiguousarray(vtx_label, np.int64)
            self._keep.append(vl)
            p.vtx_label = C.c_void_p(vl.ctypes.data)
        if e_global is not None:
            eg = np.ascontiguousarray(e_global, np.int64)
            self._keep.append(eg)
            p.e_global = C.c_void_p(eg.ctypes.data)
        self.problem = p
        self.dtype = np.dtype(dtype)
        self.V, self.K = V, max(K, 1)
        self.itMax = itMax
        self.record_obj, self.record_dif = record_obj, record_dif
        h = C.c_void_p()
        _check(self.lib.pfdr_session_create(C.byref(h), C.byref(p)),
               "pfdr_session_create")
        self.h = h

    def run(self, iters):
        it = C.c_int(0)
        _check(self.lib.pfdr_session_run(self.h, C.c_int(iters), C.byref(it)),
               "pfdr_session_run")
        return it.value

    def sync(self):
        _check(self.lib.pfdr_session_sync(self.h), "pfdr_session_sync")

    def prepare(self, iters):
        """capture the hipGraphs run(iters) will replay (no iteration runs)"""
        _check(self.lib.pfdr_session_prepare(self.h, C.c_int(int(iters))), "pfdr_session_prepare")

    def profile(self, on=True, period=1, only=None):
        """time kernels with HIP events: every `period`-th launch, of the
        kernels named in `only` (all when None)"""
        _check(self.lib.pfdr_session_profile_filter(
            self.h, None if not only else ",".join(only).encode()), "pfdr_session_profile_filter")
        _check(self.lib.pfdr_session_set_profiling(
            self.h, C.c_int(0 if not on else max(int(period), 1))), "pfdr_session_set_profiling")

    def kernel_stats(self, name):
        n, ms = C.c_int(0), C.c_double(0.0)
        _check(self.lib.pfdr_session_kernel_stats(
            self.h, name.encode(), C.byref(n), C.byref(ms)),
            "pfdr_session_kernel_stats")
        return n.value, ms.value

    def query(self, what):
        v = C.c_int64(0)
        _check(self.lib.pfdr_session_query(self.h, what.encode(), C.byref(v)),
               "pfdr_session_query")
        return v.value

    def device_bytes(self):
        return int(self.lib.pfdr_session_device_bytes(self.h))

    def result(self):
        X = np.zeros(self.V * self.K, self.dtype)
        it = C.c_int(0)
        Obj = np.zeros(self.itMax + 1, self.dtype) if self.record_obj else None
        Dif = np.zeros(max(self.itMax, 1), self.dtype) if self.record_dif else None
        _check(self.lib.pfdr_session_result(
            self.h, C.c_void_p(X.ctypes.data), C.byref(it),
            None if Obj is None else C.c_void_p(Obj.ctypes.data),
            None if Dif is None else C.c_void_p(Dif.ctypes.data)),
            "pfdr_session_result")
        return X, it.value, Obj, Dif

    def close(self):
        if getattr(self, "h", None):
            self.lib.pfdr_session_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------ device group ----
def set_devices(devices, min_vertices=-1):
    """Partition this process's drop-in calls (Lib, and any CP / C++ caller of
    the library) across `devices` (a list of device ids; [] = one GPU): one
    host thread per device, RCCL over xGMI, bit-identical to one GPU.  Calls
    below min_vertices vertices (< 0: 2^20) stay on one GPU.  A list repeating
    one device runs the ranks as threads on it (loopback; tests)."""
    devs = [int(d) for d in devices]
    arr = (C.c_int * max(len(devs), 1))(*devs)
    lib = load()
    lib.pfdr_set_devices.argtypes = [C.c_int, C.c_void_p, C.c_int64]
    _check(lib.pfdr_set_devices(len(devs), arr if devs else None, int(min_vertices)),
           "pfdr_set_devices")


# ------------------------------------------------------- native inputs ----
def gen_knn_jitter_grid(shape, k=6, seed=6, jitter=0.25, v_range=None):
    """Native twin of graphs.knn_jitter_grid (multi-threaded C++)."""
    nx, ny, nz = shape
    V = nx * ny * nz
    v0, v1 = (0, V) if v_range is None else v_range
    n = (v1 - v0) * k
    Eu = np.empty(n, np.int32)
    Ev = np.empty(n, np.int32)
    got = load().pfdr_gen_knn_jitter_grid(nx, ny, nz, k, seed, jitter, v0, v1,
                                          Eu.ctypes.data, Ev.ctypes.data)
    if got != n:
        raise PFDRError("pfdr_gen_knn_jitter_grid failed")
    return Eu, Ev


def gen_grid_edges(shape, conn, v_range=None):
    nx, ny = shape[0], shape[1]
    nz = shape[2] if len(shape) > 2 else 1
    V = nx * ny * nz
    v0, v1 = (0, V) if v_range is None else v_range
    lib = load()
    n = lib.pfdr_gen_grid_edges(nx, ny, nz, conn, v0, v1, None, None)
    if n < 0:
        raise PFDRError("pfdr_gen_grid_edges: unsupported connectivity")
    Eu = np.empty(n, np.int32)
    Ev = np.empty(n, np.int32)
    lib.pfdr_gen_grid_edges(nx, ny, nz, conn, v0, v1, Eu.ctypes.data,
                            Ev.ctypes.data)
    return Eu, Ev


def gram(A, which=0, device=False):
    """G = A^t A (which = 0) or A A^t (which = 1) on the matrix cores.
    A: (M, N) numpy array (any order; treated as the matrix) or, with
    device=True, a torch CUDA tensor holding the column-major M-by-N matrix
    as a (N, M) contiguous tensor.  Returns (G, kernel_ms)."""
    lib = load()
    ms = C.c_double(0.0)
    if device:
        import torch
        _producers_done()
        N, M = A.shape
        P = N if which == 0 else M
        G = torch.empty((P, P), dtype=A.dtype, device=A.device)
        fn = lib.pfdr_gram_f32 if A.dtype == torch.float32 else lib.pfdr_gram_f64
        _check(fn(which, M, N, C.c_void_p(A.data_ptr()), PFDR_MEM_DEVICE,
                  C.c_void_p(G.data_ptr()), C.byref(ms)), "pfdr_gram")
        return G, ms.value
    A = np.asarray(A)
    M, N = A.shape
    Af = np.asfortranarray(A)
    ct, sfx, _ = _real(Af.dtype)
    P = N if which == 0 else M
    G = np.empty((P, P), Af.dtype, order="F")
    _check(getattr(lib, "pfdr_gram_" + sfx)(which, M, N, C.c_void_p(Af.ctypes.data),
                                             PFDR_MEM_HOST, C.c_void_p(G.ctypes.data),
                                             C.byref(ms)), "pfdr_gram")
    return np.ascontiguousarray(G), ms.value


def sequential_sum(a, seed=0.0, method=0):
    """seed + a[0] + ... + a[n-1] rounded as the one-thread loop, for
    nonnegative terms (the preconditioner's amplitude sum).  method 0: the
    workgroup binade scan the solvers use, 1: one lane.  Returns (sum, ms)."""
    lib = load()
    a = np.ascontiguousarray(a)
    ct, sfx, _ = _real(a.dtype)
    fn = getattr(lib, "pfdr_sequential_sum_" + sfx)
    fn.argtypes = [C.c_int64, C.c_void_p, C.c_int, ct, C.c_int, C.c_void_p, C.c_void_p]
    out, ms = ct(0), C.c_double(0.0)
    _check(fn(a.size, C.c_void_p(a.ctypes.data) if a.size else None, PFDR_MEM_HOST, ct(seed),
              method, C.byref(out), C.byref(ms)), "pfdr_sequential_sum")
    return a.dtype.type(out.value), ms.value


def operator_norm(A, nTol=1e-3, itMax=100, nbInit=10, symmetric=False, device=False,
                  M=None, N=None, verbose=0):
    """||A||^2 (reference operator_norm_matrix).  symmetric=True: A is the
    S-by-S A^tA / AA^t itself (the reference's M or N = 0).  device=True: A
    is a torch CUDA tensor, column-major M-by-N stored as (N, M).  Returns
    (norm2, gram_ms)."""
    lib = load()
    gms = C.c_double(0.0)
    if device:
        import torch
        _producers_done()
        Nn, Mm = A.shape
        if symmetric:
            Mm, Nn = 0, Nn
        ct = C.c_float if A.dtype == torch.float32 else C.c_double
        fn = lib.pfdr_operator_norm_f32 if A.dtype == torch.float32 else lib.pfdr_operator_norm_f64
        out = ct(0)
        _check(fn(Mm, Nn, C.c_void_p(A.data_ptr()), PFDR_MEM_DEVICE, ct(nTol), itMax, nbInit,
                  verbose, C.byref(out), C.byref(gms)), "pfdr_operator_norm")
        return out.value, gms.value
    A = np.asarray(A)
    Af = np.asfortranarray(A)
    ct, sfx, _ = _real(Af.dtype)
    Mm, Nn = (0, A.shape[0]) if symmetric else A.shape
    out = ct(0)
    _check(getattr(lib, "pfdr_operator_norm_" + sfx)(Mm, Nn, C.c_void_p(Af.ctypes.data),
                                                      PFDR_MEM_HOST, ct(nTol), itMax, nbInit,
                                                      verbose, C.byref(out), C.byref(gms)),
           "pfdr_operator_norm")
    return out.value, gms.value


def cp_reduce(N, A, Y, comp_ptr, comp_vertices, preAt=True, normTol=1e-3, normItMax=100,
              normNbInit=10):
    """CP reduced-problem builder (pfdr_cp_reduce_*): A is (N, V) for
    N > 0 (or (V, V) A^tA for N < 0, length-V diagonal / None for N = 0),
    comp_ptr (rV + 1) and comp_vertices (V) the components.  Returns dict
    rA, rAA, rY, L, Leq (None where not formed)."""
    Y = np.asarray(Y)
    dt = Y.dtype
    ct, sfx, _ = _real(dt)
    ptr = np.ascontiguousarray(comp_ptr, np.int32)
    Vc = np.ascontiguousarray(comp_vertices, np.int32)
    rV, V = ptr.size - 1, Vc.size
    Af = None
    if A is not None:
        Af = np.asfortranarray(np.asarray(A, dt)) if np.ndim(A) == 2 else np.ascontiguousarray(A, dt)
    if N <= 0:
        preAt = True
    rA = np.zeros((rV, N), dt) if N > 0 else None        # column rv = rA[rv]
    rAA = (np.zeros(rV, dt) if N == 0 else np.zeros((rV, rV), dt)) if preAt else None
    rY = np.zeros(rV, dt) if preAt else None
    L = np.zeros(rV, dt)
    Leq = np.zeros(rV, dt) if N != 0 else None
    p = lambda a: None if a is None else C.c_void_p(a.ctypes.data)
    _check(getattr(load(), "pfdr_cp_reduce_" + sfx)(
        C.c_int(N), C.c_int(V), p(Af), p(np.ascontiguousarray(Y)), C.c_int(rV), p(ptr), p(Vc),
        C.c_int(int(preAt)), PFDR_MEM_HOST, ct(normTol), C.c_int(normItMax),
        C.c_int(normNbInit), p(rA), p(rAA), p(rY), p(L), p(Leq)), "pfdr_cp_reduce")
    return {"rA": None if rA is None else rA.T, "rAA": rAA, "rY": rY, "L": L, "Leq": Leq}


class CPGraph:
    """Device-resident cut-pursuit graph (pfdr_cpgraph_*, SURVEY.md §8(f)
    ranks 2-3): the full-graph steps of every CP iteration of
    src/CP_PFDR_graph_quadratic_d1_l1.cpp with the reference's results and
    orders.  Arrays in and out are numpy (host); the maxflow between
    ``capacities`` and ``activate`` is the caller's."""

    def __init__(self, V, Eu, Ev, La_d1, La_l1=None):
        La_d1 = np.asarray(La_d1)
        self.dtype = La_d1.dtype
        self.ct, _, code = _real(self.dtype)
        self.V = int(V)
        Eu, Ev = _edges(Eu, Ev)
        self.E = Eu.size
        La_d1 = _arr(La_d1, self.dtype)
        La_l1 = _arr(La_l1, self.dtype)
        self._keep = (Eu, Ev, La_d1, La_l1)
        self.h = C.c_void_p()
        p = lambda a: None if a is None else C.c_void_p(a.ctypes.data)
        _check(load().pfdr_cpgraph_create(C.byref(self.h), code, C.c_int(self.V),
                                          C.c_int(self.E), p(Eu), p(Ev), p(La_d1), p(La_l1),
                                          PFDR_MEM_HOST), "pfdr_cpgraph_create")
        self.has_l1 = La_l1 is not None
        self.rV = 1

    @staticmethod
    def _p(a):
        return None if a is None else C.c_void_p(a.ctypes.data)

    def _call(self, name, *args):
        _check(getattr(load(), name)(self.h, *args), name)

    def set_active(self, active):
        a = np.ascontiguousarray(active, np.uint8)
        self._call("pfdr_cpgraph_set_active", self._p(a), PFDR_MEM_HOST)

    def active(self):
        a = np.empty(self.E, np.uint8)
        self._call("pfdr_cpgraph_get_active", self._p(a), PFDR_MEM_HOST)
        return a

    def set_components(self, Cv, Vc, rVc):
        Cv, Vc, rVc = (np.ascontiguousarray(x, np.int32) for x in (Cv, Vc, rVc))
        self.rV = rVc.size - 1
        self._call("pfdr_cpgraph_set_components", C.c_int(self.rV), self._p(Cv), self._p(Vc),
                   self._p(rVc), PFDR_MEM_HOST)

    def components(self):
        """:566-597 -> (Cv, Vc, rVc)"""
        rV = C.c_int()
        self._call("pfdr_cpgraph_components", C.byref(rV))
        self.rV = rV.value
        Cv = np.empty(self.V, np.int32)
        Vc = np.empty(self.V, np.int32)
        rVc = np.empty(self.rV + 1, np.int32)
        self._call("pfdr_cpgraph_get_components", None, self._p(Cv), self._p(Vc), self._p(rVc),
                   PFDR_MEM_HOST)
        return Cv, Vc, rVc

    def set_values(self, rX):
        x = np.ascontiguousarray(rX, self.dtype)
        self._call("pfdr_cpgraph_set_values", self._p(x), PFDR_MEM_HOST)

    def reduced_graph(self, eps):
        """:599-661 -> (rEu, rEv, rLa_d1, rLa_l1 or None)"""
        rE = C.c_int()
        self._call("pfdr_cpgraph_reduced_graph", C.c_double(eps), C.byref(rE))
        n = rE.value
        rEu = np.empty(n, np.int32)
        rEv = np.empty(n, np.int32)
        rLa = np.empty(n, self.dtype)
        rL1 = np.empty(self.rV, self.dtype) if self.has_l1 else None
        self._call("pfdr_cpgraph_get_reduced", self._p(rEu), self._p(rEv), self._p(rLa),
                   self._p(rL1), PFDR_MEM_HOST)
        return rEu, rEv, rLa, rL1

    def merge(self, eps, difTol):
        """:863-886 -> number of deactivated edges"""
        n = C.c_int()
        self._call("pfdr_cpgraph_merge", C.c_double(eps), C.c_double(difTol), C.byref(n))
        return n.value

    def gradient(self, N=0, A=None, Y=None, R=None):
        """:339-413 -> DfS[V]"""
        Af = None
        if A is not None:
            Af = (np.asfortranarray(np.asarray(A, self.dtype)) if np.ndim(A) == 2
                  else np.ascontiguousarray(A, self.dtype))
        Y = _arr(Y, self.dtype)
        R = _arr(R, self.dtype)
        DfS = np.empty(self.V, self.dtype)
        self._call("pfdr_cpgraph_gradient", C.c_int(N), self._p(Af), self._p(Y), self._p(R),
                   PFDR_MEM_HOST, self._p(DfS))
        return DfS

    def capacities(self, cut, positivity=0):
        """:402-535 -> (tr_cap[V], r_cap[E]) of cut 0 (differentiable), 1 or 2"""
        tr = np.empty(self.V, self.dtype)
        rc = np.empty(self.E, self.dtype)
        self._call("pfdr_cpgraph_capacities", C.c_int(cut), C.c_int(int(positivity)),
                   self._p(tr), self._p(rc), PFDR_MEM_HOST)
        return tr, rc

    def capacities_bounds(self, cut, lo=-np.inf, hi=np.inf):
        """bounds driver (src/CP_PFDR_graph_quadratic_d1_bounds.cpp:386-534)
        -> (tr_cap[V], r_cap[E]) of cut 0 (no bound), 1 or 2"""
        tr = np.empty(self.V, self.dtype)
        rc = np.empty(self.E, self.dtype)
        self._call("pfdr_cpgraph_capacities_bounds", C.c_int(cut), C.c_double(lo),
                   C.c_double(hi), self._p(tr), self._p(rc), PFDR_MEM_HOST)
        return tr, rc

    def activate(self, segment):
        """activate the inactive edges the cut separates -> how many"""
        seg = np.ascontiguousarray(segment, np.uint8)
        n = C.c_int()
        self._call("pfdr_cpgraph_activate", self._p(seg), PFDR_MEM_HOST, C.byref(n))
        return n.value

    # ---- the duplex driver's two-layer cut (src/CP_PFDR_graph_quadratic_d1_l1_duplex.cpp)
    def capacities_duplex(self, positivity=0):
        """:469-527 -> (tr_cap[2V]: v1 then v2 nodes, r_link[V], r_cap[E])"""
        tr = np.empty(2 * self.V, self.dtype)
        link = np.empty(self.V, self.dtype)
        rc = np.empty(self.E, self.dtype)
        self._call("pfdr_cpgraph_capacities_duplex", C.c_int(int(positivity)), self._p(tr),
                   self._p(link), self._p(rc), PFDR_MEM_HOST)
        return tr, link, rc

    def activate_duplex(self, segment):
        """:531-545, segment[2V] -> how many edges were activated"""
        seg = np.ascontiguousarray(segment, np.uint8)
        if seg.size != 2 * self.V:
            raise ValueError("segment must hold 2V entries")
        n = C.c_int()
        self._call("pfdr_cpgraph_activate_duplex", self._p(seg), PFDR_MEM_HOST, C.byref(n))
        return n.value

    # ---- the simplex driver (src/CP_PFDR_graph_loss_d1_simplex.cpp); P
    # layouts vertex-major [v*K + k]
    def simplex_setup(self, K, al, Q):
        """K labels, loss al (0 linear, 1 quadratic, else smoothed KL), Q[V*K]"""
        self.K = int(K)
        self.al = float(al)
        self._Q = np.ascontiguousarray(Q, self.dtype).reshape(-1)
        if self._Q.size != self.V * self.K:
            raise ValueError("Q must hold V*K values")
        self._call("pfdr_cpgraph_simplex_setup", C.c_int(self.K), C.c_double(self.al),
                   self._p(self._Q), PFDR_MEM_HOST)

    def simplex_observations(self):
        """:733-766 -> (rP[rV*K], rQ[rV*K], rLa_f[rV] or None when al == 0);
        rP becomes the component values"""
        n = self.rV * self.K
        rP = np.empty(n, self.dtype)
        rQ = np.empty(n, self.dtype)
        rLa_f = np.empty(self.rV, self.dtype) if self.al != 0 else None
        self._call("pfdr_cpgraph_simplex_observations", self._p(rP), self._p(rQ),
                   self._p(rLa_f), PFDR_MEM_HOST)
        return rP, rQ, rLa_f

    def simplex_set_values(self, rP):
        x = np.ascontiguousarray(rP, self.dtype).reshape(-1)
        if x.size != self.rV * self.K:
            raise ValueError("rP must hold rV*K values")
        self._call("pfdr_cpgraph_simplex_set_values", self._p(x), PFDR_MEM_HOST)

    def simplex_gradient(self, eps):
        """:327-376, :525-536 -> (DfS[V*K], rDi[rV])"""
        DfS = np.empty(self.V * self.K, self.dtype)
        rDi = np.empty(self.rV, np.int32)
        self._call("pfdr_cpgraph_simplex_gradient", C.c_double(eps), self._p(DfS),
                   rDi.ctypes.data_as(C.POINTER(C.c_int)), PFDR_MEM_HOST)
        return DfS, rDi

    def simplex_capacities(self, n):
        """:542-595 -> (tr_cap[V], r_cap[E] of arc 2e; arc 2e + 1 has none)"""
        tr = np.empty(self.V, self.dtype)
        rc = np.empty(self.E, self.dtype)
        self._call("pfdr_cpgraph_simplex_capacities", C.c_int(n), self._p(tr), self._p(rc),
                   PFDR_MEM_HOST)
        return tr, rc

    def simplex_expand(self, n, segment):
        seg = np.ascontiguousarray(segment, np.uint8)
        self._call("pfdr_cpgraph_simplex_expand", C.c_int(n), self._p(seg), PFDR_MEM_HOST)

    def simplex_labels(self):
        D = np.empty(self.V, np.int32)
        self._call("pfdr_cpgraph_simplex_labels", D.ctypes.data_as(C.POINTER(C.c_int)),
                   PFDR_MEM_HOST)
        return D

    def simplex_activate(self):
        n = C.c_int()
        self._call("pfdr_cpgraph_simplex_activate", C.byref(n))
        return n.value

    def simplex_merge(self, eps):
        n = C.c_int()
        self._call("pfdr_cpgraph_simplex_merge", C.c_double(eps), C.byref(n))
        return n.value

    def close(self):
        if self.h:
            load().pfdr_cpgraph_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def grid_edge_count(shape, conn, v_end):
    """Edges gen_grid_edges emits for the vertices [0, v_end) (the global id
    of a slab's first edge)."""
    nx, ny = shape[0], shape[1]
    nz = shape[2] if len(shape) > 2 else 1
    n = load().pfdr_gen_grid_edges(nx, ny, nz, conn, 0, v_end, None, None)
    if n < 0:
        raise PFDRError("pfdr_gen_grid_edges: unsupported connectivity")
    return int(n)


def gen_piecewise(nx, V, seed, dtype=np.float32, noise=0.2, v_range=None):
    v0, v1 = (0, V) if v_range is None else v_range
    Y = np.empty(v1 - v0, dtype)
    fn = (load().pfdr_gen_piecewise_f32 if np.dtype(dtype) == np.float32
          else load().pfdr_gen_piecewise_f64)
    fn(nx, seed, noise, v0, v1, Y.ctypes.data)
    return Y


def _gen_fn(name, dtype):
    _, sfx, _ = _real(dtype)
    return getattr(load(), "pfdr_gen_%s_%s" % (name, sfx))


def gen_uniform(seed, n, lo, hi, dtype=np.float32, i0=0, out=None):
    """out[i] = lo + (hi - lo) U(seed, i0 + i) (native, multi-threaded)."""
    out = np.empty(n, dtype) if out is None else out
    fn = _gen_fn("uniform", out.dtype)
    fn.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_double, C.c_double, C.c_void_p]
    _check(fn(seed, i0, n, lo, hi, out.ctypes.data), "pfdr_gen_uniform")
    return out


def gen_matvec(A_cm, N, V, x):
    """y = A x for the column-major N-by-V matrix held in A_cm (length N V),
    each row summed in double in increasing column order (deterministic)."""
    y = np.empty(N, A_cm.dtype)
    x = np.ascontiguousarray(x, A_cm.dtype)
    fn = _gen_fn("matvec", A_cm.dtype)
    fn.argtypes = [C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
    _check(fn(N, V, A_cm.ctypes.data, x.ctypes.data, y.ctypes.data), "pfdr_gen_matvec")
    return y


def gen_symmetric(V, seed, s, d, dtype=np.float32):
    """Symmetric diagonally dominant V-by-V matrix (flat, column-major)."""
    G = np.empty(V * V, dtype)
    fn = _gen_fn("symmetric", dtype)
    fn.argtypes = [C.c_int64, C.c_uint64, C.c_double, C.c_double, C.c_void_p]
    _check(fn(V, seed, s, d, G.ctypes.data), "pfdr_gen_symmetric")
    return G
