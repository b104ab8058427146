"""TEST INFRASTRUCTURE ONLY — ctypes front-end of the CPU oracle.

Two back-ends with one calling convention (numpy in, numpy out):

* ``Oracle("port")``  -> ``oracle/liboracle_pfdr.so``, the clean-room C
  restatement (``oracle/pfdr_oracle_body.h``), single-threaded;
* ``Oracle("ref")``   -> ``oracle/_ref/libpfdr_ref_seq.so``, the REFERENCE
  sources compiled without OpenMP (bit-exact pin of the restatement);
* ``Oracle("ref_omp")`` -> ``oracle/_ref/libpfdr_ref_omp.so``, the reference
  with its OpenMP loops (CPU baseline timing only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product package never does.

The argument lists mirror the reference functions
(include/PFDR_graph_quadratic_d1_l1.hpp:36-42,
 include/PFDR_graph_quadratic_d1_bounds.hpp:34-40,
 include/PFDR_graph_loss_d1_simplex.hpp:24-30,
 include/proj_simplex.hpp:33-35) minus ``verbose``; outputs follow the MEX
wrappers (octave/mex/PFDR_*_mex.cpp): X (or P), it, Obj[itMax+1], Dif[itMax].
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIBS = {
    "port": (os.path.join(HERE, "liboracle_pfdr.so"), "oracle_"),
    "ref": (os.path.join(HERE, "_ref", "libpfdr_ref_seq.so"), "ref_"),
    "ref_omp": (os.path.join(HERE, "_ref", "libpfdr_ref_omp.so"), "ref_"),
}
_CACHE = {}


def build(ref=True):
    """Compile the restatement (and, where /root/reference exists, _ref)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    if ref:
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def available(kind):
    return os.path.exists(_LIBS[kind][0])


def _ptr(a, ct):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ct))


def _real(dtype):
    dtype = np.dtype(dtype)
    if dtype == np.float32:
        return C.c_float, "f32"
    if dtype == np.float64:
        return C.c_double, "f64"
    raise TypeError("oracle supports float32/float64 only, got %s" % dtype)


class Oracle:
    def __init__(self, kind="port"):
        path, prefix = _LIBS[kind]
        if path not in _CACHE:
            if not os.path.exists(path):
                raise FileNotFoundError(
                    "%s missing: run `make -C oracle %s`" %
                    (path, "ref" if kind != "port" else "all"))
            _CACHE[path] = C.CDLL(path)
        self.lib = _CACHE[path]
        self.prefix = prefix
        self.kind = kind

    def _fn(self, name, sfx):
        return getattr(self.lib, "%s%s_%s" % (self.prefix, name, sfx))

    # ---------------------------------------------------------------- l1 --
    def quadratic_d1_l1(self, X0, Y, A, N, Eu, Ev, La_d1, La_l1=None,
                        positivity=0, Ltype=0, L=None, rho=1.5, condMin=1e-3,
                        difRcd=0.0, difTol=1e-5, itMax=1000, obj=False,
                        dif=False):
        X = np.array(X0, copy=True)
        ct, sfx = _real(X.dtype)
        V, E = X.size, Eu.size
        Obj = np.zeros(itMax + 1, X.dtype) if obj else None
        Dif = np.zeros(max(itMax, 1), X.dtype) if dif else None
        it = C.c_int(0)
        fn = self._fn("pfdr_quadratic_d1_l1", sfx)
        fn(C.c_int(V), C.c_int(E), C.c_int(N), _ptr(X, ct), _ptr(Y, ct),
           _ptr(A, ct), _ptr(Eu, C.c_int), _ptr(Ev, C.c_int),
           _ptr(La_d1, ct), _ptr(La_l1, ct), C.c_int(positivity),
           C.c_int(Ltype), _ptr(L, ct), ct(rho), ct(condMin), ct(difRcd),
           ct(difTol), C.c_int(itMax), C.byref(it), _ptr(Obj, ct),
           _ptr(Dif, ct))
        return X, it.value, Obj, Dif

    # ------------------------------------------------------------ bounds --
    def quadratic_d1_bounds(self, X0, Y, A, N, Eu, Ev, La_d1, lo=-np.inf,
                            hi=np.inf, Ltype=0, L=None, rho=1.5,
                            condMin=1e-3, difRcd=0.0, difTol=1e-5,
                            itMax=1000, obj=False, dif=False):
        X = np.array(X0, copy=True)
        ct, sfx = _real(X.dtype)
        V, E = X.size, Eu.size
        Obj = np.zeros(itMax + 1, X.dtype) if obj else None
        Dif = np.zeros(max(itMax, 1), X.dtype) if dif else None
        it = C.c_int(0)
        fn = self._fn("pfdr_quadratic_d1_bounds", sfx)
        fn(C.c_int(V), C.c_int(E), C.c_int(N), _ptr(X, ct), _ptr(Y, ct),
           _ptr(A, ct), _ptr(Eu, C.c_int), _ptr(Ev, C.c_int),
           _ptr(La_d1, ct), ct(lo), ct(hi), C.c_int(Ltype), _ptr(L, ct),
           ct(rho), ct(condMin), ct(difRcd), ct(difTol), C.c_int(itMax),
           C.byref(it), _ptr(Obj, ct), _ptr(Dif, ct))
        return X, it.value, Obj, Dif

    # ----------------------------------------------------------- simplex --
    def loss_d1_simplex(self, P0, Q, K, Eu, Ev, La_d1, al=0.1, La_f=None,
                        rho=1.0, condMin=0.1, difRcd=0.0, difTol=1e-4,
                        itMax=1000, obj=False, dif=False):
        P = np.array(P0, copy=True)
        ct, sfx = _real(P.dtype)
        V, E = P.size // K, Eu.size
        Obj = np.zeros(itMax + 1, P.dtype) if obj else None
        Dif = np.zeros(max(itMax, 1), P.dtype) if dif else None
        it = C.c_int(0)
        fn = self._fn("pfdr_loss_d1_simplex", sfx)
        fn(C.c_int(K), C.c_int(V), C.c_int(E), ct(al), _ptr(La_f, ct),
           _ptr(P, ct), _ptr(Q, ct), _ptr(Eu, C.c_int), _ptr(Ev, C.c_int),
           _ptr(La_d1, ct), ct(rho), ct(condMin), ct(difRcd), ct(difTol),
           C.c_int(itMax), C.byref(it), _ptr(Obj, ct), _ptr(Dif, ct))
        return P, it.value, Obj, Dif

    def proj_simplex_metric(self, X0, M, D, N, nm, A, na):
        X = np.array(X0, copy=True)
        ct, sfx = _real(X.dtype)
        fn = self._fn("proj_simplex_metric", sfx)
        fn(_ptr(X, ct), _ptr(M, ct), C.c_int(D), C.c_int(N), C.c_int(nm),
           _ptr(A, ct), C.c_int(na))
        return X

    # ------------------------------------------------- operator norm --
    def operator_norm(self, A, M, N, nTol=1e-3, itMax=100, nbInit=10):
        """The reference's operator_norm_matrix (OpenMP build only: its
        source calls omp_* unguarded); A column-major M-by-N (M or N = 0:
        symmetric).  Time-seeded starts: an estimate, not a fixed value."""
        if self.kind != "ref_omp":
            raise NotImplementedError("operator norm: reference OpenMP build only")
        A = np.ascontiguousarray(A)
        ct, sfx = _real(A.dtype)
        fn = self._fn("operator_norm", sfx)
        fn.restype = ct
        return float(fn(C.c_int(M), C.c_int(N), _ptr(A, ct), ct(nTol), C.c_int(itMax),
                        C.c_int(nbInit)))

    # ------------------------------------------- CP reduced problem --
    def cp_reduce(self, N, A, Y, comp_ptr, comp_vertices, preAt=True):
        """oracle/cp_reduce_body.h (port only): rA, rAA, rY, Leq as the
        reference's CP forms them, without the operator norm."""
        if self.kind != "port":
            raise NotImplementedError("cp_reduce: C restatement only")
        Y = np.ascontiguousarray(Y)
        ct, sfx = _real(Y.dtype)
        ptr = np.ascontiguousarray(comp_ptr, np.int32)
        Vc = np.ascontiguousarray(comp_vertices, np.int32)
        rV, V = ptr.size - 1, Vc.size
        Af = None
        if A is not None:
            Af = (np.asfortranarray(np.asarray(A, Y.dtype)) if np.ndim(A) == 2
                  else np.ascontiguousarray(A, Y.dtype))
        if N <= 0:
            preAt = True
        rA = np.zeros((rV, N), Y.dtype) if N > 0 else None
        rAA = (np.zeros(rV, Y.dtype) if N == 0 else np.zeros((rV, rV), Y.dtype)) if preAt else None
        rY = np.zeros(rV, Y.dtype) if preAt else None
        Leq = np.zeros(rV, Y.dtype)
        fn = self._fn("cp_reduce", sfx)
        fn(C.c_int(N), C.c_int(V), _ptr(Af, ct), _ptr(Y, ct), C.c_int(rV),
           _ptr(ptr, C.c_int), _ptr(Vc, C.c_int), C.c_int(int(preAt)), _ptr(rA, ct),
           _ptr(rAA, ct), _ptr(rY, ct), _ptr(Leq, ct))
        return {"rA": None if rA is None else rA.T, "rAA": rAA, "rY": rY,
                "Leq": Leq if N != 0 else None}

    # ------------------------------------------------ CP graph steps --
    # oracle/cp_graph_body.h (port only), SURVEY.md §8(f) ranks 2-3.
    def _port_only(self, what):
        if self.kind != "port":
            raise NotImplementedError("%s: C restatement only" % what)

    def cp_components(self, V, Eu, Ev, active):
        """:566-597 -> (Cv, Vc, rVc)"""
        self._port_only("cp_components")
        Eu = np.ascontiguousarray(Eu, np.int32)
        Ev = np.ascontiguousarray(Ev, np.int32)
        act = np.ascontiguousarray(active, np.uint8)
        Cv = np.empty(V, np.int32)
        Vc = np.empty(V, np.int32)
        rVc = np.empty(V + 1, np.int32)
        fn = self.lib.oracle_cp_components
        fn.restype = C.c_int
        rV = fn(C.c_int(V), C.c_int(Eu.size), _ptr(Eu, C.c_int), _ptr(Ev, C.c_int),
                _ptr(act, C.c_uint8), _ptr(Cv, C.c_int), _ptr(Vc, C.c_int), _ptr(rVc, C.c_int))
        return Cv, Vc, rVc[:rV + 1].copy()

    def cp_activate(self, Eu, Ev, segment, active):
        """:430-440 / :521-556 -> (new active, count)"""
        self._port_only("cp_activate")
        Eu = np.ascontiguousarray(Eu, np.int32)
        Ev = np.ascontiguousarray(Ev, np.int32)
        seg = np.ascontiguousarray(segment, np.uint8)
        act = np.array(active, np.uint8, copy=True)
        fn = self.lib.oracle_cp_activate
        fn.restype = C.c_int
        w = fn(C.c_int(Eu.size), _ptr(Eu, C.c_int), _ptr(Ev, C.c_int), _ptr(seg, C.c_uint8),
               _ptr(act, C.c_uint8))
        return act, int(w)

    def cp_reduced_graph(self, V, Eu, Ev, La_d1, La_l1, active, Cv, Vc, rVc, eps):
        """:599-661 -> (rEu, rEv, rLa_d1, rLa_l1)"""
        self._port_only("cp_reduced_graph")
        La_d1 = np.ascontiguousarray(La_d1)
        ct, sfx = _real(La_d1.dtype)
        Eu = np.ascontiguousarray(Eu, np.int32)
        Ev = np.ascontiguousarray(Ev, np.int32)
        L1 = None if La_l1 is None else np.ascontiguousarray(La_l1, La_d1.dtype)
        act = np.ascontiguousarray(active, np.uint8)
        Cv = np.ascontiguousarray(Cv, np.int32)
        Vc = np.ascontiguousarray(Vc, np.int32)
        rVc = np.ascontiguousarray(rVc, np.int32)
        rV, E = rVc.size - 1, Eu.size
        rEu = np.empty(E + rV, np.int32)
        rEv = np.empty(E + rV, np.int32)
        rLa = np.empty(E + rV, La_d1.dtype)
        rL1 = None if L1 is None else np.empty(rV, La_d1.dtype)
        fn = self._fn("cp_reduced_graph", sfx)
        fn.restype = C.c_int
        rE = fn(C.c_int(V), C.c_int(E), _ptr(Eu, C.c_int), _ptr(Ev, C.c_int), _ptr(La_d1, ct),
                _ptr(L1, ct), _ptr(act, C.c_uint8), _ptr(Cv, C.c_int), _ptr(Vc, C.c_int),
                _ptr(rVc, C.c_int), C.c_int(rV), ct(eps), _ptr(rEu, C.c_int), _ptr(rEv, C.c_int),
                _ptr(rLa, ct), _ptr(rL1, ct))
        return rEu[:rE].copy(), rEv[:rE].copy(), rLa[:rE].copy(), rL1

    def cp_merge(self, Eu, Ev, Cv, rX, eps, difTol, active):
        """:863-886 -> (new active, deactivated count)"""
        self._port_only("cp_merge")
        rX = np.ascontiguousarray(rX)
        ct, sfx = _real(rX.dtype)
        Eu = np.ascontiguousarray(Eu, np.int32)
        Ev = np.ascontiguousarray(Ev, np.int32)
        Cv = np.ascontiguousarray(Cv, np.int32)
        act = np.array(active, np.uint8, copy=True)
        fn = self._fn("cp_merge", sfx)
        fn.restype = C.c_int
        n = fn(C.c_int(Eu.size), _ptr(Eu, C.c_int), _ptr(Ev, C.c_int), _ptr(Cv, C.c_int),
               _ptr(rX, ct), ct(eps), ct(difTol), _ptr(act, C.c_uint8))
        return act, int(n)

    def cp_gradient(self, N, V, A, Y, R, Eu, Ev, La_d1, La_l1, active, Cv, Vc, rVc, rX):
        """:339-400 -> DfS[V] (A: N-by-V for N > 0, V-by-V A^tA for N < 0,
        diagonal or None for N = 0; all column major)"""
        self._port_only("cp_gradient")
        rX = np.ascontiguousarray(rX)
        dt = rX.dtype
        ct, sfx = _real(dt)
        Af = None
        if A is not None:
            Af = (np.asfortranarray(np.asarray(A, dt)) if np.ndim(A) == 2
                  else np.ascontiguousarray(A, dt))
        Y = np.ascontiguousarray(Y, dt)
        R = None if R is None else np.ascontiguousarray(R, dt)
        Eu = np.ascontiguousarray(Eu, np.int32)
        Ev = np.ascontiguousarray(Ev, np.int32)
        La_d1 = np.ascontiguousarray(La_d1, dt)
        L1 = None if La_l1 is None else np.ascontiguousarray(La_l1, dt)
        act = np.ascontiguousarray(active, np.uint8)
        Cv = np.ascontiguousarray(Cv, np.int32)
        Vc = np.ascontiguousarray(Vc, np.int32)
        rVc = np.ascontiguousarray(rVc, np.int32)
        DfS = np.empty(V, dt)
        self._fn("cp_gradient", sfx)(
            C.c_int(N), C.c_int(V), C.c_int(Eu.size), _ptr(Af, ct), _ptr(Y, ct), _ptr(R, ct),
            _ptr(Eu, C.c_int), _ptr(Ev, C.c_int), _ptr(La_d1, ct), _ptr(L1, ct),
            _ptr(act, C.c_uint8), _ptr(Cv, C.c_int), _ptr(Vc, C.c_int), _ptr(rVc, C.c_int),
            C.c_int(rVc.size - 1), _ptr(rX, ct), _ptr(DfS, ct))
        return DfS

    def cp_capacities(self, cut, La_d1, La_l1, positivity, active, Cv, rX, DfS):
        """:402-535 -> (tr_cap[V], r_cap[E])"""
        self._port_only("cp_capacities")
        DfS = np.ascontiguousarray(DfS)
        dt = DfS.dtype
        ct, sfx = _real(dt)
        La_d1 = np.ascontiguousarray(La_d1, dt)
        L1 = None if La_l1 is None else np.ascontiguousarray(La_l1, dt)
        act = np.ascontiguousarray(active, np.uint8)
        Cv = np.ascontiguousarray(Cv, np.int32)
        rX = np.ascontiguousarray(rX, dt)
        V, E = DfS.size, La_d1.size
        tr = np.empty(V, dt)
        rc = np.empty(E, dt)
        self._fn("cp_capacities", sfx)(
            C.c_int(cut), C.c_int(V), C.c_int(E), _ptr(La_d1, ct), _ptr(L1, ct),
            C.c_int(int(positivity)), _ptr(act, C.c_uint8), _ptr(Cv, C.c_int), _ptr(rX, ct),
            _ptr(DfS, ct), _ptr(tr, ct), _ptr(rc, ct))
        return tr, rc


def _cap_bounds(self, cut, La_d1, lo, hi, active, Cv, rX, DfS):
    """bounds driver :386-534 -> (tr_cap[V], r_cap[E])"""
    self._port_only("cp_capacities_bounds")
    DfS = np.ascontiguousarray(DfS)
    dt = DfS.dtype
    ct, sfx = _real(dt)
    La_d1 = np.ascontiguousarray(La_d1, dt)
    act = np.ascontiguousarray(active, np.uint8)
    Cv = np.ascontiguousarray(Cv, np.int32)
    rX = np.ascontiguousarray(rX, dt)
    V, E = DfS.size, La_d1.size
    tr = np.empty(V, dt)
    rc = np.empty(E, dt)
    self._fn("cp_capacities_bounds", sfx)(
        C.c_int(cut), C.c_int(V), C.c_int(E), _ptr(La_d1, ct), ct(lo), ct(hi),
        _ptr(act, C.c_uint8), _ptr(Cv, C.c_int), _ptr(rX, ct), _ptr(DfS, ct), _ptr(tr, ct),
        _ptr(rc, ct))
    return tr, rc


Oracle.cp_capacities_bounds = _cap_bounds


class CPStepRef:
    """The REFERENCE's cut-pursuit iteration (oracle/_ref/libcp_step_ref.so,
    built from /root/reference/src by ``make -C oracle ref``; only where the
    reference exists).  N = 0 (identity / diagonal A).  See
    oracle/harness/cp_step.cpp."""

    PATH = os.path.join(HERE, "_ref", "libcp_step_ref.so")

    @staticmethod
    def available():
        return os.path.exists(CPStepRef.PATH)

    def __init__(self):
        if CPStepRef.PATH not in _CACHE:
            _CACHE[CPStepRef.PATH] = C.CDLL(CPStepRef.PATH)
        self.lib = _CACHE[CPStepRef.PATH]

    def init(self, Y, A, Eu, Ev, La_d1, La_l1, positivity):
        """rX0 of the reference's initialize() (one component)."""
        Y = np.ascontiguousarray(Y)
        ct, sfx = _real(Y.dtype)
        A = None if A is None else np.ascontiguousarray(A, Y.dtype)
        La_l1 = None if La_l1 is None else np.ascontiguousarray(La_l1, Y.dtype)
        La_d1 = np.ascontiguousarray(La_d1, Y.dtype)
        Eu = np.ascontiguousarray(Eu, np.int32)
        Ev = np.ascontiguousarray(Ev, np.int32)
        rX0 = np.zeros(1, Y.dtype)
        getattr(self.lib, "cp_ref_init_" + sfx)(
            C.c_int(Y.size), C.c_int(Eu.size), _ptr(Y, ct), _ptr(A, ct), _ptr(Eu, C.c_int),
            _ptr(Ev, C.c_int), _ptr(La_d1, ct), _ptr(La_l1, ct), C.c_int(int(positivity)),
            _ptr(rX0, ct))
        return rX0

    def step(self, Y, A, Eu, Ev, La_d1, La_l1, positivity, CP_difTol, state, rho=1.5,
             condMin=1e-3, difRcd=0.0, difTol=1e-4, itMax=1000):
        """One CP iteration from ``state`` (dict: active, Cv, Vc, rVc, rX);
        returns the new state, the last cut's segments and the recorded
        reduced problem (None when no edge was activated)."""
        Y = np.ascontiguousarray(Y)
        dt = Y.dtype
        ct, sfx = _real(dt)
        V, E = Y.size, Eu.size
        A = None if A is None else np.ascontiguousarray(A, dt)
        La_l1 = None if La_l1 is None else np.ascontiguousarray(La_l1, dt)
        La_d1 = np.ascontiguousarray(La_d1, dt)
        Eu = np.ascontiguousarray(Eu, np.int32)
        Ev = np.ascontiguousarray(Ev, np.int32)
        act = np.array(state["active"], np.uint8, copy=True)
        Cv = np.array(state["Cv"], np.int32, copy=True)
        Vc = np.array(state["Vc"], np.int32, copy=True)
        rV = C.c_int(int(state["rVc"].size - 1))
        rVc = np.zeros(V + 1, np.int32)
        rVc[:rV.value + 1] = state["rVc"]
        rX = np.zeros(V, dt)
        rX[:rV.value] = state["rX"]
        seg = np.zeros(V, np.uint8)
        called, rE = C.c_int(0), C.c_int(0)
        rEu = np.zeros(E + V, np.int32)
        rEv = np.zeros(E + V, np.int32)
        rLa = np.zeros(E + V, dt)
        rL1 = np.zeros(V, dt)
        rY = np.zeros(V, dt)
        rAA = np.zeros(V, dt)
        getattr(self.lib, "cp_ref_step_" + sfx)(
            C.c_int(V), C.c_int(E), _ptr(Y, ct), _ptr(A, ct), _ptr(Eu, C.c_int),
            _ptr(Ev, C.c_int), _ptr(La_d1, ct), _ptr(La_l1, ct), C.c_int(int(positivity)),
            ct(CP_difTol), ct(rho), ct(condMin), ct(difRcd), ct(difTol), C.c_int(itMax),
            _ptr(act, C.c_uint8), _ptr(Cv, C.c_int), _ptr(Vc, C.c_int), _ptr(rVc, C.c_int),
            C.byref(rV), _ptr(rX, ct), _ptr(seg, C.c_uint8), C.byref(called), C.byref(rE),
            _ptr(rEu, C.c_int), _ptr(rEv, C.c_int), _ptr(rLa, ct), _ptr(rL1, ct), _ptr(rY, ct),
            _ptr(rAA, ct))
        n = rV.value
        new = {"active": act, "Cv": Cv, "Vc": Vc, "rVc": rVc[:n + 1].copy(),
               "rX": rX[:n].copy()}
        red = None
        if called.value:
            m = rE.value
            red = {"rEu": rEu[:m].copy(), "rEv": rEv[:m].copy(), "rLa_d1": rLa[:m].copy(),
                   "rLa_l1": rL1[:n].copy() if La_l1 is not None else None,
                   "rY": rY[:n].copy(), "rAA": rAA[:n].copy()}
        return new, seg, red

    def init_dense(self, Y, A, N, Eu, Ev, La_d1, La_l1, positivity):
        """rX0 of the reference's initialize() for any N (one component)."""
        Y = np.ascontiguousarray(Y)
        ct, sfx = _real(Y.dtype)
        A = None if A is None else np.ascontiguousarray(A, Y.dtype)
        La_l1 = None if La_l1 is None else np.ascontiguousarray(La_l1, Y.dtype)
        V = int(np.asarray(La_l1).size) if La_l1 is not None else int(Eu.max()) + 1
        rX0 = np.zeros(1, Y.dtype)
        getattr(self.lib, "cp_ref_init_dense_" + sfx)(
            C.c_int(V), C.c_int(Eu.size), C.c_int(N), _ptr(Y, ct), _ptr(A, ct),
            _ptr(np.ascontiguousarray(Eu, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(Ev, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(La_d1, Y.dtype), ct), _ptr(La_l1, ct),
            C.c_int(int(positivity)), _ptr(rX0, ct))
        return rX0

    def step_dense(self, V, N, Y, A, Eu, Ev, La_d1, La_l1, positivity, CP_difTol, state, R,
                   rho=1.5, condMin=1e-3, difRcd=0.0, difTol=1e-5, itMax=2000):
        """One reference CP iteration with a dense A (N > 0: N-by-V column
        major, with the state's residual R = Y - A X; N < 0: A^tA), from
        ``state``; returns (new state, recorded dense reduced problem or
        None): n handed to PFDR, its data vector, matrix and L[rV]."""
        Y = np.ascontiguousarray(Y)
        dt = Y.dtype
        ct, sfx = _real(dt)
        E = Eu.size
        A = np.ascontiguousarray(A, dt)
        La_l1 = None if La_l1 is None else np.ascontiguousarray(La_l1, dt)
        act = np.array(state["active"], np.uint8, copy=True)
        Cv = np.array(state["Cv"], np.int32, copy=True)
        Vc = np.array(state["Vc"], np.int32, copy=True)
        rV = C.c_int(int(state["rVc"].size - 1))
        rVc = np.zeros(V + 1, np.int32)
        rVc[:rV.value + 1] = state["rVc"]
        rX = np.zeros(V, dt)
        rX[:rV.value] = state["rX"]
        R = None if R is None else np.ascontiguousarray(R, dt)
        seg = np.zeros(V, np.uint8)
        called, rE, n = C.c_int(0), C.c_int(0), C.c_int(0)
        rEu = np.zeros(E + V, np.int32)
        rEv = np.zeros(E + V, np.int32)
        rLa = np.zeros(E + V, dt)
        rL1 = np.zeros(V, dt)
        dY = np.zeros(max(abs(N), V), dt)
        dA = np.zeros(max(abs(N), V) * V, dt)
        dL = np.zeros(V, dt)
        getattr(self.lib, "cp_ref_step_dense_" + sfx)(
            C.c_int(V), C.c_int(E), C.c_int(N), _ptr(Y, ct), _ptr(A, ct),
            _ptr(np.ascontiguousarray(Eu, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(Ev, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(La_d1, dt), ct), _ptr(La_l1, ct), C.c_int(int(positivity)),
            ct(CP_difTol), ct(rho), ct(condMin), ct(difRcd), ct(difTol), C.c_int(itMax),
            _ptr(act, C.c_uint8), _ptr(Cv, C.c_int), _ptr(Vc, C.c_int), _ptr(rVc, C.c_int),
            C.byref(rV), _ptr(rX, ct), _ptr(R, ct), _ptr(seg, C.c_uint8), C.byref(called),
            C.byref(rE), _ptr(rEu, C.c_int), _ptr(rEv, C.c_int), _ptr(rLa, ct), _ptr(rL1, ct),
            C.byref(n), _ptr(dY, ct), _ptr(dA, ct), _ptr(dL, ct))
        k = rV.value
        new = {"active": act, "Cv": Cv, "Vc": Vc, "rVc": rVc[:k + 1].copy(), "rX": rX[:k].copy()}
        red = None
        if called.value:
            nn = n.value
            red = {"n": nn, "Y": dY[:(nn if nn > 0 else k)].copy(),
                   "A": dA[:(nn * k if nn > 0 else k * k)].copy(), "L": dL[:k].copy()}
        return new, red

    def maxflow(self, Eu, Ev, tr_cap, r_cap):
        """Segments (0 source, 1 sink) of the reference's BK maxflow."""
        tr_cap = np.ascontiguousarray(tr_cap)
        ct, sfx = _real(tr_cap.dtype)
        r_cap = np.ascontiguousarray(r_cap, tr_cap.dtype)
        Eu = np.ascontiguousarray(Eu, np.int32)
        Ev = np.ascontiguousarray(Ev, np.int32)
        seg = np.zeros(tr_cap.size, np.uint8)
        fn = getattr(self.lib, "cp_ref_maxflow_" + sfx)
        fn.restype = ct
        fn(C.c_int(tr_cap.size), C.c_int(Eu.size), _ptr(Eu, C.c_int), _ptr(Ev, C.c_int),
           _ptr(tr_cap, ct), _ptr(r_cap, ct), _ptr(seg, C.c_uint8))
        return seg


class CPStepRefBounds:
    """The REFERENCE's bounds cut pursuit, one iteration at a time
    (oracle/_ref/libcp_step_bounds_ref.so, harness/cp_step_bounds.cpp; only
    where the reference exists).  N = 0 (identity / diagonal A)."""

    PATH = os.path.join(HERE, "_ref", "libcp_step_bounds_ref.so")

    @staticmethod
    def available():
        return os.path.exists(CPStepRefBounds.PATH)

    def __init__(self):
        if CPStepRefBounds.PATH not in _CACHE:
            _CACHE[CPStepRefBounds.PATH] = C.CDLL(CPStepRefBounds.PATH)
        self.lib = _CACHE[CPStepRefBounds.PATH]

    def init(self, Y, A, Eu, Ev, La_d1, lo, hi):
        Y = np.ascontiguousarray(Y)
        ct, sfx = _real(Y.dtype)
        A = None if A is None else np.ascontiguousarray(A, Y.dtype)
        rX0 = np.zeros(1, Y.dtype)
        getattr(self.lib, "cp_refb_init_" + sfx)(
            C.c_int(Y.size), C.c_int(Eu.size), _ptr(Y, ct), _ptr(A, ct),
            _ptr(np.ascontiguousarray(Eu, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(Ev, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(La_d1, Y.dtype), ct), ct(lo), ct(hi), _ptr(rX0, ct))
        return rX0

    def step(self, Y, A, Eu, Ev, La_d1, lo, hi, CP_difTol, state, rho=1.5, condMin=1e-3,
             difRcd=0.0, difTol=1e-4, itMax=1000):
        """-> (new state, last cut's segments, reduced problem or None)"""
        Y = np.ascontiguousarray(Y)
        dt = Y.dtype
        ct, sfx = _real(dt)
        V, E = Y.size, Eu.size
        A = None if A is None else np.ascontiguousarray(A, dt)
        act = np.array(state["active"], np.uint8, copy=True)
        Cv = np.array(state["Cv"], np.int32, copy=True)
        Vc = np.array(state["Vc"], np.int32, copy=True)
        rV = C.c_int(int(state["rVc"].size - 1))
        rVc = np.zeros(V + 1, np.int32)
        rVc[:rV.value + 1] = state["rVc"]
        rX = np.zeros(V, dt)
        rX[:rV.value] = state["rX"]
        seg = np.zeros(V, np.uint8)
        called, rE = C.c_int(0), C.c_int(0)
        rEu = np.zeros(E + V, np.int32)
        rEv = np.zeros(E + V, np.int32)
        rLa = np.zeros(E + V, dt)
        rY = np.zeros(V, dt)
        rAA = np.zeros(V, dt)
        getattr(self.lib, "cp_refb_step_" + sfx)(
            C.c_int(V), C.c_int(E), _ptr(Y, ct), _ptr(A, ct),
            _ptr(np.ascontiguousarray(Eu, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(Ev, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(La_d1, dt), ct), ct(lo), ct(hi), ct(CP_difTol), ct(rho),
            ct(condMin), ct(difRcd), ct(difTol), C.c_int(itMax), _ptr(act, C.c_uint8),
            _ptr(Cv, C.c_int), _ptr(Vc, C.c_int), _ptr(rVc, C.c_int), C.byref(rV), _ptr(rX, ct),
            _ptr(seg, C.c_uint8), C.byref(called), C.byref(rE), _ptr(rEu, C.c_int),
            _ptr(rEv, C.c_int), _ptr(rLa, ct), _ptr(rY, ct), _ptr(rAA, ct))
        n = rV.value
        new = {"active": act, "Cv": Cv, "Vc": Vc, "rVc": rVc[:n + 1].copy(),
               "rX": rX[:n].copy()}
        red = None
        if called.value:
            m = rE.value
            red = {"rEu": rEu[:m].copy(), "rEv": rEv[:m].copy(), "rLa_d1": rLa[:m].copy(),
                   "rLa_l1": None, "rY": rY[:n].copy(), "rAA": rAA[:n].copy()}
        return new, seg, red


# ---- the simplex driver's steps (oracle/cp_graph_body.h, port only),
# src/CP_PFDR_graph_loss_d1_simplex.cpp; P layouts are vertex-major [v*K + k]
def _sx_reduced(self, K, al, Q, Vc, rVc):
    """:733-766 -> (rP[rV*K], rQ[rV*K], rLa_f[rV] or None when al == 0)"""
    self._port_only("cp_simplex_reduced")
    Q = np.ascontiguousarray(Q)
    ct, sfx = _real(Q.dtype)
    Vc = np.ascontiguousarray(Vc, np.int32)
    rVc = np.ascontiguousarray(rVc, np.int32)
    rV = rVc.size - 1
    rP = np.empty(rV * K, Q.dtype)
    rQ = np.empty(rV * K, Q.dtype)
    rLa_f = np.empty(rV, Q.dtype) if al != 0 else None
    self._fn("cp_simplex_reduced", sfx)(
        C.c_int(K), ct(al), _ptr(Q, ct), _ptr(Vc, C.c_int), _ptr(rVc, C.c_int), C.c_int(rV),
        _ptr(rP, ct), _ptr(rQ, ct), _ptr(rLa_f, ct))
    return rP, rQ, rLa_f


def _sx_gradient(self, K, al, Q, Eu, Ev, La_d1, active, Cv, rP, eps):
    """:327-376 and :525-536 -> (DfS[V*K], rDi[rV])"""
    self._port_only("cp_simplex_gradient")
    Q = np.ascontiguousarray(Q)
    dt = Q.dtype
    ct, sfx = _real(dt)
    V = Q.size // K
    rP = np.ascontiguousarray(rP, dt)
    rV = rP.size // K
    Eu = np.ascontiguousarray(Eu, np.int32)
    Ev = np.ascontiguousarray(Ev, np.int32)
    DfS = np.empty(V * K, dt)
    rDi = np.empty(rV, np.int32)
    self._fn("cp_simplex_gradient", sfx)(
        C.c_int(K), C.c_int(V), C.c_int(Eu.size), ct(al), _ptr(Q, ct), _ptr(Eu, C.c_int),
        _ptr(Ev, C.c_int), _ptr(np.ascontiguousarray(La_d1, dt), ct),
        _ptr(np.ascontiguousarray(active, np.uint8), C.c_uint8),
        _ptr(np.ascontiguousarray(Cv, np.int32), C.c_int), C.c_int(rV), _ptr(rP, ct), ct(eps),
        _ptr(DfS, ct), _ptr(rDi, C.c_int))
    return DfS, rDi


def _sx_capacities(self, K, n, Eu, Ev, La_d1, active, Vc, rVc, rDi, Djv, DfS):
    """:542-595 -> (tr_cap[V], r_cap[E]: arc 2e; arc 2e + 1 has none)"""
    self._port_only("cp_simplex_capacities")
    DfS = np.ascontiguousarray(DfS)
    dt = DfS.dtype
    ct, sfx = _real(dt)
    V = DfS.size // K
    Eu = np.ascontiguousarray(Eu, np.int32)
    Ev = np.ascontiguousarray(Ev, np.int32)
    rVc = np.ascontiguousarray(rVc, np.int32)
    tr = np.empty(V, dt)
    rc = np.empty(Eu.size, dt)
    self._fn("cp_simplex_capacities", sfx)(
        C.c_int(K), C.c_int(V), C.c_int(Eu.size), C.c_int(n), _ptr(Eu, C.c_int),
        _ptr(Ev, C.c_int), _ptr(np.ascontiguousarray(La_d1, dt), ct),
        _ptr(np.ascontiguousarray(active, np.uint8), C.c_uint8),
        _ptr(np.ascontiguousarray(Vc, np.int32), C.c_int), _ptr(rVc, C.c_int),
        C.c_int(rVc.size - 1), _ptr(np.ascontiguousarray(rDi, np.int32), C.c_int),
        _ptr(np.ascontiguousarray(Djv, np.int32), C.c_int), _ptr(DfS, ct), _ptr(tr, ct),
        _ptr(rc, ct))
    return tr, rc


def _sx_expand(self, n, segment, Djv):
    """:600-604 -> new Djv"""
    self._port_only("cp_simplex_expand")
    D = np.array(Djv, np.int32, copy=True)
    seg = np.ascontiguousarray(segment, np.uint8)
    self.lib.oracle_cp_simplex_expand(C.c_int(D.size), C.c_int(n), _ptr(seg, C.c_uint8),
                                      _ptr(D, C.c_int))
    return D


def _sx_activate(self, Eu, Ev, Djv, active):
    """:608-618 -> (new active, count)"""
    self._port_only("cp_simplex_activate")
    Eu = np.ascontiguousarray(Eu, np.int32)
    Ev = np.ascontiguousarray(Ev, np.int32)
    act = np.array(active, np.uint8, copy=True)
    fn = self.lib.oracle_cp_simplex_activate
    fn.restype = C.c_int
    n = fn(C.c_int(Eu.size), _ptr(Eu, C.c_int), _ptr(Ev, C.c_int),
           _ptr(np.ascontiguousarray(Djv, np.int32), C.c_int), _ptr(act, C.c_uint8))
    return act, int(n)


def _sx_merge(self, K, Eu, Ev, Cv, rP, eps, active):
    """:782-803 -> (new active, deactivated count)"""
    self._port_only("cp_simplex_merge")
    rP = np.ascontiguousarray(rP)
    ct, sfx = _real(rP.dtype)
    Eu = np.ascontiguousarray(Eu, np.int32)
    Ev = np.ascontiguousarray(Ev, np.int32)
    act = np.array(active, np.uint8, copy=True)
    fn = self._fn("cp_simplex_merge", sfx)
    fn.restype = C.c_int
    n = fn(C.c_int(K), C.c_int(Eu.size), _ptr(Eu, C.c_int), _ptr(Ev, C.c_int),
           _ptr(np.ascontiguousarray(Cv, np.int32), C.c_int), _ptr(rP, ct), ct(eps),
           _ptr(act, C.c_uint8))
    return act, int(n)


Oracle.cp_simplex_reduced = _sx_reduced
Oracle.cp_simplex_gradient = _sx_gradient
Oracle.cp_simplex_capacities = _sx_capacities
Oracle.cp_simplex_expand = _sx_expand
Oracle.cp_simplex_activate = _sx_activate
Oracle.cp_simplex_merge = _sx_merge


class CPStepRefSimplex:
    """The REFERENCE's simplex cut pursuit, one iteration at a time
    (oracle/_ref/libcp_step_simplex_ref.so, harness/cp_step_simplex.cpp;
    only where the reference exists), and its BK maxflow with the simplex
    driver's arc capacities."""

    PATH = os.path.join(HERE, "_ref", "libcp_step_simplex_ref.so")

    @staticmethod
    def available():
        return os.path.exists(CPStepRefSimplex.PATH)

    def __init__(self):
        if CPStepRefSimplex.PATH not in _CACHE:
            _CACHE[CPStepRefSimplex.PATH] = C.CDLL(CPStepRefSimplex.PATH)
        self.lib = _CACHE[CPStepRefSimplex.PATH]

    def init(self, K, al, Q, Eu, Ev, La_d1):
        Q = np.ascontiguousarray(Q)
        ct, sfx = _real(Q.dtype)
        rP0 = np.zeros(K, Q.dtype)
        getattr(self.lib, "cp_refs_init_" + sfx)(
            C.c_int(K), C.c_int(Q.size // K), C.c_int(Eu.size), ct(al), _ptr(Q, ct),
            _ptr(np.ascontiguousarray(Eu, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(Ev, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(La_d1, Q.dtype), ct), _ptr(rP0, ct))
        return rP0

    def step(self, K, al, Q, Eu, Ev, La_d1, CP_difTol, state, rho=1.5, condMin=1e-3,
             difRcd=0.0, difTol=1e-3, itMax=1000):
        """-> (new state, last expansion's segments, reduced problem or None)"""
        Q = np.ascontiguousarray(Q)
        dt = Q.dtype
        ct, sfx = _real(dt)
        V, E = Q.size // K, Eu.size
        act = np.array(state["active"], np.uint8, copy=True)
        Cv = np.array(state["Cv"], np.int32, copy=True)
        Vc = np.array(state["Vc"], np.int32, copy=True)
        rV = C.c_int(int(state["rVc"].size - 1))
        rVc = np.zeros(V + 1, np.int32)
        rVc[:rV.value + 1] = state["rVc"]
        rP = np.zeros(V * K, dt)
        rP[:rV.value * K] = state["rP"]
        seg = np.zeros(V, np.uint8)
        called, rE = C.c_int(0), C.c_int(0)
        rEu = np.zeros(E + V, np.int32)
        rEv = np.zeros(E + V, np.int32)
        rLa = np.zeros(E + V, dt)
        rQ = np.zeros(V * K, dt)
        rLa_f = np.zeros(V, dt)
        rP0 = np.zeros(V * K, dt)
        getattr(self.lib, "cp_refs_step_" + sfx)(
            C.c_int(K), C.c_int(V), C.c_int(E), ct(al), _ptr(Q, ct),
            _ptr(np.ascontiguousarray(Eu, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(Ev, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(La_d1, dt), ct), ct(CP_difTol), ct(rho), ct(condMin),
            ct(difRcd), ct(difTol), C.c_int(itMax), _ptr(act, C.c_uint8), _ptr(Cv, C.c_int),
            _ptr(Vc, C.c_int), _ptr(rVc, C.c_int), C.byref(rV), _ptr(rP, ct),
            _ptr(seg, C.c_uint8), C.byref(called), C.byref(rE), _ptr(rEu, C.c_int),
            _ptr(rEv, C.c_int), _ptr(rLa, ct), _ptr(rQ, ct), _ptr(rLa_f, ct), _ptr(rP0, ct))
        n = rV.value
        new = {"active": act, "Cv": Cv, "Vc": Vc, "rVc": rVc[:n + 1].copy(),
               "rP": rP[:n * K].copy()}
        red = None
        if called.value:
            m = rE.value
            red = {"rEu": rEu[:m].copy(), "rEv": rEv[:m].copy(), "rLa_d1": rLa[:m].copy(),
                   "rQ": rQ[:n * K].copy(), "rLa_f": rLa_f[:n].copy() if al != 0 else None,
                   "rP0": rP0[:n * K].copy()}
        return new, seg, red

    def maxflow(self, Eu, Ev, tr_cap, r_cap):
        """Segments (0 source, 1 sink) with arc 2e from r_cap[e], arc 2e+1 none."""
        tr_cap = np.ascontiguousarray(tr_cap)
        ct, sfx = _real(tr_cap.dtype)
        seg = np.zeros(tr_cap.size, np.uint8)
        getattr(self.lib, "cp_refs_maxflow_" + sfx)(
            C.c_int(tr_cap.size), C.c_int(Eu.size),
            _ptr(np.ascontiguousarray(Eu, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(Ev, np.int32), C.c_int), _ptr(tr_cap, ct),
            _ptr(np.ascontiguousarray(r_cap, tr_cap.dtype), ct), _ptr(seg, C.c_uint8))
        return seg


# ---- the duplex driver's cut (oracle/cp_graph_body.h, port only),
# src/CP_PFDR_graph_quadratic_d1_l1_duplex.cpp:469-545
def _dx_capacities(self, La_d1, La_l1, positivity, active, Cv, rX, DfS):
    """-> (tr_cap[2V]: v1 then v2 nodes, r_link[V]: arc v1 -> v2, r_cap[E]:
    every arc of edge e in both layers)"""
    self._port_only("cp_capacities_duplex")
    DfS = np.ascontiguousarray(DfS)
    dt = DfS.dtype
    ct, sfx = _real(dt)
    La_d1 = np.ascontiguousarray(La_d1, dt)
    L1 = None if La_l1 is None else np.ascontiguousarray(La_l1, dt)
    V, E = DfS.size, La_d1.size
    tr = np.empty(2 * V, dt)
    link = np.empty(V, dt)
    rc = np.empty(E, dt)
    self._fn("cp_capacities_duplex", sfx)(
        C.c_int(V), C.c_int(E), _ptr(La_d1, ct), _ptr(L1, ct), C.c_int(int(positivity)),
        _ptr(np.ascontiguousarray(active, np.uint8), C.c_uint8),
        _ptr(np.ascontiguousarray(Cv, np.int32), C.c_int),
        _ptr(np.ascontiguousarray(rX, dt), ct), _ptr(DfS, ct), _ptr(tr, ct), _ptr(link, ct),
        _ptr(rc, ct))
    return tr, link, rc


def _dx_activate(self, V, Eu, Ev, segment, active):
    """-> (new active, count); segment[2V]"""
    self._port_only("cp_activate_duplex")
    act = np.array(active, np.uint8, copy=True)
    fn = self.lib.oracle_cp_activate_duplex
    fn.restype = C.c_int
    w = fn(C.c_int(V), C.c_int(len(Eu)), _ptr(np.ascontiguousarray(Eu, np.int32), C.c_int),
           _ptr(np.ascontiguousarray(Ev, np.int32), C.c_int),
           _ptr(np.ascontiguousarray(segment, np.uint8), C.c_uint8), _ptr(act, C.c_uint8))
    return act, int(w)


Oracle.cp_capacities_duplex = _dx_capacities
Oracle.cp_activate_duplex = _dx_activate


class CPStepRefDuplex:
    """The REFERENCE's duplex cut pursuit (non-differentiable case), one
    iteration at a time (oracle/_ref/libcp_step_duplex_ref.so,
    harness/cp_step_duplex.cpp; only where the reference exists).  N = 0."""

    PATH = os.path.join(HERE, "_ref", "libcp_step_duplex_ref.so")

    @staticmethod
    def available():
        return os.path.exists(CPStepRefDuplex.PATH)

    def __init__(self):
        if CPStepRefDuplex.PATH not in _CACHE:
            _CACHE[CPStepRefDuplex.PATH] = C.CDLL(CPStepRefDuplex.PATH)
        self.lib = _CACHE[CPStepRefDuplex.PATH]

    def init(self, Y, A, Eu, Ev, La_d1, La_l1, positivity):
        Y = np.ascontiguousarray(Y)
        ct, sfx = _real(Y.dtype)
        A = None if A is None else np.ascontiguousarray(A, Y.dtype)
        La_l1 = None if La_l1 is None else np.ascontiguousarray(La_l1, Y.dtype)
        rX0 = np.zeros(1, Y.dtype)
        getattr(self.lib, "cp_refd_init_" + sfx)(
            C.c_int(Y.size), C.c_int(Eu.size), _ptr(Y, ct), _ptr(A, ct),
            _ptr(np.ascontiguousarray(Eu, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(Ev, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(La_d1, Y.dtype), ct), _ptr(La_l1, ct),
            C.c_int(int(positivity)), _ptr(rX0, ct))
        return rX0

    def step(self, Y, A, Eu, Ev, La_d1, La_l1, positivity, CP_difTol, state, rho=1.5,
             condMin=1e-3, difRcd=0.0, difTol=1e-4, itMax=1000):
        """-> (new state, segments of the 2V nodes, reduced problem or None)"""
        Y = np.ascontiguousarray(Y)
        dt = Y.dtype
        ct, sfx = _real(dt)
        V, E = Y.size, Eu.size
        A = None if A is None else np.ascontiguousarray(A, dt)
        La_l1 = None if La_l1 is None else np.ascontiguousarray(La_l1, dt)
        act = np.array(state["active"], np.uint8, copy=True)
        Cv = np.array(state["Cv"], np.int32, copy=True)
        Vc = np.array(state["Vc"], np.int32, copy=True)
        rV = C.c_int(int(state["rVc"].size - 1))
        rVc = np.zeros(V + 1, np.int32)
        rVc[:rV.value + 1] = state["rVc"]
        rX = np.zeros(V, dt)
        rX[:rV.value] = state["rX"]
        seg = np.zeros(2 * V, np.uint8)
        called, rE = C.c_int(0), C.c_int(0)
        rEu = np.zeros(E + V, np.int32)
        rEv = np.zeros(E + V, np.int32)
        rLa = np.zeros(E + V, dt)
        rL1 = np.zeros(V, dt)
        rY = np.zeros(V, dt)
        rAA = np.zeros(V, dt)
        getattr(self.lib, "cp_refd_step_" + sfx)(
            C.c_int(V), C.c_int(E), _ptr(Y, ct), _ptr(A, ct),
            _ptr(np.ascontiguousarray(Eu, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(Ev, np.int32), C.c_int),
            _ptr(np.ascontiguousarray(La_d1, dt), ct), _ptr(La_l1, ct), C.c_int(int(positivity)),
            ct(CP_difTol), ct(rho), ct(condMin), ct(difRcd), ct(difTol), C.c_int(itMax),
            _ptr(act, C.c_uint8), _ptr(Cv, C.c_int), _ptr(Vc, C.c_int), _ptr(rVc, C.c_int),
            C.byref(rV), _ptr(rX, ct), _ptr(seg, C.c_uint8), C.byref(called), C.byref(rE),
            _ptr(rEu, C.c_int), _ptr(rEv, C.c_int), _ptr(rLa, ct), _ptr(rL1, ct), _ptr(rY, ct),
            _ptr(rAA, ct))
        n = rV.value
        new = {"active": act, "Cv": Cv, "Vc": Vc, "rVc": rVc[:n + 1].copy(),
               "rX": rX[:n].copy()}
        red = None
        if called.value:
            m = rE.value
            red = {"rEu": rEu[:m].copy(), "rEv": rEv[:m].copy(), "rLa_d1": rLa[:m].copy(),
                   "rLa_l1": rL1[:n].copy() if La_l1 is not None else None,
                   "rY": rY[:n].copy(), "rAA": rAA[:n].copy()}
        return new, seg, red


def _refd_maxflow(self, V, Eu, Ev, tr_cap, r_link, r_cap):
    """Segments of the 2V nodes: the reference's BK maxflow on the duplex
    graph with the cut's capacities (tr_cap[2V], r_link[V], r_cap[E])."""
    tr_cap = np.ascontiguousarray(tr_cap)
    ct, sfx = _real(tr_cap.dtype)
    seg = np.zeros(2 * V, np.uint8)
    getattr(self.lib, "cp_refd_maxflow_" + sfx)(
        C.c_int(V), C.c_int(len(Eu)), _ptr(np.ascontiguousarray(Eu, np.int32), C.c_int),
        _ptr(np.ascontiguousarray(Ev, np.int32), C.c_int), _ptr(tr_cap, ct),
        _ptr(np.ascontiguousarray(r_link, tr_cap.dtype), ct),
        _ptr(np.ascontiguousarray(r_cap, tr_cap.dtype), ct), _ptr(seg, C.c_uint8))
    return seg


CPStepRefDuplex.maxflow = _refd_maxflow
