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
