"""1-D vertex-range partition of a PFDR graph.

* ``vertex_offsets`` / ``split_edges``: rank r owns global vertices
  [off[r], off[r+1]) and the edges whose Eu it owns, keeping their global
  edge ids (the per-vertex DR sums run in global edge order on every rank).
* ``Plan``: the library's host-only planner (pfdr_plan_* in
  include/pfdr_mi355x.h) — what a partitioned session runs at setup, drivable
  over any transport (the CPU tests use torch.distributed/gloo).
* ``locality_order`` / ``relabelled_split``: randomly labelled graphs are
  relabelled (breadth-first, pfdr_locality_order) before the vertex-range
  split, so the halos stay the size of the graph's cut surfaces
  (SURVEY.md §8(e)); the result is unchanged bit for bit.
* ``solve_loopback``: k ranks as k threads on one GPU (loopback transport);
  returns the concatenated result, which equals the unpartitioned solve.
* ``comm_init``: the RCCL communicator for one process per GPU, its unique id
  broadcast over a host (gloo) process group.
"""
import ctypes as C
import threading

import numpy as np

from . import pfdr

PLAN_GHOSTS, PLAN_EU_LOCAL, PLAN_EV_LOCAL = 0, 1, 2
PLAN_PULL_REQUEST, PLAN_PUSH_ITEMS, PLAN_PUSH_ADDR = 3, 4, 5
PLAN_PULL_INDEX, PLAN_RECV_KEYS = 6, 7
PLAN_GHOST_OFFSETS, PLAN_PULL_OFFSETS, PLAN_PUSH_OFFSETS, PLAN_RECV_OFFSETS = 8, 9, 10, 11
COMM_RCCL, COMM_LOOPBACK = 0, 1

_PLAN_DTYPES = {PLAN_GHOSTS: np.int64, PLAN_EU_LOCAL: np.int32, PLAN_EV_LOCAL: np.int32,
                PLAN_PULL_REQUEST: np.int64, PLAN_PUSH_ITEMS: np.int64,
                PLAN_PUSH_ADDR: np.uint32, PLAN_PULL_INDEX: np.int32,
                PLAN_RECV_KEYS: np.uint64, PLAN_GHOST_OFFSETS: np.int32,
                PLAN_PULL_OFFSETS: np.int32, PLAN_PUSH_OFFSETS: np.int32,
                PLAN_RECV_OFFSETS: np.int32}


def vertex_offsets(V, k):
    """Balanced contiguous vertex ranges, off[0] = 0, off[k] = V."""
    return np.array([(V * r) // k for r in range(k + 1)], np.int64)


def split_edges(Eu, off):
    """Edge ids (ascending) owned by each rank: those whose Eu it owns."""
    owner = np.searchsorted(off, np.asarray(Eu, np.int64), side="right") - 1
    return [np.nonzero(owner == r)[0].astype(np.int64) for r in range(len(off) - 1)]


def locality_order(V, Eu, Ev):
    """order[new] = old label: the library's deterministic breadth-first
    order (pfdr_locality_order, computed on the current GPU); identity for
    path-like graphs.  Returns (order, applied)."""
    lib = pfdr.load()
    Eu = np.ascontiguousarray(Eu, np.int32)
    Ev = np.ascontiguousarray(Ev, np.int32)
    order = np.empty(V, np.int32)
    applied = C.c_int(0)
    pfdr._check(lib.pfdr_locality_order(C.c_int(V), C.c_int64(Eu.size),
                                        C.c_void_p(Eu.ctypes.data), C.c_void_p(Ev.ctypes.data),
                                        C.c_int(pfdr.PFDR_MEM_HOST),
                                        C.c_void_p(order.ctypes.data), C.byref(applied)),
                "pfdr_locality_order")
    return order, bool(applied.value)


def relabelled_split(order, off, Eu, Ev):
    """The vertex-range split of a relabelled graph: new label of every old
    one (where), relabelled endpoints, and per rank the original edge ids it
    owns (relabelled Eu in its range) sorted by (relabelled Eu, edge id), so
    every rank's edges are u-sorted for the sweeps.  The summation order
    stays the reference's: the sessions key their sums by the original edge
    ids (e_global)."""
    order = np.asarray(order, np.int64)
    where = np.empty_like(order)
    where[order] = np.arange(order.size)
    nEu = where[np.asarray(Eu, np.int64)]
    nEv = where[np.asarray(Ev, np.int64)]
    parts = []
    owner = np.searchsorted(off, nEu, side="right") - 1
    for r in range(len(off) - 1):
        e = np.nonzero(owner == r)[0]
        parts.append(e[np.argsort(nEu[e], kind="stable")].astype(np.int64))
    return where, nEu.astype(np.int32), nEv.astype(np.int32), parts


class Plan:
    def __init__(self, nranks, rank, off, Eu, Ev, e_global):
        lib = pfdr.load()
        lib.pfdr_plan_get.restype = C.c_int64
        lib.pfdr_plan_get.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        lib.pfdr_plan_set_incoming.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int64,
                                               C.c_void_p]
        lib.pfdr_plan_destroy.argtypes = [C.c_void_p]
        self.lib = lib
        self.nranks, self.rank = nranks, rank
        self._off = np.ascontiguousarray(off, np.int64)
        Eu = np.ascontiguousarray(Eu, np.int32)
        Ev = np.ascontiguousarray(Ev, np.int32)
        eg = np.ascontiguousarray(e_global, np.int64)
        h = C.c_void_p()
        pfdr._check(lib.pfdr_plan_create(C.byref(h), C.c_int(nranks), C.c_int(rank),
                                         C.c_void_p(self._off.ctypes.data), C.c_int(Eu.size),
                                         C.c_void_p(Eu.ctypes.data), C.c_void_p(Ev.ctypes.data),
                                         C.c_void_p(eg.ctypes.data), C.c_int64(0)),
                    "pfdr_plan_create")
        self.h = h

    def get(self, what, peer=0):
        n = self.lib.pfdr_plan_get(self.h, what, peer, None)
        if n < 0:
            raise pfdr.PFDRError("pfdr_plan_get(%d) failed" % what)
        out = np.empty(n, _PLAN_DTYPES[what])
        if n:
            self.lib.pfdr_plan_get(self.h, what, peer, C.c_void_p(out.ctypes.data))
        return out

    def set_incoming(self, peer, what, data):
        data = np.ascontiguousarray(data, np.int64)
        pfdr._check(self.lib.pfdr_plan_set_incoming(self.h, peer, what, data.size,
                                                    C.c_void_p(data.ctypes.data)),
                    "pfdr_plan_set_incoming")

    def finish(self):
        pfdr._check(self.lib.pfdr_plan_finish(self.h), "pfdr_plan_finish")

    def close(self):
        if self.h:
            self.lib.pfdr_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def solve_loopback(k, kind, dtype, Eu, Ev, La_d1, X0, Y, A=None, La_l1=None,
                   positivity=0, lo=-np.inf, hi=np.inf, Ltype=0, L=None, rho=1.5,
                   condMin=1e-3, difRcd=0.0, difTol=0.0, itMax=100, record_obj=False,
                   record_dif=False, off=None, K=0, al=0.0, N=0, relabel=False, evolution=0,
                   spec=0):
    """Partitioned solve with k ranks as k threads on the current GPU.
    Simplex (kind PFDR_KIND_SIMPLEX): X0 = P0 and Y = Q are K-by-V (v*K + k),
    La_l1 = La_f.  Dense A: N > 0 (A is N-by-V column-major, each rank gets
    its vertices' columns, Y stays whole) or N = -V (A^tA, column blocks).
    relabel (graph modes): split the locality order instead of the labels
    (locality_order, relabelled_split).  evolution: pfdr.EVOLUTION_* (AUTO:
    sequential rounding from 2^17 vertices, as one GPU).  spec: pfdr.SPEC_* (the
    speculative decisions' concurrency).  Returns (X, it, Obj, Dif, info)
    with X for all vertices in the caller's labels."""
    lib = pfdr.load()
    Kw = max(int(K), 1)
    V = np.asarray(X0).size // Kw
    off = vertex_offsets(V, k) if off is None else np.asarray(off, np.int64)
    order = None
    if relabel:
        if N != 0:
            raise ValueError("relabel: graph modes only (identity / diagonal A, simplex)")
        order, _ = locality_order(V, Eu, Ev)
        where, Eu, Ev, parts = relabelled_split(order, off, Eu, Ev)
        oi = np.asarray(order, np.int64)

        def perm(a):  # per-vertex arrays into the new labels
            if a is None:
                return None
            a = np.asarray(a)
            if Kw > 1 and a.size == V * Kw:
                return np.ascontiguousarray(a.reshape(V, Kw)[oi].reshape(-1))
            return np.ascontiguousarray(a[oi]) if a.size == V else a
        X0, Y, A, La_l1, L = perm(X0), perm(Y), perm(A), perm(La_l1), perm(L)
    else:
        parts = split_edges(Eu, off)
    hub = C.c_void_p()
    pfdr._check(lib.pfdr_loopback_create(C.byref(hub), C.c_int(k)), "pfdr_loopback_create")
    results, errors, queries = [None] * k, [None] * k, [None] * k

    def rank_main(r):
        try:
            e = parts[r]
            v0, v1 = int(off[r]), int(off[r + 1])
            sl = slice(v0, v1)

            def vsl(a):
                if a is None:
                    return None
                a = np.asarray(a)
                if Kw > 1 and a.size == V * Kw:
                    return a[v0 * Kw:v1 * Kw]
                return a[sl] if a.size == V else a
            if N > 0:  # columns of the owned vertices; the data vector is whole
                Ar, Yr = np.asarray(A).reshape(V, N)[v0:v1].ravel(), np.asarray(Y)
            elif N < 0:
                Ar, Yr = np.asarray(A).reshape(V, V)[v0:v1].ravel(), vsl(Y)
            else:
                Ar, Yr = vsl(A), vsl(Y)
            s = pfdr.Session(kind, dtype, v1 - v0, e.size, np.asarray(Eu)[e],
                             np.asarray(Ev)[e], np.asarray(La_d1)[e], vsl(X0), Yr, N=N,
                             A=Ar, La_l1=vsl(La_l1), positivity=positivity, lo=lo, hi=hi,
                             Ltype=Ltype, L=vsl(L), rho=rho, condMin=condMin, difRcd=difRcd,
                             difTol=difTol, itMax=itMax, record_obj=record_obj,
                             record_dif=record_dif, K=K, al=al, nranks=k, rank=r, comm=hub.value,
                             comm_kind=COMM_LOOPBACK, vtx_begin=v0, V_global=V, e_global=e,
                             vtx_label=None if order is None else order[v0:v1],
                             evolution=evolution, spec=spec)
            queries[r] = {q: s.query(q) for q in ("ghosts", "speculative", "seqdif")}
            if kind != pfdr.PFDR_KIND_SIMPLEX:
                queries[r].update({q: s.query(q) for q in ("split_blocks", "ustaged", "tiled_blocks",
                                                            "record_blocks", "edge_ratio",
                                                            "vertex_pair")})
            s.run(itMax)
            results[r] = s.result()
            s.close()
        except Exception as ex:  # reported by the caller; wake the other ranks
            errors[r] = ex
            lib.pfdr_loopback_abort(hub, ("rank %d failed: %s" % (r, ex))[:200].encode())

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(k)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    lib.pfdr_loopback_destroy(hub)
    # the first failure is the cause; the others are its consequence
    first = [ex for ex in errors if ex is not None and "aborted" not in str(ex)]
    for ex in first or [ex for ex in errors if ex is not None]:
        raise ex
    X = np.concatenate([res[0] for res in results])
    if order is not None:  # back to the caller's labels
        Xo = np.empty_like(X)
        if Kw > 1:
            Xo.reshape(V, Kw)[np.asarray(order, np.int64)] = X.reshape(V, Kw)
        else:
            Xo[np.asarray(order, np.int64)] = X
        X = Xo
    its = {res[1] for res in results}
    if len(its) != 1:
        raise pfdr.PFDRError("ranks disagree on the iteration count: %s" % its)
    it = its.pop()
    return X, it, results[0][2], results[0][3], {"off": off, "edges": [p.size for p in parts],
                                                 "queries": queries, "order": order}


def comm_init(nranks, rank, host_broadcast):
    """RCCL communicator of this rank (one process per GPU): rank 0 creates
    the unique id, ``host_broadcast`` broadcasts a CPU uint8 torch tensor from
    rank 0 in place (e.g. ``lambda t: torch.distributed.broadcast(t, 0)`` on a
    gloo group), every rank joins.  This is the only RCCL communicator of the
    process: the halo exchanges, the scalar all-reduces and the timing
    reduction all use it (torch's own NCCL group is never opened)."""
    import torch
    lib = pfdr.load()
    buf = (C.c_char * 128)()
    if rank == 0:
        pfdr._check(lib.pfdr_comm_unique_id(buf), "pfdr_comm_unique_id")
    t = torch.tensor(list(bytes(buf)), dtype=torch.uint8)
    host_broadcast(t)
    idb = (C.c_char * 128).from_buffer_copy(bytes(t.tolist()))
    comm = C.c_void_p()
    pfdr._check(lib.pfdr_comm_init(C.byref(comm), nranks, rank, idb), "pfdr_comm_init")
    return comm.value


def comm_max(comm, value):
    """max over the ranks of a host double, through the RCCL communicator"""
    v = C.c_double(float(value))
    pfdr._check(pfdr.load().pfdr_comm_allreduce_max_f64(comm, C.byref(v)),
                "pfdr_comm_allreduce_max_f64")
    return v.value


def comm_destroy(comm):
    if comm:
        pfdr._check(pfdr.load().pfdr_comm_destroy(comm), "pfdr_comm_destroy")
