"""GPU: the partitioned solver (1-D vertex ranges, halo pull/push, chained
exact preconditioner sum) with k ranks as k threads on ONE GPU (loopback
transport: the same session code as RCCL, exchanges as device copies),
against the REFERENCE's golden outputs.  Expected bit-exact: partitioning
changes no arithmetic and no summation order (tests/test_partition_cpu.py)."""
import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

CASES = ["l1_grid2d_f64", "l1_grid2d_f32", "l1_knn_shuffled_f32", "l1_l22_f64",
         "l1_grid3d_pos_f32", "l1_grid2d_recond_f64", "bounds_box_f32",
         "bounds_upper_recond_f32", "l1_chain_kat_f64"] + G.names("simplex_")


def _solve(c, k, fixed, evolution=0, record_obj=True, spec=0):
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    a = dict(c)
    if fixed:
        a.update(difTol=0.0, difRcd=0.0, itMax=G.FIXED_K)
    if str(a["solver"]) == "simplex":  # K-wide halos
        P0 = a["P0"]
        return P.solve_loopback(
            k, pfdr.PFDR_KIND_SIMPLEX, P0.dtype, a["Eu"], a["Ev"], a["La_d1"], P0, a["Q"],
            La_l1=a["La_f"], rho=float(a["rho"]), condMin=float(a["condMin"]),
            difRcd=float(a["difRcd"]), difTol=float(a["difTol"]), itMax=int(a["itMax"]),
            record_obj=record_obj, record_dif=True, K=int(a["K"]), al=float(a["al"]),
            evolution=evolution, spec=spec)
    kind = pfdr.PFDR_KIND_L1 if str(a["solver"]) == "l1" else pfdr.PFDR_KIND_BOUNDS
    X0 = a["X0"]
    return P.solve_loopback(
        k, kind, X0.dtype, a["Eu"], a["Ev"], a["La_d1"], X0, a["Y"], A=a["A"], N=int(a["N"]),
        La_l1=a.get("La_l1"), positivity=int(a.get("positivity", 0)),
        lo=float(a.get("lo", -np.inf)), hi=float(a.get("hi", np.inf)), Ltype=int(a["Ltype"]),
        L=a["L"], rho=float(a["rho"]), condMin=float(a["condMin"]),
        difRcd=float(a["difRcd"]), difTol=float(a["difTol"]), itMax=int(a["itMax"]),
        record_obj=record_obj, record_dif=True, evolution=evolution, spec=spec)


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("k", [2, 3])
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
def test_partitioned_equals_reference(gpu_lib, name, k, fixed):
    c, g = G.load(name)
    V = c["X0"].size if "X0" in c else c["P0"].size // int(c["K"])
    if V < 4 * k:
        pytest.skip("graph too small for %d ranks" % k)
    X, it, Obj, Dif, info = _solve(c, k, fixed)
    tag = "fixk" if fixed else "conv"
    print("%s k=%d %s it=%d/%d edges/rank=%s bitexact=%s" % (
        name, k, tag, it, int(g[tag + "_it"]), info["edges"], np.array_equal(X, g[tag + "_X"])))
    assert it == int(g[tag + "_it"])
    assert np.array_equal(X, g[tag + "_X"])
    n = it
    assert G.rel_l2(Dif[:n], g[tag + "_Dif"][:n]) <= (1e-5 if X.dtype == np.float32 else 1e-12)
    if tag + "_Obj" in g:
        go = g[tag + "_Obj"][: n + 1]
        rtol = 1e-4 if name.startswith("simplex") and X.dtype == np.float32 else 1e-5
        assert np.allclose(Obj[: n + 1], go, rtol=rtol, atol=1e-6 * np.abs(go).max())


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("k", [2, 3])
def test_partitioned_sequential_evolution_equals_reference(gpu_lib, name, k):
    """converged golden cases with the evolution summed rank to rank in the
    reference's sequential rounding (ChainSum; forced, as these graphs are
    below AUTO's 2^17 vertices): the stopping iteration and EVERY Dif equal
    the reference's bit for bit (src/PFDR_graph_quadratic_d1_l1.cpp:514-529,
    simplex src/PFDR_graph_loss_d1_simplex.cpp:653-691)"""
    from cp_pfdr_graph_d1_amd import pfdr
    c, g = G.load(name)
    V = c["X0"].size if "X0" in c else c["P0"].size // int(c["K"])
    if V < 4 * k:
        pytest.skip("graph too small for %d ranks" % k)
    X, it, Obj, Dif, info = _solve(c, k, False, pfdr.EVOLUTION_SEQUENTIAL)
    print("%s k=%d it=%d/%d" % (name, k, it, int(g["conv_it"])))
    assert it == int(g["conv_it"])
    assert np.array_equal(X, g["conv_X"])
    assert np.array_equal(Dif[:it], g["conv_Dif"][:it])


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("k", [2, 3])
@pytest.mark.parametrize("spec", ["auto", "serial"])
def test_partitioned_speculative_equals_reference(gpu_lib, name, k, spec):
    """difRcd = 0 and no objective record: the partition decides
    speculatively -- the evolution chain and decision of iteration t run on a
    second stream over the split transport, beside the halo exchanges and
    sweeps of t + 1 (X / P ping-ponged); serial: the same on the session
    stream over the one transport -- and the stopping iteration, every Dif
    and X still equal the reference's bit for bit"""
    from cp_pfdr_graph_d1_amd import pfdr
    c, g = G.load(name)
    V = c["X0"].size if "X0" in c else c["P0"].size // int(c["K"])
    if V < 4 * k:
        pytest.skip("graph too small for %d ranks" % k)
    if float(c["difRcd"]) != 0.0:
        pytest.skip("reconditioning: no speculation")
    mode = pfdr.SPEC_SERIAL if spec == "serial" else pfdr.SPEC_AUTO
    X, it, _, Dif, info = _solve(c, k, False, pfdr.EVOLUTION_SEQUENTIAL, record_obj=False,
                                 spec=mode)
    print("%s k=%d spec=%s it=%d/%d" % (name, k, spec, it, int(g["conv_it"])))
    assert all(q["speculative"] == (2 if spec == "serial" else 1) for q in info["queries"])
    assert it == int(g["conv_it"])
    assert np.array_equal(X, g["conv_X"])
    assert np.array_equal(Dif[:it], g["conv_Dif"][:it])


def test_partitioned_headline_slab_matches_single(gpu_lib):
    """weak-scaling geometry of bench.py at a small size: slabs of a jittered
    6-NN grid, 4 ranks, against the single-GPU session"""
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    shape = (40, 30, 32)
    V = 40 * 30 * 32
    Eu, Ev = pfdr.gen_knn_jitter_grid(shape, 6, 6)
    Y = pfdr.gen_piecewise(40, V, 2, np.float32)
    La = np.full(Eu.size, 0.1, np.float32)
    L1 = np.full(V, 0.01, np.float32)
    X0 = np.zeros(V, np.float32)
    s = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, Eu.size, Eu, Ev, La, X0, Y, La_l1=L1,
                     difTol=1e-5, itMax=300, record_dif=True)
    s.run(300)
    Xs, its, _, Difs = s.result()
    s.close()
    X, it, _, Dif, _ = P.solve_loopback(4, pfdr.PFDR_KIND_L1, np.float32, Eu, Ev, La, X0, Y,
                                        La_l1=L1, difTol=1e-5, itMax=300, record_dif=True)
    assert it == its
    assert np.array_equal(X, Xs)
    # the evolution summed rank to rank like the single GPU (both sequential)
    kw = dict(La_l1=L1, difTol=1e-5, itMax=300, record_dif=True,
              evolution=pfdr.EVOLUTION_SEQUENTIAL)
    s = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, Eu.size, Eu, Ev, La, X0, Y, **kw)
    s.run(300)
    Xs, its, _, Difs = s.result()
    s.close()
    X, it, _, Dif, _ = P.solve_loopback(4, pfdr.PFDR_KIND_L1, np.float32, Eu, Ev, La, X0, Y, **kw)
    assert it == its
    assert np.array_equal(Dif[:it], Difs[:its])
    assert np.array_equal(X, Xs)


@pytest.mark.parametrize("k", [2, 3])
def test_partitioned_tiled_ratio_matches_single(gpu_lib, k):
    """tiled ranks (590K / 393K vertices each) with one edge weight, untracked:
    every rank's edge sweep reads the formed per-vertex ratios of its owned
    and ghost ends (k_ratio_vertex over the pulled metric) -- the iterate
    equals the single-GPU session's (itself on the ratio edge sweep and the
    pair vertex sweep) bit for bit"""
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    dt = np.float32
    shape = (128, 96, 96)
    V = int(np.prod(shape))
    Eu, Ev = grid_graph(shape, 6)
    Eu, Ev = Eu.astype(np.int32), Ev.astype(np.int32)
    Y = piecewise_observation(shape, 5, dt)
    La = np.full(Eu.size, 0.1, dt)
    L1 = np.full(V, 0.01, dt)
    X0 = np.zeros(V, dt)
    s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, La, X0, Y, La_l1=L1, itMax=20)
    assert s.query("edge_ratio") == 1 and s.query("vertex_pair") > 0
    s.run(20)
    Xs, its, _, _ = s.result()
    s.close()
    X, it, _, _, info = P.solve_loopback(k, pfdr.PFDR_KIND_L1, dt, Eu, Ev, La, X0, Y, La_l1=L1,
                                         itMax=20)
    print([(q["tiled_blocks"], q["edge_ratio"], q["vertex_pair"]) for q in info["queries"]])
    assert all(q["tiled_blocks"] > 0 and q["edge_ratio"] == 1 for q in info["queries"])
    assert it == its == 20
    assert np.array_equal(X, Xs)


def test_rccl_transport_single_rank(gpu_lib):
    """the RCCL transport code path (comm init, grouped send/recv, all-reduce,
    broadcast, chain) on a 1-rank communicator: equals the plain session"""
    import ctypes as C
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    lib = pfdr.load()
    idb = (C.c_char * 128)()
    assert lib.pfdr_comm_unique_id(idb) == 0
    comm = C.c_void_p()
    assert lib.pfdr_comm_init(C.byref(comm), 1, 0, idb) == 0, lib.pfdr_last_error()
    c, g = G.load("l1_grid2d_f32")
    a = dict(c, difTol=0.0, difRcd=0.0, itMax=G.FIXED_K)
    V = a["X0"].size
    s = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, a["Eu"].size, a["Eu"], a["Ev"],
                     a["La_d1"], a["X0"], a["Y"], La_l1=a["La_l1"], rho=float(a["rho"]),
                     condMin=float(a["condMin"]), itMax=G.FIXED_K, record_dif=True,
                     record_obj=True, nranks=1, rank=0, comm=comm.value,
                     comm_kind=P.COMM_RCCL, vtx_begin=0, V_global=V)
    s.run(G.FIXED_K)
    X, it, Obj, Dif = s.result()
    s.close()
    v = C.c_double(3.5)
    assert lib.pfdr_comm_allreduce_max_f64(comm, C.byref(v)) == 0 and v.value == 3.5
    lib.pfdr_comm_destroy(comm)
    assert it == G.FIXED_K and np.array_equal(X, g["fixk_X"])


@pytest.mark.parametrize("kind", ["l1", "simplex"])
def test_rccl_single_rank_graph_replay(gpu_lib, kind):
    """RCCL partitioned sessions replay their chunks of iterations as
    hipGraphs (the pull / push exchanges and the all-reduces captured with
    the sweeps), re-captured after every reconditioning: on a 1-rank
    communicator the iterates, iteration count and Dif equal the single-GPU
    session's with the same (tree) evolution sums, bit for bit"""
    import ctypes as C
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation, simplex_observation
    lib = pfdr.load()
    idb = (C.c_char * 128)()
    assert lib.pfdr_comm_unique_id(idb) == 0
    comm = C.c_void_p()
    assert lib.pfdr_comm_init(C.byref(comm), 1, 0, idb) == 0, lib.pfdr_last_error()
    dt = np.float32
    shape = (128, 96)
    V = int(np.prod(shape))
    if kind == "l1":
        Eu, Ev = grid_graph(shape, 4)
        args = (pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
                np.zeros(V, dt), piecewise_observation(shape, 3, dt))
        kw = dict(La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3, difTol=1e-5, difRcd=1e-2)
    else:
        Eu, Ev = grid_graph(shape, 8)
        v = np.arange(V)
        Q = simplex_observation(V, 4, 4, (v * 4) // V, dt)
        args = (pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.05, dt),
                Q.copy(), Q)
        kw = dict(K=4, al=0.1, rho=1.0, condMin=0.1, difTol=1e-5, difRcd=1e-2)
    kw.update(itMax=1000, record_dif=True, evolution=pfdr.EVOLUTION_TREE)
    try:
        out = []
        for part in (False, True):
            extra = dict(nranks=1, rank=0, comm=comm.value, comm_kind=P.COMM_RCCL, vtx_begin=0,
                         V_global=V) if part else {}
            s = pfdr.Session(*args, **kw, **extra)
            try:
                if part:
                    assert s.query("graphs") == 1
                for n in (50, 950):  # a partial chunk launched, whole ones replayed
                    s.run(n)
                out.append(s.result())
            finally:
                s.close()
    finally:
        lib.pfdr_comm_destroy(comm)
    (X0, it0, _, D0), (X1, it1, _, D1) = out
    print("%s: it %d / %d" % (kind, it0, it1))
    assert 0 < it0 < 1000 and it1 == it0
    assert np.array_equal(X1, X0)
    assert np.array_equal(D1[:it1], D0[:it0])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_partitioned_simplex_grid_matches_single(gpu_lib, dt):
    """C4's shape at a small size: K = 6 labels, KL loss, 8-neighbour grid,
    4 ranks with K-wide halos against the single-GPU session (fixed
    iterations, one reconditioning on the way)"""
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, simplex_observation
    n, K = 48, 6
    Eu, Ev = grid_graph((n, n), 8)
    V = n * n
    v = np.arange(V)
    lab = ((v % n) * 3 // n) + 3 * ((v // n) * 2 // n)
    Q = simplex_observation(V, K, 4, lab, dt)
    La = np.full(Eu.size, 0.05, dt)
    kw = dict(rho=1.0, condMin=0.1, difRcd=1e-2, difTol=0.0, itMax=40, record_dif=True)
    s = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev, La, Q.copy(), Q, K=K,
                     al=0.1, **kw)
    s.run(40)
    X1, it1, _, D1 = s.result()
    s.close()
    X, it, _, D, info = P.solve_loopback(4, pfdr.PFDR_KIND_SIMPLEX, dt, Eu, Ev, La, Q.copy(), Q,
                                         K=K, al=0.1, **kw)
    assert it == it1 == 40
    assert np.array_equal(X, X1)
    assert G.rel_l2(D[:it], D1[:it]) <= (1e-5 if dt == np.float32 else 1e-12)


DENSE_CASES = ["l1_direct_f32", "l1_direct_f64", "l1_AtA_f32", "l1_AtA_f64", "bounds_AtA_f64"]


@pytest.mark.parametrize("name", DENSE_CASES)
@pytest.mark.parametrize("k", [2, 3])
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
def test_partitioned_dense_matches_reference(gpu_lib, name, k, fixed):
    """dense A on the partition: column blocks, R summed over the ranks
    (all-reduce of A X) or X gathered (A^tA); the dot products regroup, so
    the single-GPU dense tolerances apply"""
    c, g = G.load(name)
    X, it, Obj, Dif, info = _solve(c, k, fixed)
    tag = "fixk" if fixed else "conv"
    gX, git = g[tag + "_X"], int(g[tag + "_it"])
    err = G.rel_l2(X, gX)
    print("%s k=%d %s it=%d/%d rel_l2=%.3e" % (name, k, tag, it, git, err))
    if fixed:
        assert it == git
        assert err <= (2e-5 if X.dtype == np.float32 else 1e-12)
    else:
        assert abs(it - git) <= 2
        assert err <= (1e-5 if X.dtype == np.float32 else 1e-9)


@pytest.mark.parametrize("k", [2, 3])
@pytest.mark.parametrize("kind", ["l1", "bounds", "simplex"])
def test_relabelled_partition_random_labels(gpu_lib, k, kind):
    """a randomly labelled graph is relabelled (breadth-first
    locality order) before the vertex-range split.  The gathered iterate, in
    the caller's labels, equals the single-GPU session's bit for bit (the
    sums keep the original edge ids; the l1 / bounds preconditioner's
    amplitude is summed in the caller's label order on every rank), and the
    ranks hold a small fraction of the ghosts of the random-label split."""
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation, uniform
    shape = (40, 36, 30)
    V = int(np.prod(shape))
    Eu, Ev = grid_graph(shape, 6)
    new_of = np.empty(V, np.int64)
    new_of[np.argsort(uniform(13, np.arange(V)), kind="stable")] = np.arange(V)
    Eu, Ev = new_of[Eu].astype(np.int32), new_of[Ev].astype(np.int32)
    dt = np.float32
    La = np.full(Eu.size, 0.1, dt)
    its = 30
    if kind == "simplex":
        K = 4
        lab = (np.arange(V) * 4) // V
        Q = np.zeros((V, K), dt)
        Q[np.arange(V), lab] = 1.0
        Q = (0.7 * Q + 0.3 * uniform(5, np.arange(V * K)).reshape(V, K)).astype(dt)
        Q = (Q / Q.sum(axis=1, keepdims=True)).astype(dt)
        Qp = np.empty_like(Q)
        Qp[new_of] = Q
        Qp = Qp.reshape(-1)
        kw = dict(K=K, al=0.1, rho=1.0, condMin=0.1, itMax=its)
        s = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev, La, Qp.copy(), Qp, **kw)
        args = (k, pfdr.PFDR_KIND_SIMPLEX, dt, Eu, Ev, La, Qp.copy(), Qp)
    else:
        Y0 = piecewise_observation(shape, 3, dt)
        Y = np.empty_like(Y0)
        Y[new_of] = Y0
        kind_c = pfdr.PFDR_KIND_L1 if kind == "l1" else pfdr.PFDR_KIND_BOUNDS
        kw = dict(rho=1.5, condMin=1e-3, itMax=its)
        kw.update(dict(La_l1=np.full(V, 0.01, dt)) if kind == "l1" else dict(lo=0.0, hi=0.8))
        s = pfdr.Session(kind_c, dt, V, Eu.size, Eu, Ev, La, np.zeros(V, dt), Y, **kw)
        args = (k, kind_c, dt, Eu, Ev, La, np.zeros(V, dt), Y)
    s.run(its)
    X1, it1, _, _ = s.result()
    s.close()
    Xr, itr, _, _, info = P.solve_loopback(*args, relabel=True, **kw)
    Xp, itp, _, _, info0 = P.solve_loopback(*args, **kw)
    g_rel = sum(q["ghosts"] for q in info["queries"])
    g_raw = sum(q["ghosts"] for q in info0["queries"])
    print("%s k=%d ghosts: relabelled %d, random labels %d" % (kind, k, g_rel, g_raw))
    assert it1 == itr == itp == its
    assert np.array_equal(Xr, X1)
    assert np.array_equal(Xp, X1)
    assert g_rel * 5 < g_raw
    # tracked, converged: the relabelled ranks gather their evolution terms at
    # the caller's labels and sum them in that order (sequential rounding)
    kw.update(itMax=2000, difTol=1e-4 if kind == "simplex" else 1e-5, record_dif=True,
              evolution=pfdr.EVOLUTION_SEQUENTIAL)
    s = pfdr.Session(args[1], dt, V, Eu.size, *args[3:], **kw)
    s.run(kw["itMax"])
    X1, it1, _, D1 = s.result()
    s.close()
    Xr, itr, _, Dr, info = P.solve_loopback(*args, relabel=True, **kw)
    print("%s k=%d converged: it %d / %d" % (kind, k, it1, itr))
    # difRcd = 0: speculative ranks, their terms routed to caller-order slices
    assert all(q["speculative"] == 1 and q["seqdif"] == 1 for q in info["queries"])
    assert 0 < it1 < kw["itMax"] and itr == it1
    assert np.array_equal(Dr[:itr], D1[:it1])
    assert np.array_equal(Xr, X1)


class _env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        import os
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        import os
        for k, v in self.old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("kind", ["l1", "simplex"])
def test_rccl_single_rank_real_calls_graph_replay(gpu_lib, kind):
    """PFDR_RCCL_SELF=1: a 1-rank communicator issues its collectives (the
    evolution chain's all-reduce and broadcast, the setup's all-reduces) as
    real RCCL calls instead of returning early, and the chunks of iterations
    capture them in hipGraphs: the iterates, counts and Dif equal the
    single-GPU session's bit for bit.  (Point-to-point to the rank itself
    crashed inside RCCL on this image: not exercised.)"""
    import ctypes as C
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation, simplex_observation
    lib = pfdr.load()
    dt = np.float32
    shape = (128, 96)
    V = int(np.prod(shape))
    if kind == "l1":
        Eu, Ev = grid_graph(shape, 4)
        args = (pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
                np.zeros(V, dt), piecewise_observation(shape, 3, dt))
        kw = dict(La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3, difTol=1e-5, difRcd=1e-2)
    else:
        Eu, Ev = grid_graph(shape, 8)
        v = np.arange(V)
        Q = simplex_observation(V, 4, 4, (v * 4) // V, dt)
        args = (pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.05, dt),
                Q.copy(), Q)
        kw = dict(K=4, al=0.1, rho=1.0, condMin=0.1, difTol=1e-5, difRcd=1e-2)
    kw.update(itMax=1000, record_dif=True, evolution=pfdr.EVOLUTION_SEQUENTIAL)
    out = []
    with _env(PFDR_RCCL_SELF="1"):
        idb = (C.c_char * 128)()
        assert lib.pfdr_comm_unique_id(idb) == 0
        comm = C.c_void_p()
        assert lib.pfdr_comm_init(C.byref(comm), 1, 0, idb) == 0, lib.pfdr_last_error()
        try:
            for part in (False, True):
                extra = dict(nranks=1, rank=0, comm=comm.value, comm_kind=P.COMM_RCCL,
                             vtx_begin=0, V_global=V) if part else {}
                s = pfdr.Session(*args, **kw, **extra)
                try:
                    if part:
                        assert s.query("graphs") == 1
                    for n in (50, 950):
                        s.run(n)
                    out.append(s.result())
                finally:
                    s.close()
        finally:
            lib.pfdr_comm_destroy(comm)
    (X0, it0, _, D0), (X1, it1, _, D1) = out
    print("%s: it %d / %d" % (kind, it0, it1))
    assert 0 < it0 < 1000 and it1 == it0
    assert np.array_equal(X1, X0)
    assert np.array_equal(D1[:it1], D0[:it0])


def test_rccl_split_communicator_kept(gpu_lib):
    """Speculative sessions on one RCCL communicator reuse the split
    communicator kept with it (one collective ncclCommSplit per parent, not
    per session); a second session alive at the same time splits its own;
    PFDR_SPLIT_CACHE=0 splits per session.  Every session's iterates, count
    and Dif equal the single-GPU session's."""
    import ctypes as C
    import time
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    lib = pfdr.load()
    dt = np.float32
    shape = (128, 96)
    V = int(np.prod(shape))
    Eu, Ev = grid_graph(shape, 4)
    args = (pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
            np.zeros(V, dt), piecewise_observation(shape, 3, dt))
    kw = dict(La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3, difTol=1e-5, difRcd=0.0,
              itMax=1000, record_dif=True, evolution=pfdr.EVOLUTION_SEQUENTIAL)
    s = pfdr.Session(*args, **kw)
    s.run(1000)
    X0, it0, _, D0 = s.result()
    s.close()

    def check(sess):
        sess.run(1000)
        X, it, _, D = sess.result()
        assert it == it0 and np.array_equal(X, X0) and np.array_equal(D[:it], D0[:it0])

    idb = (C.c_char * 128)()
    assert lib.pfdr_comm_unique_id(idb) == 0
    comm = C.c_void_p()
    assert lib.pfdr_comm_init(C.byref(comm), 1, 0, idb) == 0, lib.pfdr_last_error()
    extra = dict(nranks=1, rank=0, comm=comm.value, comm_kind=P.COMM_RCCL, vtx_begin=0,
                 V_global=V)
    setup = {}
    try:
        for cache in ("1", "0"):
            with _env(PFDR_SPLIT_CACHE=cache):
                ts = []
                for _ in range(3):
                    t = time.perf_counter()
                    a1 = pfdr.Session(*args, **kw, **extra)
                    ts.append(time.perf_counter() - t)
                    try:
                        assert a1.query("speculative") == 1
                        a2 = pfdr.Session(*args, **kw, **extra)  # alive beside it: its own split
                        try:
                            check(a2)
                        finally:
                            a2.close()
                        check(a1)
                    finally:
                        a1.close()
                setup[cache] = ts
    finally:
        lib.pfdr_comm_destroy(comm)
    print("session setup (s), split kept:", ["%.4f" % t for t in setup["1"]],
          "split per session:", ["%.4f" % t for t in setup["0"]])


@pytest.mark.slow
@pytest.mark.parametrize("spec", ["auto", "serial", "off"])
def test_rccl_single_rank_real_calls_headline_conv(gpu_lib, spec):
    """the converged full-size headline (10M vertices, 60M edges, difTol
    1e-5) as a 1-rank RCCL partition with PFDR_RCCL_SELF=1 (real 1-rank
    collectives), in every
    speculation mode: auto (the evolution chain on a split communicator and a
    second stream), serial (one stream, one communicator), off (the plain
    loop, its chunks captured in hipGraphs with the RCCL calls inside):
    sha256 of X, the iteration count and every Dif equal the reference's"""
    import ctypes as C
    import fullsize_cases as F
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize",
                             "headline_conv.npz"))
    case = F.build("headline_conv")
    assert F.input_digest(case) == str(g["in_sha256"])
    a = case["args"]
    lib = pfdr.load()
    mode = {"auto": pfdr.SPEC_AUTO, "serial": pfdr.SPEC_SERIAL, "off": pfdr.SPEC_OFF}[spec]
    V = a["X0"].size
    with _env(PFDR_RCCL_SELF="1"):
        idb = (C.c_char * 128)()
        assert lib.pfdr_comm_unique_id(idb) == 0
        comm = C.c_void_p()
        assert lib.pfdr_comm_init(C.byref(comm), 1, 0, idb) == 0, lib.pfdr_last_error()
        try:
            s = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, a["Eu"].size, a["Eu"], a["Ev"],
                             a["La_d1"], a["X0"], a["Y"], La_l1=a["La_l1"], Ltype=a["Ltype"],
                             L=a["L"], rho=a["rho"], condMin=a["condMin"], difRcd=a["difRcd"],
                             difTol=a["difTol"], itMax=a["itMax"], record_dif=True, nranks=1,
                             rank=0, comm=comm.value, comm_kind=P.COMM_RCCL, vtx_begin=0,
                             V_global=V, spec=mode)
            try:
                q = {k: s.query(k) for k in ("speculative", "graphs", "seqdif")}
                s.prepare(a["itMax"])
                s.run(a["itMax"])
                X, it, _, Dif = s.result()
            finally:
                s.close()
        finally:
            lib.pfdr_comm_destroy(comm)
    d = F.digest(X, it, Dif[:it], case["sample_m"])
    print("headline_conv 1-rank RCCL (self calls) spec=%s %s: it %d/%d sha256 equal %s" % (
        spec, q, it, int(g["it"]), str(d["sha256"]) == str(g["sha256"])))
    assert q["seqdif"] == 1
    assert q["speculative"] == {"auto": 1, "serial": 2, "off": 0}[spec]
    if spec == "off":
        assert q["graphs"] == 1  # the RCCL calls replayed inside captured chunks
    assert it == int(g["it"])
    assert np.array_equal(Dif[:it], g["Dif"][:it])
    assert str(d["sha256"]) == str(g["sha256"])
