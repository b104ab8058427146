"""GPU: partitioned ranks in tile order (SURVEY.md §8(e) at the sizes the
multi-GPU bench runs: every rank past the small-graph range).

A rank sorts its edges by (u block, v block) like a single GPU, with the
edges that have a ghost end after all the others, so the tiled edge sweep
runs the interior edge blocks while the halo pull is in flight and the rest
after it; the vertex sweep finds the u ends of those boundary edges and the
received contributions as extra runs of its blocks, each entry with its slot
in the reference's (e, side) order.  Expected bit-exact against the
single-GPU session: iterates, iteration count and Dif (the evolution is
summed rank to rank with the reference's sequential rounding), with k ranks
as k threads on one GPU (loopback transport) and on a one-rank RCCL
communicator (hipGraph-replayed chunks).  The edge block that straddles a
rank's interior / boundary cut is covered deterministically by
tests/test_erec_gpu.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _single(args, kw):
    from cp_pfdr_graph_d1_amd import pfdr
    s = pfdr.Session(*args, **kw)
    try:
        s.run(kw["itMax"])
        return s.result()
    finally:
        s.close()


@pytest.mark.parametrize("k,dt,conv", [(2, np.float32, False), (3, np.float32, True),
                                       (2, np.float64, True)],
                         ids=["k2-f32-fixk", "k3-f32-conv", "k2-f64-conv"])
def test_tiled_partition_matches_single(gpu_lib, k, dt, conv):
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import uniform
    shape = (80, 80, 128)  # 819,200 vertices: every rank past 1,024 blocks at k <= 3
    V = int(np.prod(shape))
    Eu, Ev = pfdr.gen_knn_jitter_grid(shape, 6, 6, 0.25)
    Y = pfdr.gen_piecewise(shape[0], V, 2, dt, 0.2)
    if conv:  # per-edge weights (the streamed-weight sweep), reconditioning, tolerance
        La = (0.05 + 0.1 * uniform(3, np.arange(Eu.size))).astype(dt)
        kw = dict(difTol=1e-4, difRcd=1e-2, itMax=600)
    else:
        La = np.full(Eu.size, 0.1, dt)
        kw = dict(difTol=0.0, difRcd=0.0, itMax=20)
    kw.update(La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3, record_dif=True)
    X0 = np.zeros(V, dt)
    Xs, its, _, Ds = _single((pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, La, X0, Y), kw)
    X, it, _, D, info = P.solve_loopback(k, pfdr.PFDR_KIND_L1, dt, Eu, Ev, La, X0, Y, **kw)
    q = info["queries"]
    print(k, dt.__name__, "it", it, its, q)
    assert all(r["tiled_blocks"] > 0 and r["ghosts"] > 0 for r in q)
    assert it == its and (conv or it == 20)
    assert np.array_equal(D[:it], Ds[:its])
    assert np.array_equal(X, Xs)


@pytest.mark.parametrize("k,width,dup", [(2, 420, True), (3, 420, True), (2, 640, False)],
                         ids=["k2-w420-mirrored", "k3-w420-mirrored", "k2-w640"])
def test_tiled_partition_narrow_grid(gpu_lib, k, width, dup):
    """a narrow 2-D grid (bandwidth 420 / 640 vertices, 1-3 u blocks): every
    rank past 1,024 vertex blocks, its boundary edges starting one or two u
    blocks below the interior edges they follow, so the edge block that
    straddles the cut drops its u block by less than the LDS stage spans --
    the case where a staged lookup would read the wrong u end (k_tile_erec
    marks such a block unstaged).  Mirrored duplicates give every rank
    ghost edges."""
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    shape = (width, 1400 * k // 2 + 300)
    V = int(np.prod(shape))
    Eu, Ev = grid_graph(shape, 4)
    if dup:
        Eu, Ev = np.concatenate([Eu, Ev]), np.concatenate([Ev, Eu])
    dt = np.float32
    Y = piecewise_observation(shape, 3, dt)
    La = np.full(Eu.size, 0.1, dt)
    kw = dict(La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3, difTol=0.0, difRcd=0.0,
              itMax=30, record_dif=True)
    X0 = np.zeros(V, dt)
    Xs, its, _, _ = _single((pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, La, X0, Y), kw)
    X, it, _, _, info = P.solve_loopback(k, pfdr.PFDR_KIND_L1, dt, Eu, Ev, La, X0, Y, **kw)
    q = info["queries"]
    print(k, width, q)
    assert all(r["tiled_blocks"] > 0 for r in q)
    assert all(r["ghosts"] > 0 for r in q) or not dup
    assert it == its == 30
    assert np.array_equal(X, Xs)


def test_tiled_partition_bounds_random_labels(gpu_lib):
    """box constraint, randomly labelled vertices relabelled before the
    split (locality order), 2 ranks"""
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation, uniform
    shape = (96, 80, 80)
    V = int(np.prod(shape))
    Eu, Ev = grid_graph(shape, 6)
    new_of = np.empty(V, np.int64)
    new_of[np.argsort(uniform(13, np.arange(V)), kind="stable")] = np.arange(V)
    Eu, Ev = new_of[Eu].astype(np.int32), new_of[Ev].astype(np.int32)
    dt = np.float32
    Y0 = piecewise_observation(shape, 3, dt)
    Y = np.empty_like(Y0)
    Y[new_of] = Y0
    La = np.full(Eu.size, 0.1, dt)
    kw = dict(lo=0.0, hi=0.8, rho=1.5, condMin=1e-3, itMax=25, record_dif=True)
    Xs, its, _, _ = _single((pfdr.PFDR_KIND_BOUNDS, dt, V, Eu.size, Eu, Ev, La, np.zeros(V, dt), Y),
                            kw)
    X, it, _, _, info = P.solve_loopback(2, pfdr.PFDR_KIND_BOUNDS, dt, Eu, Ev, La,
                                         np.zeros(V, dt), Y, relabel=True, **kw)
    print(info["queries"])
    assert all(r["tiled_blocks"] > 0 for r in info["queries"])
    assert it == its == 25
    assert np.array_equal(X, Xs)


def test_tiled_rccl_single_rank_graph_replay(gpu_lib):
    """a one-rank RCCL session past the small-graph range: tiled, chunks of
    iterations replayed as hipGraphs with the (empty) exchanges captured,
    re-captured after each reconditioning; equals the single-GPU session"""
    import ctypes as C
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    lib = pfdr.load()
    idb = (C.c_char * 128)()
    assert lib.pfdr_comm_unique_id(idb) == 0
    comm = C.c_void_p()
    assert lib.pfdr_comm_init(C.byref(comm), 1, 0, idb) == 0, lib.pfdr_last_error()
    dt = np.float32
    shape = (700, 600)
    V = int(np.prod(shape))
    Eu, Ev = grid_graph(shape, 4)
    args = (pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
            np.zeros(V, dt), piecewise_observation(shape, 3, dt))
    kw = dict(La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3, difTol=1e-5, difRcd=1e-2,
              itMax=1000, record_dif=True, evolution=pfdr.EVOLUTION_TREE)
    try:
        out = []
        for part in (False, True):
            extra = dict(nranks=1, rank=0, comm=comm.value, comm_kind=P.COMM_RCCL, vtx_begin=0,
                         V_global=V) if part else {}
            s = pfdr.Session(*args, **kw, **extra)
            try:
                assert s.query("tiled_blocks") > 0
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
    print("it %d / %d" % (it0, it1))
    assert 0 < it0 < 1000 and it1 == it0
    assert np.array_equal(X1, X0)
    assert np.array_equal(D1[:it1], D0[:it0])
