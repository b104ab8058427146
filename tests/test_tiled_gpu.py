"""GPU: tile-ordered contributions (tile_sum, csrc/pfdr_quadratic_kernels.hpp).

Large single-GPU graphs (past the fused small-graph range) keep their edges
sorted by (u block, v block, edge): the edge sweep writes both contributions
as streams and every vertex block stages its own contributions from a few
contiguous runs, each entry carrying its slot in the block's CSR order, so
the per-vertex sums run in the reference's (e, side) order without a
gathered load.  Blocks whose lists exceed the LDS list (hubs) keep the CSR
gather.  Every case must equal the restatement of the reference (oracle)
bit for bit: 3-D 6-neighbour grids (3 edges per vertex), jittered k-NN
lists (6 per vertex, mirrored duplicates), randomly labelled and shuffled
edges (relabelled internally first), hub vertices, f32 and f64, fixed k and
converged with reconditioning (sequential evolution sums: the reference's
decisions)."""
import numpy as np
import pytest

from cp_pfdr_graph_d1_amd import pfdr
from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation, uniform

pytestmark = pytest.mark.gpu


def _run(V, Eu, Ev, Y, dt, itMax, difTol=0.0, difRcd=0.0, La=None, reorder=pfdr.REORDER_AUTO):
    La = np.full(Eu.size, 0.1, dt) if La is None else La
    s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, La, np.zeros(V, dt), Y,
                     La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3, difTol=difTol,
                     difRcd=difRcd, itMax=itMax, record_dif=True, reorder=reorder)
    try:
        q = {k: s.query(k) for k in ("tiled_blocks", "split_blocks", "reordered", "la_uniform")}
        s.run(itMax)
        X, it, _, Dif = s.result()
    finally:
        s.close()
    return X, it, Dif, q


def _oracle(oracle_port, V, Eu, Ev, Y, dt, itMax, difTol=0.0, difRcd=0.0, La=None):
    La = np.full(Eu.size, 0.1, dt) if La is None else La
    return oracle_port.quadratic_d1_l1(np.zeros(V, dt), Y, None, 0, Eu, Ev, La,
                                       np.full(V, 0.01, dt), 0, 0, None, 1.5, 1e-3, difRcd,
                                       difTol, itMax, dif=True)


def _grid(shape, conn, seed):
    Eu, Ev = grid_graph(shape, conn)
    V = int(np.prod(shape))
    return V, Eu.astype(np.int32), Ev.astype(np.int32)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_tiled_grid_matches_oracle(gpu_lib, oracle_port, dt):
    shape = (72, 64, 64)
    V, Eu, Ev = _grid(shape, 6, 1)
    Y = piecewise_observation(shape, 3, dt)
    X, it, D, q = _run(V, Eu, Ev, Y, dt, 25)
    Xo, ito, _, Do = _oracle(oracle_port, V, Eu, Ev, Y, dt, 25)
    nb = (V + 255) // 256
    print(q)
    assert q["tiled_blocks"] == nb and q["split_blocks"] == 0
    assert it == ito == 25
    assert np.array_equal(X, Xo)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_tiled_knn_converged_matches_oracle(gpu_lib, oracle_port, dt):
    """6 nearest of 26 per vertex (mirrored duplicates), non-uniform La_d1,
    reconditioning and a tolerance: iterates, iteration count and Dif"""
    shape = (60, 60, 80)
    Eu, Ev = pfdr.gen_knn_jitter_grid(shape, 6, 6, 0.25)
    V = int(np.prod(shape))
    Y = pfdr.gen_piecewise(shape[0], V, 2, dt, 0.2)
    La = (0.05 + 0.1 * uniform(3, np.arange(Eu.size))).astype(dt)
    kw = dict(difTol=1e-4 if dt == np.float32 else 1e-5, difRcd=1e-2, La=La)
    X, it, D, q = _run(V, Eu, Ev, Y, dt, 2000, **kw)
    Xo, ito, _, Do = _oracle(oracle_port, V, Eu, Ev, Y, dt, 2000, **kw)
    print(q, it, ito)
    assert q["tiled_blocks"] > 0 and q["la_uniform"] == 0
    assert it == ito
    assert np.array_equal(D[:it], Do[:ito])
    assert np.array_equal(X, Xo)


def test_tiled_after_relabelling_matches_oracle(gpu_lib, oracle_port):
    """random vertex labels and shuffled edges (V >= 2^20: relabelled
    internally, then tile-ordered)"""
    shape = (128, 96, 96)
    V, Eu, Ev = _grid(shape, 6, 1)
    new_of = np.empty(V, np.int64)
    new_of[np.argsort(uniform(17, np.arange(V)), kind="stable")] = np.arange(V)
    ep = np.argsort(uniform(19, np.arange(Eu.size)), kind="stable")
    Eu, Ev = new_of[Eu[ep]].astype(np.int32), new_of[Ev[ep]].astype(np.int32)
    Y0 = piecewise_observation(shape, 5, np.float32)
    Y = np.empty_like(Y0)
    Y[new_of] = Y0
    X, it, _, q = _run(V, Eu, Ev, Y, np.float32, 12)
    Xo, ito, _, _ = _oracle(oracle_port, V, Eu, Ev, Y, np.float32, 12)
    print(q)
    assert q["reordered"] == 1 and q["tiled_blocks"] > 0
    assert np.array_equal(X, Xo)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_tiled_hubs_fall_back_to_the_gather(gpu_lib, oracle_port, dt):
    """hubs of 5,000 incident edges: their blocks exceed the LDS list and
    gather through the CSR; the others stage runs; bit-exact"""
    shape = (64, 64, 72)
    V, Eu, Ev = _grid(shape, 6, 1)
    hubs = np.array([5, 100000, 200001], np.int64)
    u = np.repeat(hubs, 5000)
    v = (uniform(23, np.arange(u.size)) * V).astype(np.int64)
    v[v == u] = (v[v == u] + 1) % V
    Eu = np.concatenate([Eu, u]).astype(np.int32)
    Ev = np.concatenate([Ev, v]).astype(np.int32)
    Y = piecewise_observation(shape, 7, dt)
    X, it, _, q = _run(V, Eu, Ev, Y, dt, 15)
    Xo, ito, _, _ = _oracle(oracle_port, V, Eu, Ev, Y, dt, 15)
    nb = (V + 255) // 256
    print(q)
    assert 0 < q["tiled_blocks"] < nb
    assert np.array_equal(X, Xo)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_tiled_scattered_sources(gpu_lib, oracle_port, dt):
    """random long-range edges (about 11 per vertex block): vertex blocks
    stage v ends from many short runs (up to ~30) and edge-sweep blocks see
    more v-block runs than their record holds (they read Ev); bit-exact"""
    shape = (64, 64, 72)
    V, Eu, Ev = _grid(shape, 6, 1)
    n = V // 24
    u = (uniform(29, np.arange(n)) * V).astype(np.int64)
    v = (uniform(31, np.arange(n)) * V).astype(np.int64)
    v[v == u] = (v[v == u] + 1) % V
    Eu = np.concatenate([Eu, u]).astype(np.int32)
    Ev = np.concatenate([Ev, v]).astype(np.int32)
    Y = piecewise_observation(shape, 11, dt)
    X, it, _, q = _run(V, Eu, Ev, Y, dt, 15, reorder=pfdr.REORDER_OFF)
    Xo, ito, _, _ = _oracle(oracle_port, V, Eu, Ev, Y, dt, 15)
    nb = (V + 255) // 256
    print(q)
    assert q["tiled_blocks"] == nb
    assert np.array_equal(X, Xo)



@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_tiled_sparse_rows(gpu_lib, oracle_port, dt):
    """a 2-D grid whose upper half keeps one right-hand edge in three: the
    edge-sweep blocks there span more u blocks than they stage (they read
    Eu), the dense half stages its u ends; bit-exact"""
    nx, ny = 1000, 700
    V, Eu, Ev = _grid((ny, nx), 4, 1)
    keep = (Eu < V // 2) | ((Ev == Eu + 1) & (Eu % 3 == 0))  # sparse upper rows
    Eu, Ev = Eu[keep], Ev[keep]
    Y = pfdr.gen_piecewise(nx, V, 13, dt, 0.2)
    X, it, _, q = _run(V, Eu, Ev, Y, dt, 15)
    Xo, ito, _, _ = _oracle(oracle_port, V, Eu, Ev, Y, dt, 15)
    print(q)
    assert q["tiled_blocks"] > 0
    assert np.array_equal(X, Xo)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("shape,conn", [((72, 64, 64), 6), ((640, 40, 12), 6), ((512, 600), 8)])
def test_slot_patterns_identical(gpu_lib, oracle_port, dt, shape, conn):
    """Regular grids: the record blocks' runs repeat a few slot sequences, which
    the vertex sweep reads from a small pattern table (k_run_hash) instead of
    the per-entry slot stream -- the same sums bit for bit: equal to the
    per-entry run (PFDR_TILE_PATTERNS=0) and to the oracle, fixed k and
    converged with reconditionings"""
    import os
    V, Eu, Ev = _grid(shape, conn, 1)
    Y = piecewise_observation(shape, 3, dt)
    out = []
    for pat in ("1", "0"):
        os.environ["PFDR_TILE_PATTERNS"] = pat
        try:
            s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
                             np.zeros(V, dt), Y, La_l1=np.full(V, 0.01, dt), rho=1.5,
                             condMin=1e-3, difTol=1e-6, difRcd=1e-3, itMax=400, record_dif=True,
                             evolution=pfdr.EVOLUTION_SEQUENTIAL)
            try:
                q = s.query("slot_patterns")
                s.run(400)
                out.append((s.result(), q))
            finally:
                s.close()
        finally:
            del os.environ["PFDR_TILE_PATTERNS"]
    ((X1, it1, _, D1), q1), ((X0, it0, _, D0), q0) = out
    print(shape, "patterns", q1, "it", it1)
    assert q1 > 0 and q0 == 0
    assert it1 == it0 and np.array_equal(X1, X0) and np.array_equal(D1[:it1], D0[:it0])
    Xo, ito, _, _ = oracle_port.quadratic_d1_l1(np.zeros(V, dt), Y, None, 0, Eu, Ev,
                                                 np.full(Eu.size, 0.1, dt), np.full(V, 0.01, dt),
                                                 0, 0, None, 1.5, 1e-3, 1e-3, 1e-6, 400, dif=True)
    assert ito == it1 and np.array_equal(X1, Xo)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("rcd", [0.0, 1e-3])
def test_edge_ratio_identical(gpu_lib, oracle_port, dt, rcd):
    """One edge weight, Z-direct: the tiled edge sweep reads each end's
    (c La_d1 / Aux) / Ga formed once per vertex (k_ratio_vertex) instead of
    the (Ga, 1/Aux) pair -- the quotients prox_weights forms, bit for bit:
    equal to the pair sweep (PFDR_EDGE_RATIO=0) and to the oracle; with
    reconditioning the session returns to the pair sweep at the first one"""
    import os
    shape = (72, 64, 64)
    V, Eu, Ev = _grid(shape, 6, 1)
    Y = piecewise_observation(shape, 3, dt)
    out = []
    for rat in ("1", "0"):
        os.environ["PFDR_EDGE_RATIO"] = rat
        try:
            s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
                             np.zeros(V, dt), Y, La_l1=np.full(V, 0.01, dt), rho=1.5,
                             condMin=1e-3, difTol=1e-6, difRcd=rcd, itMax=300, record_dif=True,
                             evolution=pfdr.EVOLUTION_SEQUENTIAL)
            try:
                q = s.query("edge_ratio")
                s.run(300)
                out.append((s.result(), q))
            finally:
                s.close()
        finally:
            del os.environ["PFDR_EDGE_RATIO"]
    ((X1, it1, _, D1), q1), ((X0, it0, _, D0), q0) = out
    assert q1 == 1 and q0 == 0
    assert it1 == it0 and np.array_equal(X1, X0) and np.array_equal(D1[:it1], D0[:it0])
    Xo, ito, _, _ = oracle_port.quadratic_d1_l1(np.zeros(V, dt), Y, None, 0, Eu, Ev,
                                                 np.full(Eu.size, 0.1, dt), np.full(V, 0.01, dt),
                                                 0, 0, None, 1.5, 1e-3, rcd, 1e-6, 300, dif=True)
    assert ito == it1 and np.array_equal(X1, Xo)


@pytest.mark.parametrize("track", [False, True])
def test_vertex_pair_identical(gpu_lib, oracle_port, track):
    """Regular f32 grids with at most ~10 entries per vertex: the vertex
    sweep takes two record blocks per workgroup (k_vertex_sweep_pair; an odd
    block count leaves the last one alone) -- the same sums, iterates and
    evolution partials as the one-block sweep (PFDR_VPAIR=0) and the oracle"""
    import os
    dt = np.float32
    shape = (72, 63, 63)  # 1,117 vertex blocks, the last one partial
    V, Eu, Ev = _grid(shape, 6, 1)
    Y = piecewise_observation(shape, 3, dt)
    it_max = 300 if track else 20
    kw = dict(difTol=1e-6, difRcd=1e-3, record_dif=True,
              evolution=pfdr.EVOLUTION_SEQUENTIAL) if track else dict(difTol=0.0, difRcd=0.0)
    out = []
    for pair in ("1", "0"):
        os.environ["PFDR_VPAIR"] = pair
        try:
            s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
                             np.zeros(V, dt), Y, La_l1=np.full(V, 0.01, dt), rho=1.5,
                             condMin=1e-3, itMax=it_max, **kw)
            try:
                q = s.query("vertex_pair")
                s.run(it_max)
                out.append((s.result(), q))
            finally:
                s.close()
        finally:
            del os.environ["PFDR_VPAIR"]
    ((X1, it1, _, D1), q1), ((X0, it0, _, D0), q0) = out
    print("pair cap", q1, "it", it1)
    assert q1 > 0 and q0 == 0
    assert it1 == it0 and np.array_equal(X1, X0)
    if track:
        assert np.array_equal(D1[:it1], D0[:it0])
    Xo, ito, _, _ = oracle_port.quadratic_d1_l1(np.zeros(V, dt), Y, None, 0, Eu, Ev,
                                                 np.full(Eu.size, 0.1, dt), np.full(V, 0.01, dt),
                                                 0, 0, None, 1.5, 1e-3, kw["difRcd"],
                                                 kw["difTol"], it_max, dif=True)
    assert ito == it1 and np.array_equal(X1, Xo)
