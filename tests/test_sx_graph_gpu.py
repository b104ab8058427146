"""GPU: single-GPU simplex sessions replay their iteration chunks as
hipGraphs (re-captured after a reconditioning; a profiled session launches
directly), and small ones run each chunk in one workgroup launch
(k_sx_tiny_iterate; PFDR_SX_TINY = most (edge, label) entries, 0 off, a
large value lifts the block cap to 32).  Iterates, iteration counts and the evolution record must be
identical bit for bit to the directly launched loop on
every simplex golden case (fixed-k and converged: l1 and label-count
evolution, reconditioning, La_f, self-loops) -- and, at the fixed iteration
count, to the reference's golden iterates -- and on grids stopped at a
tolerance, at itMax inside a chunk, after reconditionings, with the run
split into calls of odd and even lengths."""
import os

import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

SX = [n for n in G.names() if n.startswith("simplex_")]


class _env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("name", SX)
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
def test_sx_graph_golden_identical(gpu_lib, name, fixed):
    c, g = G.load(name)
    res = []
    for env in ({}, {"PFDR_SX_TINY": "0"}, {"PFDR_SX_TINY": "100000000"},
                {"PFDR_SX_TINY": "0", "PFDR_SX_TILE": "1"},  # edges in tile order
                {"PFDR_SX_TINY": "0", "PFDR_SX_TILE": "1", "PFDR_SX_STAGE": "1"}):  # staged sweep
        with _env(**env):
            res.append(G.replay(gpu_lib, c, fixed, obj=False, dif=True))
    X0, it0, _, D0 = res[0]
    for X1, it1, _, D1 in res[1:]:
        assert it1 == it0
        assert np.array_equal(X1, X0)
        assert np.array_equal(D1[:it1], D0[:it0])
    if fixed:
        assert np.array_equal(X0, g["fixk_X"])


CASES = [  # shape, dtype, K, al, itMax, difTol, difRcd, run() lengths
    ((40, 40), np.float32, 4, 0.1, 3000, 1e-5, 1e-2, (3000,)),
    ((40, 40), np.float64, 3, 0.0, 400, 1e-4, 0.0, (400,)),            # linear loss
    ((64, 48), np.float32, 6, 1.0, 70, 0.0, 1e-1, (70,)),              # itMax inside a chunk
    ((30, 30), np.float32, 5, 0.3, 500, 2.0, 20.0, (7, 33, 1, 64, 500)),  # label counts
    ((100, 100), np.float64, 4, 0.1, 200, 1e-9, 1e-3, (31, 200)),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%dx%d-%s-K%d-al%g" % (
    c[0][0], c[0][1], np.dtype(c[1]).name, c[2], c[3]))
def test_sx_graph_sessions_identical(gpu_lib, case):
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph
    shape, dt, K, al, itMax, difTol, difRcd, runs = case
    Eu, Ev = grid_graph(shape, 8)
    V = int(np.prod(shape))
    rng = np.random.default_rng(V + K)
    Q = rng.random((V, K))
    Q[: V // 2, 0] += 2.0
    Q = (Q / Q.sum(axis=1, keepdims=True)).reshape(-1).astype(dt)
    res = []
    for env in ({"PFDR_SX_TINY": "0"}, {"PFDR_SX_TINY": "0", "launch": "direct"},
                {"PFDR_SX_TINY": "100000000"}, {},
                {"PFDR_SX_TINY": "0", "PFDR_SX_TILE": "1"},
                {"PFDR_SX_TINY": "0", "PFDR_SX_TILE": "1", "launch": "direct"},
                {"PFDR_SX_TINY": "0", "PFDR_SX_TILE": "1", "PFDR_SX_STAGE": "1"},
                {"PFDR_SX_TINY": "0", "PFDR_SX_TILE": "1", "PFDR_SX_STAGE": "1",
                 "PFDR_SX_TILEM": "1"}):
        direct = env.pop("launch", None) == "direct"
        with _env(**env):
            s = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev,
                             np.full(Eu.size, 0.05, dt), Q.copy(), Q, K=K, al=al, rho=1.0,
                             condMin=0.1, difRcd=difRcd, difTol=difTol, itMax=itMax,
                             record_dif=True)
        try:
            nb = (V + (256 // K) - 1) // (256 // K)
            if env.get("PFDR_SX_TINY") == "100000000":
                assert s.query("tiny") == (1 if nb <= 32 else 0)
            elif env.get("PFDR_SX_TINY") == "0":
                assert s.query("tiny") == 0
            if env.get("PFDR_SX_TILE") == "1":
                assert (s.query("tiled_blocks") > 0) == (K <= 64)
            if direct:  # profiled: every chunk launched directly, no graph replay
                s.profile(True)
            for n in runs:
                s.run(n)
            res.append(s.result())
        finally:
            s.close()
    X0, it0, _, D0 = res[0]
    assert 0 < it0 <= itMax
    for X1, it1, _, D1 in res[1:]:
        assert it1 == it0
        assert np.array_equal(X1, X0)
        assert np.array_equal(D1[:it1], D0[:it0])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("K,al,difRcd", [(10, 0.1, 1e-2), (8, 1.0, 0.0), (3, 0.0, 1e-1),
                                         (64, 0.2, 0.0), (7, 0.1, 1e-2)])
def test_sx_tile_order_identical(gpu_lib, dt, K, al, difRcd):
    """Edges in tile order (PFDR_SX_TILE=1: stably sorted by (u block, v
    block), La_d1 permuted with them, the incidence keys the original ids)
    against the caller's order, on a shuffled k-NN-like graph with
    duplicates, self-loops, both end orders and per-edge weights, with and
    without reconditionings: identical iterates, counts and Dif."""
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph
    rng = np.random.default_rng(K * 7 + int(al * 10))
    Eu, Ev = grid_graph((70, 60), 8)
    V = 70 * 60
    flip = rng.random(Eu.size) < 0.3
    Eu, Ev = np.where(flip, Ev, Eu), np.where(flip, Eu, Ev)
    extra = rng.integers(0, V, (2, 500)).astype(np.int32)
    extra[1, :50] = extra[0, :50]  # self-loops
    Eu = np.concatenate([Eu, extra[0], Eu[:300]]).astype(np.int32)  # + duplicates
    Ev = np.concatenate([Ev, extra[1], Ev[:300]]).astype(np.int32)
    p = rng.permutation(Eu.size)
    Eu, Ev = Eu[p], Ev[p]
    La = (0.02 + 0.06 * rng.random(Eu.size)).astype(dt)
    Q = rng.random((V, K))
    Q[: V // 3, 1 % K] += 1.5
    Q = (Q / Q.sum(axis=1, keepdims=True)).reshape(-1).astype(dt)
    res = []
    for tile, stage in (("0", "0"), ("1", "0"), ("1", "1")):
        with _env(PFDR_SX_TINY="0", PFDR_SX_TILE=tile, PFDR_SX_STAGE=stage):
            s = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev, La, Q.copy(), Q,
                             K=K, al=al, rho=1.0, condMin=0.1, difRcd=difRcd, difTol=1e-6,
                             itMax=150, record_dif=True)
        try:
            assert (s.query("tiled_blocks") > 0) == (tile == "1")
            s.run(150)
            res.append(s.result())
        finally:
            s.close()
    X0, it0, _, D0 = res[0]
    assert it0 > 0
    for X1, it1, _, D1 in res[1:]:
        assert it0 == it1
        assert np.array_equal(X0, X1)
        assert np.array_equal(D0[:it0], D1[:it1])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("K,al", [(10, 0.1), (3, 0.0), (64, 1.0), (7, 0.1)])
def test_sx_fused_widths_identical(gpu_lib, dt, K, al):
    """The one-GPU fused sweep on workgroups of 64, 128 or 256 lanes
    (PFDR_SX_NT) or of 2 / 4 vertex blocks (PFDR_SX_M), with and without the
    padded block lists (PFDR_SX_PAD=0):
    identical iterates, counts and (sequential) Dif, tracked to a tolerance
    with reconditionings and at a fixed iteration count"""
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph
    rng = np.random.default_rng(K + 11)
    Eu, Ev = grid_graph((90, 70), 8)
    V = 90 * 70
    Q = rng.random((V, K))
    Q[: V // 2, 0] += 1.0
    Q = (Q / Q.sum(axis=1, keepdims=True)).reshape(-1).astype(dt)
    La = np.full(Eu.size, 0.05, dt)
    for kw in (dict(difTol=1e-6, difRcd=1e-2, evolution=pfdr.EVOLUTION_SEQUENTIAL),
               dict(difTol=0.0, difRcd=0.0)):
        res = []
        for env in ({"PFDR_SX_M": "1"}, {"PFDR_SX_M": "2"}, {"PFDR_SX_M": "4"},
                    {"PFDR_SX_M": "2", "PFDR_SX_PAD": "0"}, {"PFDR_SX_M": "1", "PFDR_SX_NT": "128"},
                    {"PFDR_SX_M": "1", "PFDR_SX_NT": "64"},
                    {"PFDR_SX_M": "1", "PFDR_SX_NT": "64", "PFDR_SX_PAD": "0"},
                    {"PFDR_SX_M": "1", "PFDR_SX_PAD": "0"}):
            with _env(PFDR_SX_TINY="0", **env):
                s = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev, La, Q.copy(), Q,
                                 K=K, al=al, rho=1.0, condMin=0.1, itMax=120, record_dif=True, **kw)
            try:
                s.run(120)
                res.append(s.result())
            finally:
                s.close()
        X0, it0, _, D0 = res[0]
        assert it0 > 0
        for X1, it1, _, D1 in res[1:]:
            assert it1 == it0
            assert np.array_equal(X1, X0)
            assert np.array_equal(D1[:it1], D0[:it0])
