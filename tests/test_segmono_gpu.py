"""GPU: ordered segment sums of very long segments (a giant component's l1
weights, a reduced edge's group of TV weights, the simplex driver's label
sums, the CP builder's component sums) by the binade scan of
pfdr_monosum.hpp when every term is nonnegative and finite
(pfdr_cpgraph.hip segsum; a segment with a negative or non-finite term
keeps one workgroup).  Both must equal the oracle (the reference's sequential loops,
oracle/cp_graph_body.h, oracle/cp_reduce_body.h) bit for bit: segments of
75,000 terms, a segment with a negative term (falls back), a signed
observation vector next to a positive diagonal."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _eq(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    if a.dtype.kind == "f":
        b = np.ascontiguousarray(b, a.dtype)
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), (what, np.flatnonzero(a != b)[:5])
    else:
        assert np.array_equal(a, b), (what, np.flatnonzero(a != b)[:5])


def _quadrants(nx=600, ny=500):
    """a 4-NN grid cut into four giant components (~75,000 vertices each)"""
    from cp_pfdr_graph_d1_amd.graphs import grid_graph
    Eu, Ev = grid_graph((nx, ny), 4)
    x, y = np.arange(nx * ny) % nx, np.arange(nx * ny) // nx
    q = (x >= nx // 2).astype(np.int64) + 2 * (y >= ny // 2)
    act = (q[Eu] != q[Ev]).astype(np.uint8)
    return nx * ny, Eu, Ev, act


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("negative", [False, True], ids=["nonneg", "negative_term"])
def test_reduced_graph_giant_components(gpu_lib, oracle_port, dt, negative):
    from cp_pfdr_graph_d1_amd.pfdr import CPGraph
    o = oracle_port
    V, Eu, Ev, act = _quadrants()
    rng = np.random.default_rng(17)
    La = (0.01 + rng.random(Eu.size)).astype(dt)
    L1 = (0.02 * rng.random(V) + 1e-3).astype(dt)
    if negative:
        L1[V // 3] = -L1[V // 3]  # one component's sum leaves mono_sum's domain
    oCv, oVc, orVc = o.cp_components(V, Eu, Ev, act)
    assert orVc.size - 1 == 4
    eps = float(np.finfo(dt).eps)
    ored = o.cp_reduced_graph(V, Eu, Ev, La, L1, act, oCv, oVc, orVc, eps)
    g = CPGraph(V, Eu, Ev, La, L1)
    try:
        g.set_active(act)
        Cv, Vc, rVc = g.components()
        _eq(Vc, oVc, "Vc")
        red = g.reduced_graph(eps)
        for a, b, nm in zip(red, ored, ("rEu", "rEv", "rLa_d1", "rLa_l1")):
            _eq(a, b, nm)
    finally:
        g.close()


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_simplex_observations_giant_components(gpu_lib, oracle_port, dt):
    from cp_pfdr_graph_d1_amd.pfdr import CPGraph
    o = oracle_port
    V, Eu, Ev, act = _quadrants()
    K = 4
    rng = np.random.default_rng(23)
    Q = rng.random((V, K))
    Q = (Q / Q.sum(axis=1, keepdims=True)).reshape(-1).astype(dt)
    La = np.full(Eu.size, 0.05, dt)
    for al in (0.0, 0.3):
        g = CPGraph(V, Eu, Ev, La)
        try:
            g.simplex_setup(K, al, Q)
            g.set_active(act)
            Cv, Vc, rVc = g.components()
            oP, oQ, oL = o.cp_simplex_reduced(K, al, Q, Vc, rVc)
            rP, rQ, rL = g.simplex_observations()
            _eq(rP, oP, "rP")
            _eq(rQ, oQ, "rQ")
            if oL is not None:
                _eq(rL, oL, "rLa_f")
        finally:
            g.close()


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_builder_long_components(gpu_lib, oracle_port, dt):
    """N = 0 builder: rAA = component sums of a positive diagonal (binade
    scan), rY = component sums of a signed Y (one workgroup each)"""
    from cp_pfdr_graph_d1_amd import pfdr
    V, rV = 200000, 3
    rng = np.random.default_rng(29)
    lab = rng.integers(0, rV, V)
    lab[:rV] = np.arange(rV)
    order = rng.permutation(V)
    Vc = np.concatenate([order[lab[order] == r] for r in range(rV)]).astype(np.int32)
    ptr = np.r_[0, np.cumsum(np.bincount(lab, minlength=rV))].astype(np.int32)
    A = (0.5 + rng.random(V)).astype(dt)
    Y = (rng.random(V) - 0.5).astype(dt)
    o = oracle_port.cp_reduce(0, A, Y, ptr, Vc, preAt=True)
    g = pfdr.cp_reduce(0, A, Y, ptr, Vc, preAt=True, normTol=1e-6, normItMax=500)
    for k in ("rAA", "rY"):
        assert np.array_equal(g[k], o[k]), k
