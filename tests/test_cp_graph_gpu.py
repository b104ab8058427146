"""GPU parity of the cut-pursuit graph steps (pfdr_cpgraph_*, SURVEY.md
§8(f) ranks 2-3) through the C ABI.

* Golden replay: every recorded iteration of the reference's own cut
  pursuit (tests/golden/cp_*.npz) — gradient and capacities against the
  oracle (itself pinned to the reference), activation with the iteration's
  segments, components (Cv, Vc queue order, rVc), reduced graph and merge
  against the reference's outputs: all bit for bit.
* Larger graphs against the oracle (bit for bit): 3-D grids, a k-NN
  multigraph, a long chain (thousands of BFS levels), an edgeless graph,
  random activity patterns; dense gradients (N > 0, N = -V).
"""
import numpy as np
import pytest

import cp_cases as CC
from test_cp_graph_oracle import (BNAMES, DNAMES, NAMES, SNAMES, expansion_segments,
                                  iteration_state, load_case)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cpgraph_cls(gpu_lib):
    from cp_pfdr_graph_d1_amd.pfdr import CPGraph
    return CPGraph


def _eq(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    if a.dtype.kind == "f":
        assert np.array_equal(a.view(np.uint8), np.ascontiguousarray(b, a.dtype).view(np.uint8)), \
            (what, np.flatnonzero(a != b)[:5])
    else:
        assert np.array_equal(a, b), (what, np.flatnonzero(a != b)[:5])


@pytest.mark.parametrize("name", NAMES + BNAMES)
def test_gpu_replays_reference_cp(cpgraph_cls, oracle_port, name):
    c, d = load_case(name)
    o = oracle_port
    dt = c["Y"].dtype
    eps = CC.cp_eps(dt, c["CP_difTol"])
    g = cpgraph_cls(c["Y"].size, c["Eu"], c["Ev"], c["La_d1"], c["La_l1"])
    bounds = name in BNAMES
    if bounds:  # the bounds driver (src/CP_PFDR_graph_quadratic_d1_bounds.cpp)
        two_cuts = not (c["lo"] == -np.inf and c["hi"] == np.inf)
    else:
        two_cuts = c["La_l1"] is not None or c["positivity"]
    for k in range(int(d["meta_steps"])):
        st, new = iteration_state(d, k, "in"), iteration_state(d, k, "out")
        g.set_active(st["active"])
        g.set_components(st["Cv"], st["Vc"], st["rVc"])
        g.set_values(st["rX"])
        DfS = g.gradient(0, c["A"], c["Y"])
        oD = o.cp_gradient(0, c["Y"].size, c["A"], c["Y"], None, c["Eu"], c["Ev"], c["La_d1"],
                           c["La_l1"], st["active"], st["Cv"], st["Vc"], st["rVc"], st["rX"])
        _eq(DfS, oD, "DfS")
        cuts = (1, 2) if two_cuts else (0,)
        caps = {}
        for cut in cuts:
            if bounds:
                tr, rc = g.capacities_bounds(cut, c["lo"], c["hi"])
                otr, orc = o.cp_capacities_bounds(cut, c["La_d1"], c["lo"], c["hi"],
                                                  st["active"], st["Cv"], st["rX"], oD)
            else:
                tr, rc = g.capacities(cut, c["positivity"])
                otr, orc = o.cp_capacities(cut, c["La_d1"], c["La_l1"], c["positivity"],
                                           st["active"], st["Cv"], st["rX"], oD)
            _eq(tr, otr, "tr_cap cut %d" % cut)
            _eq(rc, orc, "r_cap cut %d" % cut)
            caps[cut] = (tr, rc)
        segs = ([d["k%d_seg_first" % k]] if two_cuts else []) + [d["k%d_seg_last" % k]]
        w = sum(g.activate(s) for s in segs)
        act = st["active"]
        ow = 0
        for s in segs:
            act, n = o.cp_activate(c["Eu"], c["Ev"], s, act)
            ow += n
        assert w == ow
        _eq(g.active(), act, "active before merge")
        if w == 0:
            continue
        Cv, Vc, rVc = g.components()
        _eq(Cv, new["Cv"], "Cv")
        _eq(Vc, new["Vc"], "Vc")
        _eq(rVc, new["rVc"], "rVc")
        rEu, rEv, rLa, rL1 = g.reduced_graph(eps)
        _eq(rEu, d["k%d_red_rEu" % k], "rEu")
        _eq(rEv, d["k%d_red_rEv" % k], "rEv")
        _eq(rLa, d["k%d_red_rLa_d1" % k], "rLa_d1")
        if rL1 is not None:
            _eq(rL1, d["k%d_red_rLa_l1" % k], "rLa_l1")
        g.set_values(new["rX"])
        g.merge(eps, c["CP_difTol"])
        _eq(g.active(), new["active"], "active after merge")
    g.close()


# ------------------------------------------------------- larger graphs --
def _graph(kind):
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, knn_jitter_grid
    if kind == "grid3d":
        Eu, Ev = grid_graph((40, 36, 30), 6)
        return 40 * 36 * 30, Eu, Ev
    if kind == "knn":
        Eu, Ev = knn_jitter_grid((30, 28, 24), k=6, seed=21)
        return 30 * 28 * 24, Eu, Ev
    if kind == "chain":
        V = 6000
        return V, np.arange(V - 1, dtype=np.int32), np.arange(1, V, dtype=np.int32)
    if kind == "grid2d8":
        Eu, Ev = grid_graph((300, 200), 8)
        return 300 * 200, Eu, Ev
    raise ValueError(kind)


def _activity(kind, V, Eu, Ev, seed):
    """cut-like activity: edges between random blobs, plus random extras"""
    rng = np.random.default_rng(seed)
    lab = (np.arange(V) // max(1, V // 37) * 7919 + rng.integers(0, 3, V) // 2) % 11
    act = (lab[Eu] != lab[Ev]).astype(np.uint8)
    act[rng.random(Eu.size) < 0.05] = 1
    if kind == "chain":
        act[:] = 0
        act[rng.choice(Eu.size, 5, replace=False)] = 1
    return act


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("kind", ["grid3d", "knn", "chain", "grid2d8"])
def test_gpu_graph_steps_match_oracle(cpgraph_cls, oracle_port, kind, dt):
    o = oracle_port
    V, Eu, Ev = _graph(kind)
    rng = np.random.default_rng(5)
    La = (0.01 + rng.random(Eu.size)).astype(dt)
    La[rng.random(Eu.size) < 0.02] = 0
    L1 = (0.02 * rng.random(V)).astype(dt)
    act = _activity(kind, V, Eu, Ev, 7)
    g = cpgraph_cls(V, Eu, Ev, La, L1)
    g.set_active(act)
    Cv, Vc, rVc = g.components()
    oCv, oVc, orVc = o.cp_components(V, Eu, Ev, act)
    _eq(Cv, oCv, "Cv")
    _eq(Vc, oVc, "Vc")
    _eq(rVc, orVc, "rVc")
    eps = float(np.finfo(dt).eps)
    red = g.reduced_graph(eps)
    ored = o.cp_reduced_graph(V, Eu, Ev, La, L1, act, oCv, oVc, orVc, eps)
    for a, b, nm in zip(red, ored, ("rEu", "rEv", "rLa_d1", "rLa_l1")):
        _eq(a, b, nm)
    rV = rVc.size - 1
    rX = np.round(rng.standard_normal(rV), 2).astype(dt)  # ties -> merges
    rX[rng.random(rV) < 0.2] = 0
    g.set_values(rX)
    Y = rng.standard_normal(V).astype(dt)
    A = (0.5 + rng.random(V)).astype(dt)
    for AA in (None, A):
        D = g.gradient(0, AA, Y)
        oD = o.cp_gradient(0, V, AA, Y, None, Eu, Ev, La, L1, act, oCv, oVc, orVc, rX)
        _eq(D, oD, "DfS")
        for cut, pos in ((0, 0), (1, 0), (2, 0), (2, 1)):
            tr, rc = g.capacities(cut, pos)
            otr, orc = o.cp_capacities(cut, La, L1, pos, act, oCv, rX, oD)
            _eq(tr, otr, "tr")
            _eq(rc, orc, "rc")
    seg = (rng.random(V) < 0.5).astype(np.uint8)
    n = g.activate(seg)
    oact, on = o.cp_activate(Eu, Ev, seg, act)
    assert n == on
    _eq(g.active(), oact, "activate")
    m = g.merge(eps, 1e-3)
    oact2, om = o.cp_merge(Eu, Ev, oCv, rX, eps, 1e-3, oact)
    assert m == om
    _eq(g.active(), oact2, "merge")
    g.close()


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_gpu_edgeless_and_all_active(cpgraph_cls, oracle_port, dt):
    o = oracle_port
    V = 1000
    Eu = np.zeros(0, np.int32)
    g = cpgraph_cls(V, Eu, Eu, np.zeros(0, dt))
    Cv, Vc, rVc = g.components()
    assert rVc.size == V + 1 and np.array_equal(Cv, np.arange(V))
    rEu, rEv, rLa, _ = g.reduced_graph(1e-7)
    oEu, oEv, oLa, _ = o.cp_reduced_graph(V, Eu, Eu, np.zeros(0, dt), None, np.zeros(0, np.uint8),
                                          Cv, Vc, rVc, 1e-7)
    _eq(rEu, oEu, "rEu")
    _eq(rEv, oEv, "rEv")
    _eq(rLa, oLa, "rLa")
    g.close()
    from cp_pfdr_graph_d1_amd.graphs import grid_graph
    Eu, Ev = grid_graph((50, 40), 4)
    La = np.full(Eu.size, 0.1, dt)
    act = np.ones(Eu.size, np.uint8)
    g = cpgraph_cls(2000, Eu, Ev, La)
    g.set_active(act)
    Cv, Vc, rVc = g.components()
    oCv, oVc, orVc = o.cp_components(2000, Eu, Ev, act)
    _eq(Vc, oVc, "Vc")
    red = g.reduced_graph(1e-7)
    ored = o.cp_reduced_graph(2000, Eu, Ev, La, None, act, oCv, oVc, orVc, 1e-7)
    for a, b, nm in zip(red[:3], ored[:3], ("rEu", "rEv", "rLa")):
        _eq(a, b, nm)
    g.close()


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_gpu_dense_gradients_match_oracle(cpgraph_cls, oracle_port, dt):
    o = oracle_port
    from cp_pfdr_graph_d1_amd.graphs import grid_graph
    rng = np.random.default_rng(9)
    Eu, Ev = grid_graph((20, 15), 4)
    V = 300
    La = np.full(Eu.size, 0.05, dt)
    act = _activity("grid2d8", V, Eu, Ev, 3)
    g = cpgraph_cls(V, Eu, Ev, La)
    g.set_active(act)
    Cv, Vc, rVc = g.components()
    rX = rng.standard_normal(rVc.size - 1).astype(dt)
    rX[::3] = 0
    g.set_values(rX)
    for N in (37, 200):  # direct: A N-by-V, R the residual
        A = rng.standard_normal((N, V)).astype(dt)
        R = rng.standard_normal(N).astype(dt)
        D = g.gradient(N, A, None, R)
        oD = o.cp_gradient(N, V, A, np.zeros(V, dt), R, Eu, Ev, La, None, act, Cv, Vc, rVc, rX)
        _eq(D, oD, "DfS N=%d" % N)
    B = rng.standard_normal((V, V)).astype(dt)
    AtA = (B + B.T).astype(dt)
    AtY = rng.standard_normal(V).astype(dt)
    D = g.gradient(-V, AtA, AtY)
    oD = o.cp_gradient(-V, V, AtA, AtY, None, Eu, Ev, La, None, act, Cv, Vc, rVc, rX)
    _eq(D, oD, "DfS N=-V")
    g.close()


# ------------------------------------------------- the simplex driver --
@pytest.mark.parametrize("name", SNAMES)
def test_gpu_replays_reference_simplex_cp(cpgraph_cls, oracle_port, name):
    """every recorded iteration of the reference's simplex cut pursuit:
    gradient, most confident labels and each alpha-expansion's capacities
    against the oracle, the expansions with the iteration's segments,
    activation, components, reduced graph, reduced observations (rQ, rLa_f,
    barycentre warm start) and merge against the reference: bit for bit"""
    c, d = load_case(name)
    o = oracle_port
    K, al, Q = c["K"], c["al"], c["Q"]
    dt = Q.dtype
    V = Q.size // K
    eps = CC.simplex_eps(dt.type, V, c["CP_difTol"], CC.SIMPLEX_PFDR_DIFTOL)
    g = cpgraph_cls(V, c["Eu"], c["Ev"], c["La_d1"])
    g.simplex_setup(K, al, Q)
    rP0, _, _ = g.simplex_observations()  # one component: initialize() (:96-108)
    _eq(rP0, d["k0_in_rP"], "initial rP")
    for k in range(int(d["meta_steps"])):
        st, new = iteration_state(d, k, "in"), iteration_state(d, k, "out")
        g.set_active(st["active"])
        g.set_components(st["Cv"], st["Vc"], st["rVc"])
        g.simplex_set_values(st["rP"])
        DfS, rDi = g.simplex_gradient(eps)
        oD, orDi = o.cp_simplex_gradient(K, al, Q, c["Eu"], c["Ev"], c["La_d1"], st["active"],
                                         st["Cv"], st["rP"], eps)
        _eq(DfS, oD, "DfS")
        _eq(rDi, orDi, "rDi")
        Djv = np.zeros(V, np.int32)
        for n, seg in enumerate(expansion_segments(d, K, k), 1):
            tr, rc = g.simplex_capacities(n)
            otr, orc = o.cp_simplex_capacities(K, n, c["Eu"], c["Ev"], c["La_d1"], st["active"],
                                               st["Vc"], st["rVc"], orDi, Djv, oD)
            _eq(tr, otr, "tr_cap expansion %d" % n)
            _eq(rc, orc, "r_cap expansion %d" % n)
            g.simplex_expand(n, seg)
            Djv = o.cp_simplex_expand(n, seg, Djv)
            _eq(g.simplex_labels(), Djv, "Djv after expansion %d" % n)
        w = g.simplex_activate()
        act, ow = o.cp_simplex_activate(c["Eu"], c["Ev"], Djv, st["active"])
        assert w == ow
        _eq(g.active(), act, "active before merge")
        if w == 0:
            assert ("k%d_red_rEu" % k) not in d.files
            continue
        Cv, Vc, rVc = g.components()
        _eq(Cv, new["Cv"], "Cv")
        _eq(Vc, new["Vc"], "Vc")
        _eq(rVc, new["rVc"], "rVc")
        rEu, rEv, rLa, _ = g.reduced_graph(eps)
        _eq(rEu, d["k%d_red_rEu" % k], "rEu")
        _eq(rEv, d["k%d_red_rEv" % k], "rEv")
        _eq(rLa, d["k%d_red_rLa_d1" % k], "rLa_d1")
        rP, rQ, rLa_f = g.simplex_observations()
        _eq(rP, d["k%d_red_rP0" % k], "rP0")
        _eq(rQ, d["k%d_red_rQ" % k], "rQ")
        if rLa_f is not None:
            _eq(rLa_f, d["k%d_red_rLa_f" % k], "rLa_f")
        g.simplex_set_values(new["rP"])
        g.simplex_merge(eps)
        _eq(g.active(), new["active"], "active after merge")
    g.close()


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("kind,K,al", [("grid3d", 4, 0.1), ("knn", 3, 1.0), ("chain", 5, 0.0),
                                       ("grid2d8", 6, 0.3)])
def test_gpu_simplex_steps_match_oracle(cpgraph_cls, oracle_port, kind, K, al, dt):
    """larger graphs, random label likelihoods, activity and label vectors
    (ties on purpose, zero-weight edges): every simplex step against the
    oracle, through all K - 1 expansions with random segments"""
    o = oracle_port
    V, Eu, Ev = _graph(kind)
    rng = np.random.default_rng(11 + K)
    La = (0.01 + rng.random(Eu.size)).astype(dt)
    La[rng.random(Eu.size) < 0.02] = 0
    Q = rng.random((V, K))
    Q = (Q / Q.sum(axis=1, keepdims=True)).reshape(-1).astype(dt)
    act = _activity(kind, V, Eu, Ev, 9)
    g = cpgraph_cls(V, Eu, Ev, La)
    g.simplex_setup(K, al, Q)
    g.set_active(act)
    Cv, Vc, rVc = g.components()
    rV = rVc.size - 1
    oP, oQ, oL = o.cp_simplex_reduced(K, al, Q, Vc, rVc)
    rP, rQ, rL = g.simplex_observations()
    _eq(rP, oP, "rP")
    _eq(rQ, oQ, "rQ")
    if oL is not None:
        _eq(rL, oL, "rLa_f")
    P = np.round(rng.random((rV, K)), 1)  # ties -> merges, equal labels
    P[rng.random(rV) < 0.3] = P[0]
    P = (P / np.maximum(P.sum(axis=1, keepdims=True), 1e-9)).reshape(-1).astype(dt)
    g.simplex_set_values(P)
    eps = float(np.finfo(dt).eps)
    D, rDi = g.simplex_gradient(eps)
    oD, orDi = o.cp_simplex_gradient(K, al, Q, Eu, Ev, La, act, Cv, P, eps)
    _eq(D, oD, "DfS")
    _eq(rDi, orDi, "rDi")
    Djv = np.zeros(V, np.int32)
    for n in range(1, K):
        tr, rc = g.simplex_capacities(n)
        otr, orc = o.cp_simplex_capacities(K, n, Eu, Ev, La, act, Vc, rVc, orDi, Djv, oD)
        _eq(tr, otr, "tr %d" % n)
        _eq(rc, orc, "rc %d" % n)
        seg = (rng.random(V) < 0.3).astype(np.uint8)
        g.simplex_expand(n, seg)
        Djv = o.cp_simplex_expand(n, seg, Djv)
    _eq(g.simplex_labels(), Djv, "Djv")
    w = g.simplex_activate()
    oact, ow = o.cp_simplex_activate(Eu, Ev, Djv, act)
    assert w == ow
    _eq(g.active(), oact, "activate")
    m = g.simplex_merge(eps)
    oact2, om = o.cp_simplex_merge(K, Eu, Ev, Cv, P, eps, oact)
    assert m == om
    _eq(g.active(), oact2, "merge")
    g.close()


# -------------------------------------------------- the duplex driver --
@pytest.mark.parametrize("name", DNAMES)
def test_gpu_replays_reference_duplex_cp(cpgraph_cls, oracle_port, name):
    """every recorded iteration of the reference's duplex cut pursuit: the
    gradient and the two-layer cut's capacities against the oracle, the
    activation with the recorded 2V segments, components, reduced graph and
    merge against the reference: bit for bit"""
    c, d = load_case(name)
    o = oracle_port
    dt = c["Y"].dtype
    V = c["Y"].size
    eps = CC.cp_eps(dt, c["CP_difTol"])
    g = cpgraph_cls(V, c["Eu"], c["Ev"], c["La_d1"], c["La_l1"])
    for k in range(int(d["meta_steps"])):
        st, new = iteration_state(d, k, "in"), iteration_state(d, k, "out")
        g.set_active(st["active"])
        g.set_components(st["Cv"], st["Vc"], st["rVc"])
        g.set_values(st["rX"])
        DfS = g.gradient(0, c["A"], c["Y"])
        oD = o.cp_gradient(0, V, c["A"], c["Y"], None, c["Eu"], c["Ev"], c["La_d1"], c["La_l1"],
                           st["active"], st["Cv"], st["Vc"], st["rVc"], st["rX"])
        _eq(DfS, oD, "DfS")
        tr, link, rc = g.capacities_duplex(c["positivity"])
        otr, olink, orc = o.cp_capacities_duplex(c["La_d1"], c["La_l1"], c["positivity"],
                                                 st["active"], st["Cv"], st["rX"], oD)
        _eq(tr, otr, "tr_cap")
        _eq(link, olink, "r_link")
        _eq(rc, orc, "r_cap")
        seg = d["k%d_seg_last" % k]
        w = g.activate_duplex(seg)
        act, ow = o.cp_activate_duplex(V, c["Eu"], c["Ev"], seg, st["active"])
        assert w == ow
        _eq(g.active(), act, "active before merge")
        if w == 0:
            continue
        Cv, Vc, rVc = g.components()
        _eq(Cv, new["Cv"], "Cv")
        _eq(Vc, new["Vc"], "Vc")
        _eq(rVc, new["rVc"], "rVc")
        rEu, rEv, rLa, rL1 = g.reduced_graph(eps)
        _eq(rEu, d["k%d_red_rEu" % k], "rEu")
        _eq(rEv, d["k%d_red_rEv" % k], "rEv")
        _eq(rLa, d["k%d_red_rLa_d1" % k], "rLa_d1")
        _eq(rL1, d["k%d_red_rLa_l1" % k], "rLa_l1")
        g.set_values(new["rX"])
        g.merge(eps, c["CP_difTol"])
        _eq(g.active(), new["active"], "active after merge")
    g.close()


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("kind", ["grid3d", "knn", "grid2d8"])
def test_gpu_duplex_cut_matches_oracle(cpgraph_cls, oracle_port, kind, dt):
    """the two-layer cut on larger graphs, zero components (l1, positivity)"""
    o = oracle_port
    V, Eu, Ev = _graph(kind)
    rng = np.random.default_rng(17)
    La = (0.01 + rng.random(Eu.size)).astype(dt)
    L1 = (0.05 * rng.random(V)).astype(dt)
    act = _activity(kind, V, Eu, Ev, 3)
    g = cpgraph_cls(V, Eu, Ev, La, L1)
    g.set_active(act)
    Cv, Vc, rVc = g.components()
    rV = rVc.size - 1
    rX = np.round(rng.standard_normal(rV), 1).astype(dt)
    rX[rng.random(rV) < 0.3] = 0
    g.set_values(rX)
    Y = rng.standard_normal(V).astype(dt)
    D = g.gradient(0, None, Y)
    for pos in (0, 1):
        tr, link, rc = g.capacities_duplex(pos)
        otr, olink, orc = o.cp_capacities_duplex(La, L1, pos, act, Cv, rX, D)
        _eq(tr, otr, "tr")
        _eq(link, olink, "link")
        _eq(rc, orc, "rc")
    seg = (rng.random(2 * V) < 0.5).astype(np.uint8)
    n = g.activate_duplex(seg)
    oact, on = o.cp_activate_duplex(V, Eu, Ev, seg, act)
    assert n == on
    _eq(g.active(), oact, "activate")
    g.close()
