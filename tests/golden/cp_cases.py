"""CP graph-step cases and the oracle's
statement of one cut-pursuit iteration around them.

Each case is a small N = 0 problem (identity or diagonal A) for the
reference's CP_PFDR_graph_quadratic_d1_l1; tests/golden/make_cp_golden.py
runs the REFERENCE CP iteration by iteration (warm restart, one iteration
per call) and stores every iteration's input state, the state it produced,
the last cut's segments and the reduced problem it handed to PFDR.

``cp_graph_iteration`` restates the graph part of one iteration with the
oracle (oracle/cp_graph_body.h) around a maxflow callable: gradient ->
capacities -> maxflow -> activation (one cut when the problem is
differentiable, two otherwise, src/CP_PFDR_graph_quadratic_d1_l1.cpp:402-560)
-> components (:566-597) -> reduced graph (:599-661); the PFDR values rX of
the iteration are then given, and the merge (:863-886) deactivates edges.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from cp_pfdr_graph_d1_amd.graphs import grid_graph, knn_jitter_grid, uniform  # noqa: E402

STEPS = 6  # CP iterations recorded per case


def _y(V, nx, seed, dt, noise=0.2):
    v = np.arange(V)
    base = np.where((v % nx) < nx // 2, 1.0, -0.5)
    base = base + np.where((v // nx) % 7 < 3, 0.6, 0.0)
    return (base + noise * (2 * uniform(seed, v) - 1)).astype(dt)


def make_cases():
    cases = {}
    for dt, nm in ((np.float32, "f32"), (np.float64, "f64")):
        eps = float(np.finfo(dt).eps)
        # differentiable: one cut per iteration
        Eu, Ev = grid_graph((24, 20), 4)
        V = 24 * 20
        cases["cp_grid2d_diff_" + nm] = dict(
            Y=_y(V, 24, 11, dt), A=None, Eu=Eu, Ev=Ev,
            La_d1=np.full(Eu.size, 0.05, dt), La_l1=None, positivity=0, CP_difTol=1e-3)
        # l1: two cuts, zero components
        cases["cp_grid2d_l1_" + nm] = dict(
            Y=_y(V, 24, 12, dt), A=None, Eu=Eu, Ev=Ev,
            La_d1=(0.03 + 0.04 * uniform(13, np.arange(Eu.size))).astype(dt),
            La_l1=np.full(V, 0.2, dt), positivity=0, CP_difTol=1e-3)
        # positivity: -inf sink capacities on zero components
        cases["cp_grid2d_pos_" + nm] = dict(
            Y=_y(V, 24, 14, dt), A=None, Eu=Eu, Ev=Ev,
            La_d1=np.full(Eu.size, 0.04, dt), La_l1=None, positivity=1, CP_difTol=1e-3)
        # k-NN multigraph (mirrored duplicates; BK forbids self-loops,
        # include/graph.hpp:391), diagonal A, l1 + positivity
        Ku, Kv = knn_jitter_grid((10, 8, 6), k=6, seed=15)
        Vk = 10 * 8 * 6
        cases["cp_knn_diag_l1pos_" + nm] = dict(
            Y=_y(Vk, 10, 16, dt), A=(0.5 + uniform(17, np.arange(Vk))).astype(dt), Eu=Ku,
            Ev=Kv, La_d1=np.full(Ku.size, 0.02, dt), La_l1=np.full(Vk, 0.05, dt),
            positivity=1, CP_difTol=1e-4)
        # disconnected graph: an isolated vertex (vertex 0), two grids,
        # zero-weight edges — isolated components and their eps self-loops,
        # including the reference's re-attribution of an isolated
        # component's self-loop to the next non-isolated one (:642-656)
        Au, Av = grid_graph((12, 10), 8)
        Bu, Bv = grid_graph((9, 7), 4)
        Vd = 1 + 120 + 63
        Du = np.concatenate([Au + 1, Bu + 121]).astype(np.int32)
        Dv = np.concatenate([Av + 1, Bv + 121]).astype(np.int32)
        La = np.full(Du.size, 0.05, dt)
        La[::17] = 0
        Yd = _y(Vd, 12, 18, dt)
        Yd[0] = 3.0
        Yd[121:] += 0.3
        cases["cp_disconnected_" + nm] = dict(
            Y=Yd, A=None, Eu=Du, Ev=Dv, La_d1=La, La_l1=None, positivity=0,
            CP_difTol=1e-3)
        for c in cases.values():
            c.setdefault("eps", eps)
    return cases


def make_bounds_cases():
    """cases of the bounds driver (src/CP_PFDR_graph_quadratic_d1_bounds.cpp):
    a box both of whose ends bind, one-sided boxes, no bound (one cut), a
    k-NN multigraph with a diagonal A"""
    inf = float("inf")
    cases = {}
    for dt, nm in ((np.float32, "f32"), (np.float64, "f64")):
        eps = float(np.finfo(dt).eps)
        Eu, Ev = grid_graph((24, 20), 4)
        V = 24 * 20
        for tag, lo, hi in (("box", 0.0, 1.0), ("lower", 0.0, inf), ("upper", -inf, 0.8),
                            ("free", -inf, inf)):
            cases["cp_bounds_%s_%s" % (tag, nm)] = dict(
                Y=_y(V, 24, 21, dt, noise=0.3), A=None, Eu=Eu, Ev=Ev,
                La_d1=np.full(Eu.size, 0.05, dt), lo=lo, hi=hi, CP_difTol=1e-3)
        Ku, Kv = knn_jitter_grid((10, 8, 6), k=6, seed=22)
        Vk = 10 * 8 * 6
        cases["cp_bounds_knn_diag_" + nm] = dict(
            Y=_y(Vk, 10, 23, dt), A=(0.5 + uniform(24, np.arange(Vk))).astype(dt), Eu=Ku,
            Ev=Kv, La_d1=np.full(Ku.size, 0.02, dt), lo=-0.2, hi=1.1, CP_difTol=1e-4)
        for c in cases.values():
            c.setdefault("eps", eps)
    return cases


def cp_graph_iteration_bounds(o, maxflow, case, state, rX_new=None):
    """cp_graph_iteration for the bounds driver: gradient (no l1 term) ->
    one cut (no bound) or two (+1_U then -1_U, :386-534) -> components ->
    reduced graph (no rLa_l1) -> merge"""
    c = case
    V = c["Y"].size
    dt = c["Y"].dtype
    act0 = np.asarray(state["active"], np.uint8)
    DfS = o.cp_gradient(0, V, c["A"], c["Y"], None, c["Eu"], c["Ev"], c["La_d1"], None,
                        act0, state["Cv"], state["Vc"], state["rVc"], state["rX"])
    out = {"DfS": DfS}
    lo, hi = c["lo"], c["hi"]
    if lo == -np.inf and hi == np.inf:
        tr, rc = o.cp_capacities_bounds(0, c["La_d1"], lo, hi, act0, state["Cv"], state["rX"],
                                        DfS)
        seg = maxflow(tr, rc)
        act, w = o.cp_activate(c["Eu"], c["Ev"], seg, act0)
        out["caps"] = [(tr, rc)]
        out["segments"] = [seg]
    else:
        tr1, rc1 = o.cp_capacities_bounds(1, c["La_d1"], lo, hi, act0, state["Cv"],
                                          state["rX"], DfS)
        seg1 = maxflow(tr1, rc1)
        tr2, rc2 = o.cp_capacities_bounds(2, c["La_d1"], lo, hi, act0, state["Cv"],
                                          state["rX"], DfS)
        act, w1 = o.cp_activate(c["Eu"], c["Ev"], seg1, act0)
        seg2 = maxflow(tr2, rc2)
        act, w2 = o.cp_activate(c["Eu"], c["Ev"], seg2, act)
        w = w1 + w2
        out["caps"] = [(tr1, rc1), (tr2, rc2)]
        out["segments"] = [seg1, seg2]
    out["activated"] = w
    out["active_pre"] = act
    if w == 0:
        return out
    Cv, Vc, rVc = o.cp_components(V, c["Eu"], c["Ev"], act)
    out.update(Cv=Cv, Vc=Vc, rVc=rVc)
    out["reduced"] = o.cp_reduced_graph(V, c["Eu"], c["Ev"], c["La_d1"], None, act, Cv, Vc,
                                        rVc, cp_eps(dt, c["CP_difTol"]))
    if rX_new is not None:
        out["active_post"], out["merged"] = o.cp_merge(
            c["Eu"], c["Ev"], Cv, np.asarray(rX_new, dt), cp_eps(dt, c["CP_difTol"]),
            c["CP_difTol"], act)
    return out


def cp_eps(dt, CP_difTol):
    """:236-251: eps = CP_difTol if 0 < CP_difTol < machine eps, else it"""
    m = float(np.finfo(dt).eps)
    return CP_difTol if 0 < CP_difTol < m else m


def cp_graph_iteration(o, maxflow, case, state, rX_new=None):
    """One CP iteration's graph steps with the oracle ``o`` around
    ``maxflow(tr_cap, r_cap) -> segments``; returns a dict with DfS, the
    segments of each cut, activation count, pre-merge activity, components,
    reduced graph and (when rX_new is given) post-merge activity."""
    c = case
    V = c["Y"].size
    dt = c["Y"].dtype
    act0 = np.asarray(state["active"], np.uint8)
    DfS = o.cp_gradient(0, V, c["A"], c["Y"], None, c["Eu"], c["Ev"], c["La_d1"], c["La_l1"],
                        act0, state["Cv"], state["Vc"], state["rVc"], state["rX"])
    out = {"DfS": DfS}
    if c["La_l1"] is None and not c["positivity"]:
        tr, rc = o.cp_capacities(0, c["La_d1"], None, 0, act0, state["Cv"], state["rX"], DfS)
        seg = maxflow(tr, rc)
        act, w = o.cp_activate(c["Eu"], c["Ev"], seg, act0)
        out["caps"] = [(tr, rc)]
        out["segments"] = [seg]
    else:
        tr1, rc1 = o.cp_capacities(1, c["La_d1"], c["La_l1"], c["positivity"], act0,
                                   state["Cv"], state["rX"], DfS)
        seg1 = maxflow(tr1, rc1)
        tr2, rc2 = o.cp_capacities(2, c["La_d1"], c["La_l1"], c["positivity"], act0,
                                   state["Cv"], state["rX"], DfS)
        act, w1 = o.cp_activate(c["Eu"], c["Ev"], seg1, act0)
        seg2 = maxflow(tr2, rc2)
        act, w2 = o.cp_activate(c["Eu"], c["Ev"], seg2, act)
        w = w1 + w2
        out["caps"] = [(tr1, rc1), (tr2, rc2)]
        out["segments"] = [seg1, seg2]
    out["activated"] = w
    out["active_pre"] = act
    if w == 0:
        return out
    Cv, Vc, rVc = o.cp_components(V, c["Eu"], c["Ev"], act)
    out.update(Cv=Cv, Vc=Vc, rVc=rVc)
    out["reduced"] = o.cp_reduced_graph(V, c["Eu"], c["Ev"], c["La_d1"], c["La_l1"], act, Cv,
                                        Vc, rVc, cp_eps(dt, c["CP_difTol"]))
    if rX_new is not None:
        out["active_post"], out["merged"] = o.cp_merge(
            c["Eu"], c["Ev"], Cv, np.asarray(rX_new, dt), cp_eps(dt, c["CP_difTol"]),
            c["CP_difTol"], act)
    return out


# ------------------------------------------------ the simplex driver --
def _q(V, K, nx, seed, dt, noise=0.35):
    """label likelihoods in the simplex: a spatial label map (stripes and
    blocks) blurred with uniform noise, normalised per vertex"""
    v = np.arange(V)
    lab = ((v % nx) * K // nx + (v // nx) // 5) % K
    Q = np.full((V, K), 0.0)
    Q[v, lab] = 1.0
    Q = (1 - noise) * Q + noise * uniform(seed, np.arange(V * K)).reshape(V, K)
    Q /= Q.sum(axis=1, keepdims=True)
    return Q.reshape(-1).astype(dt)


def make_simplex_cases():
    """cases of the simplex driver (src/CP_PFDR_graph_loss_d1_simplex.cpp):
    linear (al = 0), quadratic (al = 1) and smoothed-KL losses, 2-D grids, a
    k-NN multigraph, a disconnected graph with zero-weight edges"""
    cases = {}
    for dt, nm in ((np.float32, "f32"), (np.float64, "f64")):
        Eu, Ev = grid_graph((24, 20), 4)
        V = 24 * 20
        cases["cp_simplex_linear_" + nm] = dict(
            K=3, al=0.0, Q=_q(V, 3, 24, 31, dt), Eu=Eu, Ev=Ev,
            La_d1=np.full(Eu.size, 0.08, dt), CP_difTol=1e-3)
        cases["cp_simplex_quad_" + nm] = dict(
            K=4, al=1.0, Q=_q(V, 4, 24, 32, dt), Eu=Eu, Ev=Ev,
            La_d1=(0.02 + 0.03 * uniform(33, np.arange(Eu.size))).astype(dt), CP_difTol=1e-3)
        cases["cp_simplex_kl_" + nm] = dict(
            K=3, al=0.1, Q=_q(V, 3, 24, 34, dt), Eu=Eu, Ev=Ev,
            La_d1=np.full(Eu.size, 0.05, dt), CP_difTol=1e-3)
        Ku, Kv = knn_jitter_grid((10, 8, 6), k=6, seed=35)
        Vk = 10 * 8 * 6
        cases["cp_simplex_knn_kl_" + nm] = dict(
            K=5, al=0.05, Q=_q(Vk, 5, 10, 36, dt), Eu=Ku, Ev=Kv,
            La_d1=np.full(Ku.size, 0.03, dt), CP_difTol=1e-4)
        Au, Av = grid_graph((12, 10), 8)
        Bu, Bv = grid_graph((9, 7), 4)
        Vd = 1 + 120 + 63
        Du = np.concatenate([Au + 1, Bu + 121]).astype(np.int32)
        Dv = np.concatenate([Av + 1, Bv + 121]).astype(np.int32)
        La = np.full(Du.size, 0.06, dt)
        La[::13] = 0
        cases["cp_simplex_disconnected_" + nm] = dict(
            K=3, al=1.0, Q=_q(Vd, 3, 12, 37, dt), Eu=Du, Ev=Dv, La_d1=La, CP_difTol=1e-3)
    return cases


def simplex_eps(dt, V, CP_difTol, PFDR_difTol):
    """:214-231, as compiled: ``(ZERO < c < a)`` is ``((0 < c) < a)``, so eps
    is the machine epsilon a unless c = min(b, c) <= 0 (b, c: CP / PFDR
    tolerances, divided by V when >= 1)"""
    a = float(np.finfo(dt).eps)
    b = dt(CP_difTol) / dt(V) if CP_difTol >= 1 else dt(CP_difTol)
    c = dt(PFDR_difTol) / dt(V) if PFDR_difTol >= 1 else dt(PFDR_difTol)
    c = b if b < c else c
    return float(c) if not (c > 0) else a


SIMPLEX_PFDR_DIFTOL = 1e-3  # the step harness's PFDR difTol (oracle.CPStepRefSimplex.step)


def cp_graph_iteration_simplex(o, maxflow, case, state, rP_new=None):
    """One iteration of the simplex driver's graph steps with the oracle
    around ``maxflow(tr_cap, r_cap) -> segments``: gradient and most
    confident labels (:327-376, :525-536) -> K - 1 alpha-expansions
    (capacities :542-595, maxflow, :600-604) -> activation (:608-618) ->
    components -> reduced graph (:684-729) -> reduced observations
    (:733-766) -> (given the PFDR values rP_new) merge (:782-803)."""
    c = case
    K, al = int(c["K"]), float(c["al"])
    Q = c["Q"]
    dt = Q.dtype
    V = Q.size // K
    eps = simplex_eps(dt.type, V, c["CP_difTol"], SIMPLEX_PFDR_DIFTOL)
    act0 = np.asarray(state["active"], np.uint8)
    DfS, rDi = o.cp_simplex_gradient(K, al, Q, c["Eu"], c["Ev"], c["La_d1"], act0, state["Cv"],
                                     state["rP"], eps)
    out = {"DfS": DfS, "rDi": rDi, "caps": [], "segments": []}
    Djv = np.zeros(V, np.int32)
    for n in range(1, K):
        tr, rc = o.cp_simplex_capacities(K, n, c["Eu"], c["Ev"], c["La_d1"], act0, state["Vc"],
                                         state["rVc"], rDi, Djv, DfS)
        seg = maxflow(tr, rc)
        Djv = o.cp_simplex_expand(n, seg, Djv)
        out["caps"].append((tr, rc))
        out["segments"].append(seg)
    out["Djv"] = Djv
    act, w = o.cp_simplex_activate(c["Eu"], c["Ev"], Djv, act0)
    out["activated"] = w
    out["active_pre"] = act
    if w == 0:
        return out
    Cv, Vc, rVc = o.cp_components(V, c["Eu"], c["Ev"], act)
    out.update(Cv=Cv, Vc=Vc, rVc=rVc)
    out["reduced"] = o.cp_reduced_graph(V, c["Eu"], c["Ev"], c["La_d1"], None, act, Cv, Vc, rVc,
                                        eps)
    out["observations"] = o.cp_simplex_reduced(K, al, Q, Vc, rVc)
    if rP_new is not None:
        out["active_post"], out["merged"] = o.cp_simplex_merge(K, c["Eu"], c["Ev"], Cv,
                                                               np.asarray(rP_new, dt), eps, act)
    return out


# ------------------------------------------------- the duplex driver --
def make_duplex_cases():
    """cases of the duplex driver (src/CP_PFDR_graph_quadratic_d1_l1_duplex.cpp)
    in its non-differentiable case (La_l1 or positivity: the two-layer
    graph): the l1 cases with an l1 term or positivity, renamed"""
    out = {}
    for name, c in make_cases().items():
        # differentiable (no La_l1, no positivity): the l1 driver's one-layer
        # graph, indexed as if it had four arcs per edge (La_d1[e / 2],
        # :407, :628) -- not reproduced; positivity without
        # La_l1: the reference reads its up / down directions of the
        # nonzero components from uninitialised memory (:470-502)
        if c["La_l1"] is None:
            continue
        out[name.replace("cp_", "cp_duplex_", 1)] = dict(c)
    # positivity together with an l1 term; the disconnected graph with an l1
    # term (isolated components' eps self-loops)
    for dt, nm in ((np.float32, "f32"), (np.float64, "f64")):
        d = dict(make_cases()["cp_disconnected_" + nm])
        d["La_l1"] = np.full(d["Y"].size, 0.15, dt)
        out["cp_duplex_disconnected_l1_" + nm] = d
        Eu, Ev = grid_graph((24, 20), 4)
        V = 24 * 20
        out["cp_duplex_grid2d_l1pos_" + nm] = dict(
            Y=_y(V, 24, 19, dt), A=None, Eu=Eu, Ev=Ev,
            La_d1=np.full(Eu.size, 0.03, dt), La_l1=np.full(V, 0.1, dt), positivity=1,
            CP_difTol=1e-3, eps=float(np.finfo(dt).eps))
    return out


def cp_graph_iteration_duplex(o, maxflow, case, state, rX_new=None):
    """One iteration of the duplex driver's graph steps with the oracle: the
    l1 driver's gradient -> the two-layer cut's capacities (:469-527) ->
    ``maxflow(tr_cap[2V], r_link[V], r_cap[E]) -> segments[2V]`` ->
    activation in either layer (:531-545) -> components -> reduced graph ->
    merge (the l1 driver's, :599-661 / :863-886 as in the duplex source)"""
    c = case
    V = c["Y"].size
    dt = c["Y"].dtype
    act0 = np.asarray(state["active"], np.uint8)
    DfS = o.cp_gradient(0, V, c["A"], c["Y"], None, c["Eu"], c["Ev"], c["La_d1"], c["La_l1"],
                        act0, state["Cv"], state["Vc"], state["rVc"], state["rX"])
    tr, link, rc = o.cp_capacities_duplex(c["La_d1"], c["La_l1"], c["positivity"], act0,
                                          state["Cv"], state["rX"], DfS)
    seg = maxflow(tr, link, rc)
    act, w = o.cp_activate_duplex(V, c["Eu"], c["Ev"], seg, act0)
    out = {"DfS": DfS, "caps": [(tr, link, rc)], "segments": [seg], "activated": w,
           "active_pre": act}
    if w == 0:
        return out
    Cv, Vc, rVc = o.cp_components(V, c["Eu"], c["Ev"], act)
    out.update(Cv=Cv, Vc=Vc, rVc=rVc)
    eps = cp_eps(dt, c["CP_difTol"])
    out["reduced"] = o.cp_reduced_graph(V, c["Eu"], c["Ev"], c["La_d1"], c["La_l1"], act, Cv,
                                        Vc, rVc, eps)
    if rX_new is not None:
        out["active_post"], out["merged"] = o.cp_merge(
            c["Eu"], c["Ev"], Cv, np.asarray(rX_new, dt), eps, c["CP_difTol"], act)
    return out
