"""The oracle's CP graph steps (oracle/cp_graph_body.h, SURVEY.md §8(f)
ranks 2-3) against the reference's own cut-pursuit iterations
(tests/golden/cp_*.npz, made by tests/golden/make_cp_golden.py): the l1
driver's and (cp_bounds_*) the bounds driver's, whose cuts use the box
instead of the l1 term (src/CP_PFDR_graph_quadratic_d1_bounds.cpp:386-534).

Per recorded iteration: gradient -> capacities -> (the iteration's
segments, from the fixture) -> activation -> components -> reduced graph
-> merge with the iteration's PFDR values must reproduce the reference's
state and reduced problem bit for bit; the reduced problem's rY / rAA
(N = 0) must equal the CP builder restatement (cp_reduce_body.h).  Where
the reference harness is built (this container), the oracle's capacities
are also fed to the reference's BK maxflow, which must return the recorded
segments.  CPU only.
"""
import glob
import os

import numpy as np
import pytest

import cp_cases as CC
from oracle import CPStepRef, CPStepRefDuplex, CPStepRefSimplex

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FILES = sorted(glob.glob(os.path.join(GOLDEN, "cp_*.npz")))
_ALL = [os.path.basename(f)[:-4] for f in FILES]
# the l1 driver's iterations; the bounds driver's (cp_bounds_*); the dense
# reduced problems are test_cp_reduce.py's (cp_dense_*)
NAMES = [n for n in _ALL
         if not n.startswith(("cp_bounds_", "cp_dense_", "cp_simplex_", "cp_duplex_"))]
BNAMES = [n for n in _ALL if n.startswith("cp_bounds_")]
# the simplex driver's (src/CP_PFDR_graph_loss_d1_simplex.cpp): K - 1
# alpha-expansions per iteration, label vectors rP
SNAMES = [n for n in _ALL if n.startswith("cp_simplex_")]
# the duplex driver's (src/CP_PFDR_graph_quadratic_d1_l1_duplex.cpp): one
# two-layer cut per iteration, 2V segments
DNAMES = [n for n in _ALL if n.startswith("cp_duplex_")]


def load_case(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    c = {k[3:]: d[k] for k in d.files if k.startswith("in_")}
    for k in ("A", "La_l1"):
        c.setdefault(k, None)
    c["positivity"] = int(c.get("positivity", 0))
    for k in ("K",):
        if k in c:
            c[k] = int(c[k])
    if "al" in c:
        c["al"] = float(c["al"])
    c["CP_difTol"] = float(c["CP_difTol"])
    for k in ("lo", "hi"):
        if k in c:
            c[k] = float(c[k])
    return c, d


def iteration_state(d, k, io):
    vals = "rP" if ("k%d_%s_rP" % (k, io)) in d.files else "rX"
    return {key: d["k%d_%s_%s" % (k, io, key)] for key in ("active", "Cv", "Vc", "rVc", vals)}


def expansion_segments(d, K, k):
    """the segments of the K - 1 alpha-expansions of recorded iteration k"""
    return [d["k%d_seg_exp%d" % (k, n)] for n in range(1, K - 1)] + [d["k%d_seg_last" % k]]


def test_fixtures_present():
    assert len(NAMES) >= 10, NAMES
    assert len(BNAMES) >= 10, BNAMES
    assert len(SNAMES) >= 10, SNAMES
    assert len(DNAMES) >= 8, DNAMES


@pytest.mark.parametrize("name", NAMES + BNAMES)
def test_oracle_replays_reference_cp(oracle_port, name):
    c, d = load_case(name)
    o = oracle_port
    step = CC.cp_graph_iteration_bounds if name in BNAMES else CC.cp_graph_iteration
    for k in range(int(d["meta_steps"])):
        st, new = iteration_state(d, k, "in"), iteration_state(d, k, "out")
        segs = [d["k%d_seg_first" % k]] if ("k%d_seg_first" % k) in d.files else []
        segs.append(d["k%d_seg_last" % k])
        it = iter(segs)
        r = step(o, lambda tr, rc: next(it), c, st, rX_new=new["rX"])
        if r["activated"] == 0:
            assert ("k%d_red_rEu" % k) not in d.files
            continue
        assert np.array_equal(r["Cv"], new["Cv"])
        assert np.array_equal(r["Vc"], new["Vc"])
        assert np.array_equal(r["rVc"], new["rVc"])
        rEu, rEv, rLa, rL1 = r["reduced"]
        assert np.array_equal(rEu, d["k%d_red_rEu" % k])
        assert np.array_equal(rEv, d["k%d_red_rEv" % k])
        assert np.array_equal(rLa, d["k%d_red_rLa_d1" % k])
        if rL1 is not None:
            assert np.array_equal(rL1, d["k%d_red_rLa_l1" % k])
        assert np.array_equal(r["active_post"], new["active"])
        # the reduced problem's rY / rAA: the CP builder restatement (N = 0)
        red = o.cp_reduce(0, c["A"], c["Y"], new["rVc"], new["Vc"])
        assert np.array_equal(red["rY"], d["k%d_red_rY" % k])
        assert np.array_equal(red["rAA"], d["k%d_red_rAA" % k])


@pytest.mark.skipif(not CPStepRef.available(), reason="reference harness not built here")
@pytest.mark.parametrize("name", NAMES + BNAMES)
def test_oracle_capacities_through_reference_maxflow(oracle_port, name):
    c, d = load_case(name)
    ref = CPStepRef()
    step = CC.cp_graph_iteration_bounds if name in BNAMES else CC.cp_graph_iteration
    for k in range(int(d["meta_steps"])):
        st = iteration_state(d, k, "in")
        r = step(oracle_port, lambda tr, rc: ref.maxflow(c["Eu"], c["Ev"], tr, rc), c, st)
        assert np.array_equal(r["segments"][-1], d["k%d_seg_last" % k])
        if ("k%d_seg_first" % k) in d.files:
            assert np.array_equal(r["segments"][0], d["k%d_seg_first" % k])


def test_isolated_selfloop_reattribution_is_pinned():
    """The reference gives an isolated component's eps self-loop to the next
    non-isolated component (rEc reset, :645-656): the disconnected case
    holds such an edge (1, 0) at every iteration."""
    for nm in ("f32", "f64"):
        _, d = load_case("cp_disconnected_" + nm)
        k = 0
        u, v, w = d["k%d_red_rEu" % k], d["k%d_red_rEv" % k], d["k%d_red_rLa_d1" % k]
        tiny = w < 1e-6
        assert list(zip(u[tiny].tolist(), v[tiny].tolist())) == [(1, 0)]


@pytest.mark.parametrize("name", SNAMES)
def test_oracle_replays_reference_simplex_cp(oracle_port, name):
    """the simplex driver: gradient -> K - 1 expansions with the recorded
    segments -> activation -> components -> reduced graph -> reduced
    observations (rQ, rLa_f and the barycentre warm start rP0 CP handed to
    PFDR) -> merge with the iteration's PFDR values"""
    c, d = load_case(name)
    o = oracle_port
    K = c["K"]
    st0 = iteration_state(d, 0, "in")
    rP0, _, _ = o.cp_simplex_reduced(K, c["al"], c["Q"], st0["Vc"], st0["rVc"])
    assert np.array_equal(rP0, st0["rP"])  # initialize() (:96-108)
    for k in range(int(d["meta_steps"])):
        st, new = iteration_state(d, k, "in"), iteration_state(d, k, "out")
        it = iter(expansion_segments(d, K, k))
        r = CC.cp_graph_iteration_simplex(o, lambda tr, rc: next(it), c, st, rP_new=new["rP"])
        if r["activated"] == 0:
            assert ("k%d_red_rEu" % k) not in d.files
            assert np.array_equal(st["active"], new["active"])
            continue
        for key in ("Cv", "Vc", "rVc"):
            assert np.array_equal(r[key], new[key]), key
        rEu, rEv, rLa, _ = r["reduced"]
        assert np.array_equal(rEu, d["k%d_red_rEu" % k])
        assert np.array_equal(rEv, d["k%d_red_rEv" % k])
        assert np.array_equal(rLa, d["k%d_red_rLa_d1" % k])
        rP, rQ, rLa_f = r["observations"]
        assert np.array_equal(rP, d["k%d_red_rP0" % k])
        assert np.array_equal(rQ, d["k%d_red_rQ" % k])
        if rLa_f is not None:
            assert np.array_equal(rLa_f, d["k%d_red_rLa_f" % k])
        assert np.array_equal(r["active_post"], new["active"])


@pytest.mark.skipif(not CPStepRefSimplex.available(), reason="reference harness not built here")
@pytest.mark.parametrize("name", SNAMES)
def test_oracle_simplex_capacities_through_reference_maxflow(oracle_port, name):
    c, d = load_case(name)
    ref = CPStepRefSimplex()
    K = c["K"]
    for k in range(int(d["meta_steps"])):
        st = iteration_state(d, k, "in")
        r = CC.cp_graph_iteration_simplex(
            oracle_port, lambda tr, rc: ref.maxflow(c["Eu"], c["Ev"], tr, rc), c, st)
        for n, (a, b) in enumerate(zip(r["segments"], expansion_segments(d, K, k)), 1):
            assert np.array_equal(a, b), (k, n)


@pytest.mark.parametrize("name", DNAMES)
def test_oracle_replays_reference_duplex_cp(oracle_port, name):
    """the duplex driver: gradient -> two-layer capacities -> (the recorded
    2V segments) -> activation in either layer -> components -> reduced
    graph -> merge; rY / rAA through the CP builder restatement"""
    c, d = load_case(name)
    o = oracle_port
    for k in range(int(d["meta_steps"])):
        st, new = iteration_state(d, k, "in"), iteration_state(d, k, "out")
        seg = d["k%d_seg_last" % k]
        r = CC.cp_graph_iteration_duplex(o, lambda tr, link, rc: seg, c, st, rX_new=new["rX"])
        if r["activated"] == 0:
            assert ("k%d_red_rEu" % k) not in d.files
            continue
        for key in ("Cv", "Vc", "rVc"):
            assert np.array_equal(r[key], new[key]), key
        rEu, rEv, rLa, rL1 = r["reduced"]
        assert np.array_equal(rEu, d["k%d_red_rEu" % k])
        assert np.array_equal(rEv, d["k%d_red_rEv" % k])
        assert np.array_equal(rLa, d["k%d_red_rLa_d1" % k])
        assert np.array_equal(rL1, d["k%d_red_rLa_l1" % k])
        assert np.array_equal(r["active_post"], new["active"])
        red = o.cp_reduce(0, c["A"], c["Y"], new["rVc"], new["Vc"])
        assert np.array_equal(red["rY"], d["k%d_red_rY" % k])
        assert np.array_equal(red["rAA"], d["k%d_red_rAA" % k])


@pytest.mark.skipif(not CPStepRefDuplex.available(), reason="reference harness not built here")
@pytest.mark.parametrize("name", DNAMES)
def test_oracle_duplex_capacities_through_reference_maxflow(oracle_port, name):
    c, d = load_case(name)
    ref = CPStepRefDuplex()
    V = c["Y"].size
    for k in range(int(d["meta_steps"])):
        st = iteration_state(d, k, "in")
        r = CC.cp_graph_iteration_duplex(
            oracle_port, lambda tr, link, rc: ref.maxflow(V, c["Eu"], c["Ev"], tr, link, rc), c,
            st)
        assert np.array_equal(r["segments"][0], d["k%d_seg_last" % k])
