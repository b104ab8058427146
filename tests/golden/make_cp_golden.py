"""Generate the CP graph-step golden fixtures from the REFERENCE itself.

For every case of cp_cases.py, run the reference's cut pursuit
(oracle/_ref/libcp_step_ref.so: its CP_PFDR_graph_quadratic_d1_l1, graph
and BK maxflow compiled from /root/reference/src without OpenMP) one
iteration at a time from its own initial state, and store per iteration k:

* ``k{k}_in_*``  : the state the iteration starts from (edge activity, Cv,
                   Vc, rVc, rX);
* ``k{k}_out_*`` : the state it produced (activity after the merge, Cv, Vc,
                   rVc, rX) and ``k{k}_seg_last``, the segments of its last
                   maxflow;
* ``k{k}_red_*`` : the reduced problem CP handed to PFDR (rEu, rEv, rLa_d1,
                   rLa_l1, rY, rAA);
* ``k{k}_seg_first`` (two-cut iterations): the first cut's segments,
                   DERIVED here (oracle capacities -> the reference's own BK
                   maxflow) — the reference discards them — and accepted only
                   because the whole derived chain reproduces the
                   reference's outputs of that iteration bit for bit.

Before saving, the script checks the oracle restatement
(oracle/cp_graph_body.h) against every iteration: its capacities fed to the
reference maxflow give the reference's last segments, and its activation,
components, reduced graph and merge give the reference's state and reduced
problem exactly.  Usage:  python tests/golden/make_cp_golden.py [--bounds]
(--bounds: the cases of the bounds driver, CP_PFDR_graph_quadratic_d1_bounds,
 through oracle/_ref/libcp_step_bounds_ref.so; files cp_bounds_*.npz;
 --simplex: the simplex driver, CP_PFDR_graph_loss_d1_simplex, through
 oracle/_ref/libcp_step_simplex_ref.so; files cp_simplex_*.npz;
 --duplex: the duplex driver's two-layer cut, CP_PFDR_graph_quadratic_d1_l1_duplex,
 through oracle/_ref/libcp_step_duplex_ref.so; files cp_duplex_*.npz)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, HERE)
from oracle import CPStepRef, CPStepRefBounds, CPStepRefDuplex, CPStepRefSimplex, Oracle  # noqa: E402
import cp_cases as CC  # noqa: E402


def check_iteration(o, ref, c, state, new, seg_last, red, iteration=CC.cp_graph_iteration):
    """The oracle chain against one reference iteration; returns derived
    first-cut segments (or None)."""
    d = iteration(o, lambda tr, rc: ref.maxflow(c["Eu"], c["Ev"], tr, rc), c, state,
                  rX_new=new["rX"])
    assert np.array_equal(d["segments"][-1], seg_last), "last cut segments"
    if d["activated"] == 0:
        assert red is None
        for k in ("active", "Cv", "Vc", "rVc", "rX"):
            assert np.array_equal(state[k], new[k]), k
        return None
    assert red is not None
    assert np.array_equal(d["Cv"], new["Cv"]), "Cv"
    assert np.array_equal(d["Vc"], new["Vc"]), "Vc"
    assert np.array_equal(d["rVc"], new["rVc"]), "rVc"
    rEu, rEv, rLa, rL1 = d["reduced"]
    assert np.array_equal(rEu, red["rEu"]), "rEu"
    assert np.array_equal(rEv, red["rEv"]), "rEv"
    assert np.array_equal(rLa, red["rLa_d1"]), "rLa_d1"
    if rL1 is not None:
        assert np.array_equal(rL1, red["rLa_l1"]), "rLa_l1"
    assert np.array_equal(d["active_post"], new["active"]), "active after merge"
    return d["segments"][0] if len(d["segments"]) == 2 else None


def main_bounds():
    """the bounds driver (src/CP_PFDR_graph_quadratic_d1_bounds.cpp), same
    records; maxflow of the derived first cut through the l1 library's BK
    (same vendored graph code)"""
    o = Oracle("port")
    refb = CPStepRefBounds()
    mf = CPStepRef()
    for name, c in CC.make_bounds_cases().items():
        out = {}
        for k, v in c.items():
            if v is not None:
                out["in_" + k] = np.asarray(v)
        V, E = c["Y"].size, c["Eu"].size
        rX0 = refb.init(c["Y"], c["A"], c["Eu"], c["Ev"], c["La_d1"], c["lo"], c["hi"])
        state = {"active": np.zeros(E, np.uint8), "Cv": np.zeros(V, np.int32),
                 "Vc": np.arange(V, dtype=np.int32), "rVc": np.array([0, V], np.int32),
                 "rX": rX0}
        hist = []
        for k in range(CC.STEPS):
            new, seg, red = refb.step(c["Y"], c["A"], c["Eu"], c["Ev"], c["La_d1"], c["lo"],
                                      c["hi"], c["CP_difTol"], state)
            seg_first = check_iteration(o, mf, c, state, new, seg, red,
                                        CC.cp_graph_iteration_bounds)
            for key, val in state.items():
                out["k%d_in_%s" % (k, key)] = val
            for key, val in new.items():
                out["k%d_out_%s" % (k, key)] = val
            out["k%d_seg_last" % k] = seg
            if seg_first is not None:
                out["k%d_seg_first" % k] = seg_first
            if red is not None:
                for key, val in red.items():
                    if val is not None:
                        out["k%d_red_%s" % (k, key)] = val
            hist.append("%d:%d/%s" % (new["rVc"].size - 1, int(new["active"].sum()),
                                       "-" if red is None else red["rEu"].size))
            state = new
        out["meta_steps"] = np.int32(CC.STEPS)
        out["meta_build"] = np.str_("g++ -O3 -ffp-contract=off, no OpenMP")
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print("%-26s V=%d E=%d  rV:active/rE per iteration %s" % (name, V, E, " ".join(hist)))


def check_iteration_simplex(o, ref, c, state, new, seg_last, red):
    """the oracle chain of the simplex driver against one reference
    iteration; returns the derived segments of every expansion but the last"""
    d = CC.cp_graph_iteration_simplex(o, lambda tr, rc: ref.maxflow(c["Eu"], c["Ev"], tr, rc),
                                      c, state, rP_new=new["rP"])
    assert np.array_equal(d["segments"][-1], seg_last), "last expansion segments"
    if d["activated"] == 0:
        assert red is None
        for k in ("active", "Cv", "Vc", "rVc", "rP"):
            assert np.array_equal(state[k], new[k]), k
        return d["segments"][:-1]
    assert red is not None
    for k in ("Cv", "Vc", "rVc"):
        assert np.array_equal(d[k], new[k]), k
    rEu, rEv, rLa, _ = d["reduced"]
    assert np.array_equal(rEu, red["rEu"]), "rEu"
    assert np.array_equal(rEv, red["rEv"]), "rEv"
    assert np.array_equal(rLa, red["rLa_d1"]), "rLa_d1"
    rP0, rQ, rLa_f = d["observations"]
    assert np.array_equal(rP0, red["rP0"]), "rP0"
    assert np.array_equal(rQ, red["rQ"]), "rQ"
    if rLa_f is not None:
        assert np.array_equal(rLa_f, red["rLa_f"]), "rLa_f"
    assert np.array_equal(d["active_post"], new["active"]), "active after merge"
    return d["segments"][:-1]


def main_simplex():
    """the simplex driver (src/CP_PFDR_graph_loss_d1_simplex.cpp); per
    iteration also ``k{k}_seg_exp{n}`` for the expansions before the last
    (derived through the reference's BK maxflow like seg_first above)"""
    o = Oracle("port")
    ref = CPStepRefSimplex()
    for name, c in CC.make_simplex_cases().items():
        out = {}
        for k, v in c.items():
            if v is not None:
                out["in_" + k] = np.asarray(v)
        K, al = c["K"], c["al"]
        V, E = c["Q"].size // K, c["Eu"].size
        rP0 = ref.init(K, al, c["Q"], c["Eu"], c["Ev"], c["La_d1"])
        state = {"active": np.zeros(E, np.uint8), "Cv": np.zeros(V, np.int32),
                 "Vc": np.arange(V, dtype=np.int32), "rVc": np.array([0, V], np.int32),
                 "rP": rP0}
        # the initial values are the reduced observations of one component
        oP, _, _ = o.cp_simplex_reduced(K, al, c["Q"], state["Vc"], state["rVc"])
        assert np.array_equal(oP, rP0), "initial rP"
        hist = []
        for k in range(CC.STEPS):
            new, seg, red = ref.step(K, al, c["Q"], c["Eu"], c["Ev"], c["La_d1"],
                                     c["CP_difTol"], state, difTol=CC.SIMPLEX_PFDR_DIFTOL)
            segs = check_iteration_simplex(o, ref, c, state, new, seg, red)
            for key, val in state.items():
                out["k%d_in_%s" % (k, key)] = val
            for key, val in new.items():
                out["k%d_out_%s" % (k, key)] = val
            out["k%d_seg_last" % k] = seg
            for n, sg in enumerate(segs, 1):
                out["k%d_seg_exp%d" % (k, n)] = sg
            if red is not None:
                for key, val in red.items():
                    if val is not None:
                        out["k%d_red_%s" % (k, key)] = val
            hist.append("%d:%d/%s" % (new["rVc"].size - 1, int(new["active"].sum()),
                                       "-" if red is None else red["rEu"].size))
            state = new
        out["meta_steps"] = np.int32(CC.STEPS)
        out["meta_build"] = np.str_("g++ -O3 -ffp-contract=off, no OpenMP")
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print("%-28s V=%d E=%d K=%d rV:active/rE per iteration %s"
              % (name, V, E, K, " ".join(hist)))


def main_duplex():
    """the duplex driver's non-differentiable case
    (src/CP_PFDR_graph_quadratic_d1_l1_duplex.cpp): one two-layer cut per
    iteration, whose 2V segments the reference records (k{k}_seg_last)"""
    o = Oracle("port")
    ref = CPStepRefDuplex()
    for name, c in CC.make_duplex_cases().items():
        out = {}
        for k, v in c.items():
            if v is not None:
                out["in_" + k] = np.asarray(v)
        V, E = c["Y"].size, c["Eu"].size
        rX0 = ref.init(c["Y"], c["A"], c["Eu"], c["Ev"], c["La_d1"], c["La_l1"],
                       c["positivity"])
        state = {"active": np.zeros(E, np.uint8), "Cv": np.zeros(V, np.int32),
                 "Vc": np.arange(V, dtype=np.int32), "rVc": np.array([0, V], np.int32),
                 "rX": rX0}
        hist = []
        for k in range(CC.STEPS):
            new, seg, red = ref.step(c["Y"], c["A"], c["Eu"], c["Ev"], c["La_d1"], c["La_l1"],
                                     c["positivity"], c["CP_difTol"], state)
            mf = lambda tr, link, rc: ref.maxflow(V, c["Eu"], c["Ev"], tr, link, rc)
            d = CC.cp_graph_iteration_duplex(o, mf, c, state, rX_new=new["rX"])
            assert np.array_equal(d["segments"][0], seg), "segments"
            if d["activated"] == 0:
                assert red is None
            else:
                for key in ("Cv", "Vc", "rVc"):
                    assert np.array_equal(d[key], new[key]), key
                rEu, rEv, rLa, rL1 = d["reduced"]
                assert np.array_equal(rEu, red["rEu"]), "rEu"
                assert np.array_equal(rEv, red["rEv"]), "rEv"
                assert np.array_equal(rLa, red["rLa_d1"]), "rLa_d1"
                if rL1 is not None:
                    assert np.array_equal(rL1, red["rLa_l1"]), "rLa_l1"
                assert np.array_equal(d["active_post"], new["active"]), "active after merge"
            for key, val in state.items():
                out["k%d_in_%s" % (k, key)] = val
            for key, val in new.items():
                out["k%d_out_%s" % (k, key)] = val
            out["k%d_seg_last" % k] = seg
            if red is not None:
                for key, val in red.items():
                    if val is not None:
                        out["k%d_red_%s" % (k, key)] = val
            hist.append("%d:%d/%s" % (new["rVc"].size - 1, int(new["active"].sum()),
                                       "-" if red is None else red["rEu"].size))
            state = new
        out["meta_steps"] = np.int32(CC.STEPS)
        out["meta_build"] = np.str_("g++ -O3 -ffp-contract=off, no OpenMP")
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print("%-30s V=%d E=%d  rV:active/rE per iteration %s" % (name, V, E, " ".join(hist)))


def main():
    if "--bounds" in sys.argv:
        return main_bounds()
    if "--duplex" in sys.argv:
        return main_duplex()
    if "--simplex" in sys.argv:
        return main_simplex()
    o = Oracle("port")
    ref = CPStepRef()
    for name, c in CC.make_cases().items():
        out = {}
        for k, v in c.items():
            if v is not None:
                out["in_" + k] = np.asarray(v)
        V, E = c["Y"].size, c["Eu"].size
        rX0 = ref.init(c["Y"], c["A"], c["Eu"], c["Ev"], c["La_d1"], c["La_l1"],
                       c["positivity"])
        state = {"active": np.zeros(E, np.uint8), "Cv": np.zeros(V, np.int32),
                 "Vc": np.arange(V, dtype=np.int32), "rVc": np.array([0, V], np.int32),
                 "rX": rX0}
        hist = []
        for k in range(CC.STEPS):
            new, seg, red = ref.step(c["Y"], c["A"], c["Eu"], c["Ev"], c["La_d1"], c["La_l1"],
                                     c["positivity"], c["CP_difTol"], state)
            seg_first = check_iteration(o, ref, c, state, new, seg, red)
            for key, val in state.items():
                out["k%d_in_%s" % (k, key)] = val
            for key, val in new.items():
                out["k%d_out_%s" % (k, key)] = val
            out["k%d_seg_last" % k] = seg
            if seg_first is not None:
                out["k%d_seg_first" % k] = seg_first
            if red is not None:
                for key, val in red.items():
                    if val is not None:
                        out["k%d_red_%s" % (k, key)] = val
            hist.append("%d:%d/%s" % (new["rVc"].size - 1, int(new["active"].sum()),
                                       "-" if red is None else red["rEu"].size))
            state = new
        out["meta_steps"] = np.int32(CC.STEPS)
        out["meta_build"] = np.str_("g++ -O3 -ffp-contract=off, no OpenMP")
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print("%-26s V=%d E=%d  rV:active/rE per iteration %s" % (name, V, E, " ".join(hist)))


if __name__ == "__main__":
    main()
