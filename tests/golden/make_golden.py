"""Generate the golden fixtures from the REFERENCE itself.

Runs the reference PFDR sources compiled without OpenMP
(oracle/_ref/libpfdr_ref_seq.so, built by `make -C oracle ref` from
/root/reference/src) on every case of cases.py and stores, per case, one
compressed .npz holding the inputs and:

* ``conv_*``  : X/P, it, Obj[0..it], Dif[0..it-1] of the run as specified;
* ``fixk_*``  : the same after exactly FIXED_K iterations with
                difTol = difRcd = 0 (Dif still recorded).

Obj is stored only where the reference computes it without its stale-index
read (src/PFDR_graph_quadratic_d1_l1.cpp:417): positivity or La_l1 == NULL.
Single-threaded build, so no thread-count-dependent rounding
(SURVEY.md §8(a) quirks).  Usage:  python tests/golden/make_golden.py
[name prefix ...]  (no prefix: every case)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, HERE)
from oracle import Oracle  # noqa: E402
import cases as C  # noqa: E402


def run_case(lib, c, fixed):
    kw = {}
    if fixed:
        kw = dict(difTol=0.0, difRcd=0.0, itMax=C.FIXED_K)
    s = c["solver"]
    if s == "l1":
        a = dict(c, **kw)
        return lib.quadratic_d1_l1(
            a["X0"], a["Y"], a["A"], a["N"], a["Eu"], a["Ev"], a["La_d1"],
            a["La_l1"], a["positivity"], a["Ltype"], a["L"], a["rho"],
            a["condMin"], a["difRcd"], a["difTol"], a["itMax"], obj=True,
            dif=True)
    if s == "bounds":
        a = dict(c, **kw)
        return lib.quadratic_d1_bounds(
            a["X0"], a["Y"], a["A"], a["N"], a["Eu"], a["Ev"], a["La_d1"],
            a["lo"], a["hi"], a["Ltype"], a["L"], a["rho"], a["condMin"],
            a["difRcd"], a["difTol"], a["itMax"], obj=True, dif=True)
    if s == "simplex":
        a = dict(c, **kw)
        return lib.loss_d1_simplex(
            a["P0"], a["Q"], a["K"], a["Eu"], a["Ev"], a["La_d1"], a["al"],
            a["La_f"], a["rho"], a["condMin"], a["difRcd"], a["difTol"],
            a["itMax"], obj=True, dif=True)
    raise ValueError(s)


def obj_valid(c):
    return not (c["solver"] == "l1" and c["La_l1"] is not None
                and not c["positivity"])


def main(prefixes=()):
    """prefixes: regenerate only the cases whose name starts with one of
    them (round 5 added the wide-K cases without rewriting the others)"""
    lib = Oracle("ref")
    cases = C.make_cases()
    for name, c in cases.items():
        if prefixes and not name.startswith(tuple(prefixes)):
            continue
        out = {}
        for k, v in c.items():
            if v is None:
                continue
            out["in_" + k] = np.asarray(v)
        if c["solver"] == "proj":
            out["out_X"] = lib.proj_simplex_metric(c["X"], c["M"], c["D"],
                                                   c["N"], c["nm"], c["A"],
                                                   c["na"])
        else:
            for tag, fixed in (("conv", False), ("fixk", True)):
                X, it, Obj, Dif = run_case(lib, c, fixed)
                out[tag + "_X"] = X
                out[tag + "_it"] = np.int32(it)
                out[tag + "_Dif"] = Dif[:it]
                if obj_valid(c):
                    out[tag + "_Obj"] = Obj[:it + 1]
        out["meta_threads"] = np.int32(1)
        out["meta_build"] = np.str_("g++ -O3 -ffp-contract=off, no OpenMP")
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print("%-28s %s" % (name, "it=%d" % out["conv_it"]
                            if "conv_it" in out else "proj"))


if __name__ == "__main__":
    main(sys.argv[1:])
