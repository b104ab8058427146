"""Pin the CP reduced-problem builder of the dense modes (SURVEY.md §8(f)
rank 1, N != 0) to the REFERENCE itself.

Runs the reference's cut pursuit (oracle/_ref/libcp_step_ref.so, built from
/root/reference/src) on dense CP problems one iteration at a time, through
its warm-restart path, and records what CP hands to PFDR at every
iteration: the components it used (Vc, rVc), the N it passes (-rV when it
premultiplies by A^t, N for the direct reduced matrix,
src/CP_PFDR_graph_quadratic_d1_l1.cpp:671, :848-858), the data vector (rY or
Y), the matrix (rAA = rA^t rA, or rA) after the equilibration round trip
(:772-836) and the Lipschitz metric L (DIAG, from the operator norm; the
harness fixes the norm's time seed).  Cases: direct N > 0 with few
observations (the direct branch once components multiply) and with many
(premultiplied throughout), and A^tA given (N < 0); f32 and f64.
Writes tests/golden/cp_dense_<case>.npz.  Usage:
    python tests/golden/make_cp_dense_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import CPStepRef  # noqa: E402
import cp_problems as P  # noqa: E402

STEPS = 5
CASES = {"direct_few": ("direct", dict(N=12, nx=40, ny=30)),
         "direct_many": ("direct", dict(N=160, nx=24, ny=18)),
         "AtA": ("AtA", dict(nx=24, ny=18))}


def main():
    ref = CPStepRef()
    for cname, (mode, kw) in CASES.items():
        for dt, tag in ((np.float32, "f32"), (np.float64, "f64")):
            p = P.problem("l1", mode, dt, **kw)
            V, E, N = p["V"], p["E"], p["N"]
            A = p["A"]
            out = {"in_" + k: np.asarray(v) for k, v in p.items()
                   if isinstance(v, np.ndarray)}
            out["in_N"] = np.int32(N)
            rX0 = ref.init_dense(p["Y"], A, N, p["Eu"], p["Ev"], p["La_d1"], p["La_l1"], 0)
            state = {"active": np.zeros(E, np.uint8), "Cv": np.zeros(V, np.int32),
                     "Vc": np.arange(V, dtype=np.int32), "rVc": np.array([0, V], np.int32),
                     "rX": rX0}
            hist = []
            for k in range(STEPS):
                R = None
                if N > 0:  # residual of the state, Y - A X (float64, rounded once)
                    X = state["rX"].astype(np.float64)[state["Cv"]]
                    R = (p["Y"].astype(np.float64) -
                         A.reshape(V, N).astype(np.float64).T @ X).astype(dt)
                new, red = ref.step_dense(V, N, p["Y"], A, p["Eu"], p["Ev"], p["La_d1"],
                                          p["La_l1"], 0, p["CP_difTol"], state, R)
                if red is None:
                    hist.append("-")
                    state = new
                    continue
                out["k%d_Vc" % k] = new["Vc"]
                out["k%d_rVc" % k] = new["rVc"]
                for key in ("n", "Y", "A", "L"):
                    out["k%d_red_%s" % (k, key)] = np.asarray(red[key])
                hist.append("rV=%d,n=%d" % (new["rVc"].size - 1, red["n"]))
                state = new
            out["meta_steps"] = np.int32(STEPS)
            np.savez_compressed(os.path.join(HERE, "cp_dense_%s_%s.npz" % (cname, tag)), **out)
            print("%-14s %s V=%d N=%d: %s" % (cname, tag, V, N, " ".join(hist)), flush=True)


if __name__ == "__main__":
    main()
