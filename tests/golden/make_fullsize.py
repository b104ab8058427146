"""Pin every BASELINE.json configuration at its FULL size to the REFERENCE.

Container-side (needs oracle/_ref/libpfdr_ref_seq.so, i.e. the reference
PFDR sources compiled without OpenMP by `make -C oracle ref`): regenerates
each case of tests/fullsize_cases.py with the native generators, runs the
reference on it and writes tests/golden/fullsize/<case>.npz holding
sha256(X bytes), ||X||_2, X at deterministic sample positions, it and Dif
(plus the C3 Lipschitz constant L, an INPUT of that case, estimated here by
a float64 power method).  Single-threaded reference build: no
thread-count-dependent rounding.

    python tests/golden/make_fullsize.py [case ...]      (default: all)

Run times here (8-core container, one thread): c5_k1 is the largest
(V = 262M, E = 785M, ~40 GB of host memory)."""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import Oracle  # noqa: E402
import fullsize_cases as F  # noqa: E402

OUT = os.path.join(HERE, "fullsize")


def power_norm(A_cm, N, V, its=60, seed=11):
    """||A||^2 of the column-major N-by-V matrix (float64 power method on
    A^t A; a value, not a pin: it is stored as an input of the case)."""
    A2 = A_cm.reshape(V, N)  # row v = column v of A
    x = np.asarray(F.pfdr.gen_uniform(seed, V, -1.0, 1.0, np.float64))
    lam = 0.0
    for _ in range(its):
        x /= np.linalg.norm(x)
        r = A2.T @ x.astype(np.float32)                        # A x   (N)
        y = (A2 @ r).astype(np.float64)                        # A^t A x (V)
        lam_new = float(np.dot(x, y))
        x = y
        if abs(lam_new - lam) <= 1e-7 * lam_new:
            lam = lam_new
            break
        lam = lam_new
    return lam * (1.0 + 1e-3)  # a hair above the estimate


def main():
    names = sys.argv[1:] or list(F.CASES)
    os.makedirs(OUT, exist_ok=True)
    ref = Oracle("ref")
    for name in names:
        t0 = time.perf_counter()
        extra = {}
        L = None
        if name in ("c3_direct_k2", "c3_direct_conv"):
            case = F.build(name)
            a = case["args"]
            L = power_norm(a["A"], a["N"], a["X0"].size)
            a["L"] = np.array([L], np.float32)
            extra["L"] = np.float32(L)
        else:
            case = F.build(name)
        in_sha = F.input_digest(case)
        t1 = time.perf_counter()
        X, it, Dif = F.run(ref, case)
        t2 = time.perf_counter()
        d = F.digest(X, it, Dif, case["sample_m"])
        if os.environ.get("PFDR_SAVE_X"):  # whole iterate, for local analysis only
            np.save(os.path.join(os.environ["PFDR_SAVE_X"], name + ".npy"), X)
        if name in F.DENSE:
            # the same problem through the reference's double instantiation
            # (inputs widened exactly): the accuracy yardstick of the f32 runs
            # (the reference's sequential f32 dot products over V terms carry
            # rounding error of their own)
            a = case["args"]
            for k in ("X0", "Y", "A", "La_d1", "La_l1", "L"):
                if a.get(k) is not None:
                    a[k] = a[k].astype(np.float64)
            del X
            t3 = time.perf_counter()
            X64, it64, Dif64 = F.run(ref, case)
            d64 = F.digest(X64, it64, np.zeros(0), case["sample_m"])
            extra["ref64_Dif"] = np.asarray(Dif64)
            extra["ref64_sample"] = d64["sample"]
            extra["ref64_norm2"] = d64["norm2"]
            extra["ref64_it"] = d64["it"]
            print("  f64 reference %.1fs" % (time.perf_counter() - t3), flush=True)
            X = X64
        d.update(extra)
        d["in_sha256"] = np.str_(in_sha)
        d["meta_build"] = np.str_("reference src/PFDR_*.cpp, g++ -O3 -ffp-contract=off, no OpenMP")
        d["meta_seconds"] = np.float64(t2 - t1)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **d)
        print("%-14s it=%-5d |X|=%.9g finite=%s gen %.1fs ref %.1fs" % (
            name, it, d["norm2"], bool(d["finite"]), t1 - t0, t2 - t1), flush=True)
        del case, X


if __name__ == "__main__":
    main()
