"""GPU parity at BASELINE.json's FULL sizes against the REFERENCE.

tests/golden/make_fullsize.py ran the reference PFDR (its own sources,
single-threaded build) on every configuration of tests/fullsize_cases.py
at full size — C1 (fixed 25 and converged to 1e-6), the 10M/60M headline,
C2 256^3, C3 dense N = 1024 x V = 2M direct and the V = 32,768 A^tA mode,
C4 simplex K = 10 on 5M vertices, C5 bounds on 640^3 (262M vertices, 785M
edges) — and committed digests of its output.  Here the MI355X library runs
the same inputs (regenerated on this host; their sha256 is checked first)
through the host-pointer C ABI that CP callers use, and:

  * graph modes (identity / diagonal A) and the simplex: sha256 of X equal
    to the reference's (bit-exact at full size), same iteration count, Dif
    within 1e-4 (f32) / 1e-9 (f64) relative (the evolution statistic is
    tree-reduced, it does not feed the iterate);
  * dense A (c3_*): the dot products are regrouped, so X at 65,536 (V = 2M)
    / every (V = 32,768) sampled coordinate within 1e-5 relative l2 (the
    north star's bound) and ||X|| within 1e-5;
  * converged C1: iteration count within 2 and 1e-9 relative l2 (f64) on
    every coordinate, bit-exact when the counts agree.

These catch size-only bugs the small fixtures cannot: int32 offsets, the
split-incidence / staged-sweep fallbacks, CSR chunks beyond one workgroup.
"""
import os

import numpy as np
import pytest

import fullsize_cases as F

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize")
DENSE = ("c3_direct_k2", "c3_ata_k3")


def _gold(name):
    p = os.path.join(GOLD, name + ".npz")
    if not os.path.exists(p):
        pytest.fail("%s missing: run tests/golden/make_fullsize.py where the reference exists" % p)
    return np.load(p)


@pytest.mark.parametrize("name", F.CASES)
def test_fullsize_matches_reference(gpu_lib, name):
    g = _gold(name)
    case = F.build(name, L_c3=float(g["L"]) if "L" in g else None)
    assert F.input_digest(case) == str(g["in_sha256"]), \
        "the native generators produced different inputs on this host"
    X, it, Dif = F.run(gpu_lib, case)
    d = F.digest(X, it, Dif, case["sample_m"])
    del case
    git = int(g["it"])
    samp, gs = d["sample"].astype(np.float64), g["sample"].astype(np.float64)
    assert np.array_equal(d["idx"], g["idx"])
    err = np.linalg.norm(samp - gs) / max(np.linalg.norm(gs), 1e-300)
    exact = str(d["sha256"]) == str(g["sha256"])
    print("%s: it %d/%d sample rel_l2 %.3e |X| %.9g/%.9g bit-exact %s" % (
        name, it, git, err, float(d["norm2"]), float(g["norm2"]), exact))
    assert bool(d["finite"])
    if name in DENSE:
        assert it == git
        assert err <= 1e-5
        assert abs(float(d["norm2"]) - float(g["norm2"])) <= 1e-5 * float(g["norm2"])
        return
    if name == "c1_conv":
        assert abs(it - git) <= 2 and err <= 1e-9
        if it == git:
            assert exact
        return
    assert it == git
    assert exact, "graph-mode / simplex iterate differs from the reference at full size"
    n = min(it, git)
    tol = 1e-4 if X.dtype == np.float32 else 1e-9
    gd = g["Dif"][:n].astype(np.float64)
    assert np.linalg.norm(Dif[:n] - gd) <= tol * np.linalg.norm(gd)
