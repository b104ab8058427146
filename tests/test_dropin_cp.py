"""The drop-in boundary end to end: the REFERENCE's four cut-pursuit drivers
(src/CP_PFDR_graph_quadratic_d1_l1.cpp, _l1_duplex.cpp, _bounds.cpp,
src/CP_PFDR_graph_loss_d1_simplex.cpp, with maxflow and the operator norm;
compiled unchanged by oracle/Makefile through oracle/harness/cp_drivers.cpp)
linked once with the reference PFDR and once with libpfdr_mi355x.so.  Both
binaries of a kind live in oracle/_ref (built where /root/reference exists,
shipped with the snapshot).

CPU: every MI355X-linked binary resolves its PFDR symbols from our library.
GPU: both binaries solve the same CP problems (tests/cp_problems.py) and the
CP outputs — components Cv, component values rX (simplex: rP), CP iteration
count — must be IDENTICAL, in f32 and f64, for
  * N = 0 (diagonal A^tA; identity for bounds): the graph modes, bit-exact;
  * N > 0 (dense A): CP hands PFDR premultiplied reduced problems (n = -rV)
    while rV is small and the direct N-by-rV matrix once rV grows
    (src/CP_PFDR_graph_quadratic_d1_l1.cpp:671, :848-858) -- both bit-exact
    through the sequential-order dense products of small problems;
  * N < 0 (A^tA given) for l1;
  * the simplex with its barycentre warm start and rLa_f = component sizes
    (src/CP_PFDR_graph_loss_d1_simplex.cpp:733-780).
The operator norm (time-seeded in the reference) is made deterministic by
the harness (see cp_drivers.cpp), so the two binaries differ only in PFDR.
"""
import os
import subprocess

import numpy as np
import pytest

import cp_problems as P

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
REF = os.path.join(ROOT, "oracle", "_ref")

CASES = [("l1", "diag"), ("l1", "direct"), ("l1", "AtA"), ("duplex", "diag"),
         ("duplex", "direct"), ("bounds", "identity"), ("bounds", "diag"),
         ("bounds", "direct"), ("simplex", "")]


def _need(path):
    if not os.path.exists(path):
        pytest.skip("%s not built (needs /root/reference at build time)" % path)


@pytest.mark.parametrize("kind", list(P.KINDS))
def test_cp_driver_links_against_dropin(kind):
    drv = P.driver(kind, "mi355x", REF)
    _need(drv)
    out = subprocess.run(["nm", "-D", "--undefined-only", drv], capture_output=True,
                         text=True, check=True).stdout
    und = [l.split()[-1] for l in out.splitlines() if "PFDR_graph" in l]
    want = {"l1": "26PFDR_graph_quadratic_d1_l1", "duplex": "26PFDR_graph_quadratic_d1_l1",
            "bounds": "30PFDR_graph_quadratic_d1_bounds",
            "simplex": "26PFDR_graph_loss_d1_simplex"}[kind]
    assert und and all(want in u for u in und), und
    # the library defines exactly those symbols
    lib = os.path.join(ROOT, "cp_pfdr_graph_d1_amd", "libpfdr_mi355x.so")
    defs = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True,
                          check=True).stdout
    for u in und:
        assert u in defs, u
    ldd = subprocess.run(["ldd", drv], capture_output=True, text=True).stdout
    assert "libpfdr_mi355x.so" in ldd and "not found" not in ldd


def test_reference_cp_drivers_run_on_cpu(tmp_path):
    """The reference-linked binaries solve every problem here (CPU only) and
    find more than one component: the problems exercise real cuts."""
    for kind, mode in CASES:
        drv = P.driver(kind, "ref", REF)
        _need(drv)
        p = P.problem(kind, mode, np.float32)
        inp, out = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
        P.write(inp, p)
        subprocess.run([drv, inp, out], check=True, timeout=300, capture_output=True)
        rV, it, Cv, rX = P.read(out, p)
        assert 1 < rV < p["V"] and it >= 1 and np.all(np.isfinite(rX)), (kind, mode, rV)
        assert Cv.min() == 0 and Cv.max() == rV - 1


def _solve_both(tmp_path, p):
    inp = str(tmp_path / "in.bin")
    P.write(inp, p)
    res = {}
    for prov in ("ref", "mi355x"):
        drv = P.driver(p["kind"], prov, REF)
        _need(drv)
        out = str(tmp_path / ("out_%s.bin" % prov))
        r = subprocess.run([drv, inp, out], timeout=600, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-2000:]
        res[prov] = P.read(out, p)
    return res["ref"], res["mi355x"]


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [np.float32, np.float64], ids=["f32", "f64"])
@pytest.mark.parametrize("kind,mode", CASES, ids=["%s-%s" % c if c[1] else c[0] for c in CASES])
def test_cp_with_mi355x_pfdr_matches_reference_cp(tmp_path, kind, mode, dt):
    p = P.problem(kind, mode, dt)
    (rv1, it1, cv1, x1), (rv2, it2, cv2, x2) = _solve_both(tmp_path, p)
    print("CP %s %s %s: rV %d/%d it %d/%d" % (kind, mode, dt.__name__, rv1, rv2, it1, it2))
    assert (rv1, it1) == (rv2, it2)
    assert np.array_equal(cv1, cv2)
    assert np.array_equal(x1, x2)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [np.float32, np.float64], ids=["f32", "f64"])
@pytest.mark.parametrize("shape", [(64, 48), (160, 120)])
def test_cp_l1_larger_grids(tmp_path, dt, shape):
    p = P.problem("l1", "diag", dt, nx=shape[0], ny=shape[1])
    (rv1, it1, cv1, x1), (rv2, it2, cv2, x2) = _solve_both(tmp_path, p)
    assert (rv1, it1) == (rv2, it2)
    assert np.array_equal(cv1, cv2)
    assert np.array_equal(x1, x2)
