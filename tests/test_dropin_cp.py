"""The drop-in boundary end to end: the REFERENCE's cut-pursuit driver
(src/CP_PFDR_graph_quadratic_d1_l1.cpp + maxflow + operator norm, compiled
unchanged by oracle/Makefile) linked once with the reference PFDR and once
with libpfdr_mi355x.so.  Both binaries live in oracle/_ref (built where
/root/reference exists and shipped with the snapshot).

CPU: the MI355X-linked binary resolves every PFDR symbol from our library.
GPU: both binaries solve the same CP problems; the CP outputs (components,
component values, CP iterations) must be identical — CP calls PFDR on
reduced graphs with diagonal A^tA, a mode in which the MI355X PFDR is
bit-exact."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
REF = os.path.join(ROOT, "oracle", "_ref")
DRV_REF = os.path.join(REF, "cp_driver_ref")
DRV_GPU = os.path.join(REF, "cp_driver_mi355x")


def _need(path):
    if not os.path.exists(path):
        pytest.skip("%s not built (needs /root/reference at build time)" % path)


def test_cp_driver_links_against_dropin():
    _need(DRV_GPU)
    out = subprocess.run(["nm", "-D", "--undefined-only", DRV_GPU], capture_output=True,
                         text=True, check=True).stdout
    und = [l.split()[-1] for l in out.splitlines() if "PFDR_graph" in l]
    assert und == ["_Z26PFDR_graph_quadratic_d1_l1IdEviiiPT_PKS0_S3_PKiS5_S3_S3_i10LipschtypeS3_S0_S0_S0_S0_iPiS1_S1_i",
                   "_Z26PFDR_graph_quadratic_d1_l1IfEviiiPT_PKS0_S3_PKiS5_S3_S3_i10LipschtypeS3_S0_S0_S0_S0_iPiS1_S1_i"] \
        or sorted(und) == sorted(set(und))
    ldd = subprocess.run(["ldd", DRV_GPU], capture_output=True, text=True).stdout
    assert "libpfdr_mi355x.so" in ldd and "not found" not in ldd


def _write_problem(path, shape, dt, seed, la_d1=0.3, la_l1=0.02):
    import sys
    sys.path.insert(0, ROOT)
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation, uniform
    Eu, Ev = grid_graph(shape, 4)
    V = int(np.prod(shape))
    Y = piecewise_observation(shape, seed, dt, noise=0.4)
    A = (0.5 + uniform(seed + 1, np.arange(V))).astype(dt)
    with open(path, "wb") as f:
        np.array([V, Eu.size, 1 if dt == np.float64 else 0, 8, 2000, 0], np.int32).tofile(f)
        np.array([1e-4, 1e-5, 1.5, 1e-3], np.float64).tofile(f)
        (A * Y).astype(dt).tofile(f)
        A.tofile(f)
        Eu.astype(np.int32).tofile(f)
        Ev.astype(np.int32).tofile(f)
        np.full(Eu.size, la_d1, dt).tofile(f)
        np.full(V, la_l1, dt).tofile(f)
    return V


def _read(path, V, dt):
    raw = open(path, "rb").read()
    h = np.frombuffer(raw[:8], np.int32)
    Cv = np.frombuffer(raw[8:8 + 4 * V], np.int32)
    rX = np.frombuffer(raw[8 + 4 * V:], dt)
    assert rX.size == h[0]
    return int(h[0]), int(h[1]), Cv, rX


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("shape", [(64, 48), (160, 120)])
def test_cp_with_mi355x_pfdr_matches_reference_cp(tmp_path, dt, shape):
    _need(DRV_REF)
    _need(DRV_GPU)
    inp = str(tmp_path / "in.bin")
    V = _write_problem(inp, shape, dt, 7)
    res = {}
    for name, drv in (("ref", DRV_REF), ("gpu", DRV_GPU)):
        out = str(tmp_path / ("out_%s.bin" % name))
        subprocess.run([drv, inp, out], check=True, timeout=600)
        res[name] = _read(out, V, dt)
    (rv1, it1, cv1, x1), (rv2, it2, cv2, x2) = res["ref"], res["gpu"]
    print("CP %s %s: rV %d/%d it %d/%d" % (shape, dt.__name__, rv1, rv2, it1, it2))
    assert (rv1, it1) == (rv2, it2)
    assert np.array_equal(cv1, cv2)
    assert np.array_equal(x1, x2)
