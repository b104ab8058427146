"""CPU: the C-ABI library loads, exports every entry point the header
declares and the reference's C++ drop-in symbols; host-side pieces work
without a GPU; compute entries fail loudly without one."""
import os
import re
import subprocess

import numpy as np
import pytest

from cp_pfdr_graph_d1_amd import pfdr
from cp_pfdr_graph_d1_amd.graphs import (grid_graph, knn_jitter_grid,
                                        piecewise_observation)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HEADER = os.path.join(ROOT, "include", "pfdr_mi355x.h")

# explicit instantiations of the reference, verified with nm
REFERENCE_SYMBOLS = [
    "_Z26PFDR_graph_quadratic_d1_l1IfEviiiPT_PKS0_S3_PKiS5_S3_S3_i10LipschtypeS3_S0_S0_S0_S0_iPiS1_S1_i",
    "_Z26PFDR_graph_quadratic_d1_l1IdEviiiPT_PKS0_S3_PKiS5_S3_S3_i10LipschtypeS3_S0_S0_S0_S0_iPiS1_S1_i",
    "_Z30PFDR_graph_quadratic_d1_boundsIfEviiiPT_PKS0_S3_PKiS5_S3_S0_S0_10LipschtypeS3_S0_S0_S0_S0_iPiS1_S1_i",
    "_Z30PFDR_graph_quadratic_d1_boundsIdEviiiPT_PKS0_S3_PKiS5_S3_S0_S0_10LipschtypeS3_S0_S0_S0_S0_iPiS1_S1_i",
    "_Z26PFDR_graph_loss_d1_simplexIfEviiiT_PKS0_PS0_S2_PKiS5_S2_S0_S0_S0_S0_iPiS3_S3_i",
    "_Z26PFDR_graph_loss_d1_simplexIdEviiiT_PKS0_PS0_S2_PKiS5_S2_S0_S0_S0_S0_iPiS3_S3_i",
    "_Z19proj_simplex_metricIfEvPT_PKS0_iiiS3_i",
    "_Z19proj_simplex_metricIdEvPT_PKS0_iiiS3_i",
    "_Z20operator_norm_matrixIfET_iiPKS0_S0_iii",
    "_Z20operator_norm_matrixIdET_iiPKS0_S0_iii",
]


def header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(pfdr_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_python_list():
    assert header_functions() == sorted(pfdr.EXPORTED)


def test_library_exports_every_declared_symbol():
    lib = pfdr.load()
    for name in header_functions():
        assert hasattr(lib, name), name


def _dynsyms(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True,
                         capture_output=True, text=True).stdout
    return {l.split()[-1] for l in out.splitlines() if l.strip()}


def test_dropin_cxx_symbols_exported():
    syms = _dynsyms(pfdr.LIB_PATH)
    for s in REFERENCE_SYMBOLS:
        assert s in syms, s


def test_dropin_symbols_equal_reference_build():
    path = os.path.join(ROOT, "oracle", "_ref", "libpfdr_ref_omp.so")
    if not os.path.exists(path):
        pytest.skip("reference build absent")
    def cxx(syms):
        return {s for s in syms if s.startswith("_Z") and
                ("PFDR_graph" in s or "proj_simplex_metric" in s or "operator_norm_matrix" in s)}
    ref, ours = cxx(_dynsyms(path)), cxx(_dynsyms(pfdr.LIB_PATH))
    assert ref == ours == set(REFERENCE_SYMBOLS)


def test_abi_version():
    assert pfdr.load().pfdr_abi_version() == pfdr.ABI_VERSION == 4


@pytest.mark.parametrize("shape", [(7, 5, 4), (12, 9, 6), (3, 3, 3)])
def test_native_knn_generator_matches_numpy(shape):
    a = knn_jitter_grid(shape, 6, 6)
    b = pfdr.gen_knn_jitter_grid(shape, 6, 6)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    V = int(np.prod(shape))
    c = pfdr.gen_knn_jitter_grid(shape, 6, 6, v_range=(V // 3, V // 2))
    assert np.array_equal(c[0], a[0][6 * (V // 3): 6 * (V // 2)])


@pytest.mark.parametrize("shape,conn", [((7, 5), 4), ((7, 5), 8), ((4, 5, 6), 6),
                                        ((4, 5, 6), 26)])
def test_native_grid_generator_matches_numpy(shape, conn):
    a = grid_graph(shape, conn)
    b = pfdr.gen_grid_edges(shape, conn)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_native_observation_matches_numpy():
    for dt in (np.float32, np.float64):
        y1 = piecewise_observation((10, 4, 3), 2, dt)
        y2 = pfdr.gen_piecewise(10, 120, 2, dt)
        assert np.array_equal(y1, y2)


def test_knn_headline_edge_count():
    Eu, Ev = knn_jitter_grid((6, 5, 4), 6)
    assert Eu.size == 6 * 120
    assert np.all(Eu != Ev)


def test_compute_fails_loudly_without_gpu():
    lib = pfdr.load()
    if lib.pfdr_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(pfdr.PFDRError):
        pfdr.Lib().quadratic_d1_l1(np.zeros(4, np.float32), np.ones(4, np.float32), None, 0,
                                   np.array([0, 1, 2]), np.array([1, 2, 3]),
                                   np.ones(3, np.float32))
