"""GPU: small graphs iterate in one workgroup launch per chunk
(k_tiny_iterate, PFDR_TINY = largest edge count, 0 = off).  The kernel runs
the same device code as the per-iteration sweeps (edge_full, vertex_block,
reduce_decide_block), so iterates, iteration counts and the evolution
record must be identical bit for bit to the multi-launch path -- and, for
f64 at a fixed iteration count, to the reference's golden iterates -- on
every graph-mode golden case, fixed-k and converged (with reconditioning
where the case has it), and on CP-sized grids."""
import os

import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

QUAD = [n for n in G.names() if n.startswith(("l1_", "bounds_"))
        and "direct" not in n and "AtA" not in n]


def _replay(lib, c, fixed, tiny):
    old = os.environ.get("PFDR_TINY")
    os.environ["PFDR_TINY"] = tiny
    try:
        return G.replay(lib, c, fixed, obj=False, dif=True)
    finally:
        if old is None:
            del os.environ["PFDR_TINY"]
        else:
            os.environ["PFDR_TINY"] = old


@pytest.mark.parametrize("name", QUAD)
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
def test_tiny_identical(gpu_lib, name, fixed):
    c, g = G.load(name)
    X1, it1, _, D1 = _replay(gpu_lib, c, fixed, "100000")
    X0, it0, _, D0 = _replay(gpu_lib, c, fixed, "0")
    assert it1 == it0
    assert np.array_equal(X1, X0)
    assert np.array_equal(D1[:it1], D0[:it0])
    if fixed and X1.dtype == np.float64:
        assert np.array_equal(X1, g["fixk_X"])


def test_tiny_taken_and_cp_sized(gpu_lib):
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    for n, dt in ((16, np.float32), (45, np.float64), (64, np.float32)):
        shape = (n, n)
        Eu, Ev = grid_graph(shape, 4)
        V = n * n
        Y = piecewise_observation(shape, 1, dt)
        res = []
        for tiny in ("100000", "0"):
            os.environ["PFDR_TINY"] = tiny
            try:
                s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev,
                                 np.full(Eu.size, 0.1, dt), np.zeros(V, dt), Y,
                                 La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3,
                                 difRcd=1e-2, difTol=1e-5, itMax=2000, record_dif=True)
            finally:
                del os.environ["PFDR_TINY"]
            assert s.query("tiny") == (1 if tiny != "0" else 0)
            s.run(2000)
            res.append(s.result())
            s.close()
        (X1, it1, _, D1), (X0, it0, _, D0) = res
        assert it1 == it0 and it1 < 2000
        assert np.array_equal(X1, X0)
        assert np.array_equal(D1[:it1], D0[:it0])
