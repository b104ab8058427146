"""GPU: mid-size graphs iterate in one persistent launch per chunk
(k_coop_iterate: resident workgroups, grid barriers between the edge pass,
the vertex pass and the decision; PFDR_COOP = most vertex blocks, 0 = off;
PFDR_COOP_G = most workgroups).  The kernel runs the sweeps' own device code
(edge_lane, vertex_block, k_reduce_decide's tree in every workgroup), so
iterates, iteration counts and the evolution record must be identical bit
for bit to the multi-launch path -- and, for f64 at a fixed iteration count,
to the reference's golden iterates -- on every graph-mode golden case,
fixed-k and converged (with reconditioning where the case has it), on
C1-sized grids, and with several blocks per workgroup (grid-stride loops)."""
import os

import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

QUAD = [n for n in G.names() if n.startswith(("l1_", "bounds_"))
        and "direct" not in n and "AtA" not in n]


class _env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("name", QUAD)
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
@pytest.mark.parametrize("G_", ["0", "2"], ids=["fullgrid", "2wg"])
def test_coop_identical(gpu_lib, name, fixed, G_):
    c, g = G.load(name)
    with _env(PFDR_TINY="0", PFDR_COOP="100000", PFDR_COOP_G=G_):
        X1, it1, _, D1 = G.replay(gpu_lib, c, fixed, obj=False, dif=True)
    with _env(PFDR_TINY="0", PFDR_COOP="0"):
        X0, it0, _, D0 = G.replay(gpu_lib, c, fixed, obj=False, dif=True)
    assert it1 == it0
    assert np.array_equal(X1, X0)
    assert np.array_equal(D1[:it1], D0[:it0])
    if fixed and X1.dtype == np.float64:
        assert np.array_equal(X1, g["fixk_X"])


def _grid_session(n, dt, extra_env, **kw):
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    shape = (n, n)
    Eu, Ev = grid_graph(shape, 4)
    V = n * n
    Y = piecewise_observation(shape, 1, dt)
    with _env(**extra_env):
        s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev,
                         np.full(Eu.size, 0.1, dt), np.zeros(V, dt), Y,
                         La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3, **kw)
    return s


@pytest.mark.parametrize("n,dt", [(64, np.float32), (256, np.float64), (300, np.float32)])
def test_coop_c1_sized(gpu_lib, n, dt):
    """C1's 256^2 grid in f64 (and ragged sizes: 300^2 leaves a partial vertex
    block and a partial edge chunk) converged with reconditioning."""
    res = []
    for env in ({"PFDR_COOP": "100000"}, {"PFDR_COOP": "0"}):
        s = _grid_session(n, dt, env, difRcd=1e-2, difTol=1e-6, itMax=3000, record_dif=True)
        coop = s.query("coop")
        assert (coop > 0) == (env["PFDR_COOP"] != "0")
        s.run(3000)
        res.append(s.result())
        s.close()
    (X1, it1, _, D1), (X0, it0, _, D0) = res
    assert it1 == it0 and it1 < 3000
    assert np.array_equal(X1, X0)
    assert np.array_equal(D1[:it1], D0[:it0])


def test_coop_ungated_fixed_count(gpu_lib):
    """difTol = difRcd = 0 and no records: the kernel runs exactly the chunk
    (no control block), across several run() calls."""
    res = []
    for env in ({"PFDR_COOP": "100000", "PFDR_COOP_G": "7"}, {"PFDR_COOP": "0"}):
        s = _grid_session(200, np.float32, env, difRcd=0.0, difTol=0.0, itMax=100)
        for k in (1, 33, 66):
            s.run(k)
        res.append(s.result())
        s.close()
    (X1, it1, _, _), (X0, it0, _, _) = res
    assert it1 == it0 == 100
    assert np.array_equal(X1, X0)
