"""The Python front-end with the reference binding's conventions
(cp_pfdr_graph_d1_amd.pfdr.PFDR_quadratic_l1, SURVEY.md §8(f) rank 4;
python/CP_quadratic_l1_py.cpp): argument checking on CPU, results on the GPU
against the C restatement (oracle) called with the explicit arguments the
conventions stand for."""
import numpy as np
import pytest

from cp_pfdr_graph_d1_amd import pfdr
from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation, uniform


def _problem(dt, shape=(12, 10)):
    Eu, Ev = grid_graph(shape, 4)
    obs = piecewise_observation(shape, 3, dt, noise=0.3)
    return obs, Eu.astype(np.uint32), Ev.astype(np.uint32)


def test_rejects_bad_dtype_and_shapes():
    obs, s, t = _problem(np.float32)
    with pytest.raises(TypeError):
        pfdr.PFDR_quadratic_l1(obs.astype(np.int32), s, t, 0.1, 1.0, 0.01)
    with pytest.raises(ValueError):
        pfdr.PFDR_quadratic_l1(obs, s, t, 0.1, np.ones(obs.size + 1, np.float32), 0.01)
    with pytest.raises(ValueError):
        pfdr.PFDR_quadratic_l1(obs, s, t, 0.1, np.ones((obs.size + 1, 5), np.float32), 0.01)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("mode", ["identity", "diagonal", "matrix"])
def test_conventions_match_explicit_call(gpu_lib, oracle_port, dt, mode):
    obs, s, t = _problem(dt)
    V = obs.size
    Eu, Ev = s.astype(np.int32), t.astype(np.int32)
    ew = np.full(Eu.size, 0.2, dt)
    lw = np.full(V, 0.02, dt)
    kw = dict(PFDR_rho=1.5, PFDR_condMin=1e-3, PFDR_difRcd=0.0, PFDR_difTol=0.0, PFDR_itMax=40)
    if mode == "identity":
        X, it = pfdr.PFDR_quadratic_l1(obs, s, t, 0.2, 1.0, 0.02, **kw)
        ref = oracle_port.quadratic_d1_l1(np.zeros(V, dt), obs, None, 0, Eu, Ev, ew, lw, 0, 0,
                                          None, 1.5, 1e-3, 0.0, 0.0, 40)[0]
        assert np.array_equal(X, ref)
    elif mode == "diagonal":
        a = (0.5 + uniform(4, np.arange(V))).astype(dt)
        X, it = pfdr.PFDR_quadratic_l1(obs, s, t, ew, a, lw, **kw)
        ref = oracle_port.quadratic_d1_l1(np.zeros(V, dt), (obs * a).astype(dt), (a * a).astype(dt),
                                          0, Eu, Ev, ew, lw, 0, 1, (a * a).astype(dt), 1.5, 1e-3,
                                          0.0, 0.0, 40)[0]
        assert np.array_equal(X, ref)
    else:
        N = 48
        A = ((uniform(5, np.arange(N * V)) - 0.5).reshape(N, V) * 0.5).astype(dt)
        y = (A @ obs).astype(dt)
        X, it = pfdr.PFDR_quadratic_l1(y, s, t, 0.2, A, 0.02, **kw)
        L = np.array([np.linalg.norm(A.astype(np.float64), 2) ** 2], dt)
        ref = oracle_port.quadratic_d1_l1(np.zeros(V, dt), y, np.asfortranarray(A).ravel(order="F"),
                                          N, Eu, Ev, ew, lw, 0, 0, L, 1.5, 1e-3, 0.0, 0.0, 40)[0]
        # L comes from the power method (nTol 1e-3) here, from the SVD in the
        # oracle call: same problem, slightly different metric
        assert np.linalg.norm(X - ref) / np.linalg.norm(ref) < 2e-2
    assert it == 40
