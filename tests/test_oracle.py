"""CPU: the C restatement (oracle/) against the golden fixtures produced by
the REFERENCE itself (tests/golden/make_golden.py), and against the
reference build directly where /root/reference is present.

Expectation: bit-exact.  Both are single-threaded with no FMA contraction,
and the restatement performs every floating point operation in the
reference's order (oracle/pfdr_oracle_body.h)."""
import numpy as np
import pytest

import golden_io as G

CASES = [n for n in G.names() if not n.startswith("proj_")]


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
def test_oracle_matches_reference_golden(oracle_port, name, fixed):
    c, g = G.load(name)
    X, it, Obj, Dif = G.replay(oracle_port, c, fixed)
    tag = "fixk" if fixed else "conv"
    assert it == int(g[tag + "_it"])
    assert np.array_equal(X, g[tag + "_X"]), "X differs from the reference"
    assert np.array_equal(Dif[:it], g[tag + "_Dif"])
    if tag + "_Obj" in g:
        assert np.array_equal(Obj[:it + 1], g[tag + "_Obj"])


@pytest.mark.parametrize("name", G.names("proj_"))
def test_oracle_projection_golden(oracle_port, name):
    c, g = G.load(name)
    X = oracle_port.proj_simplex_metric(c["X"], c["M"], int(c["D"]), int(c["N"]),
                                        int(c["nm"]), c["A"], int(c["na"]))
    assert np.array_equal(X, g["out_X"])


def test_chain_known_answer(oracle_port):
    """closed form of the 1-D chain: [1.1, 1.6, -0.6, 2.9]"""
    c, _ = G.load("l1_chain_kat_f64")
    X, it, _, _ = G.replay(oracle_port, c, False)
    assert np.allclose(X, [1.1, 1.6, -0.6, 2.9], atol=1e-7)
    assert it == 23  # the reference's count


def test_projection_identity_on_feasible(oracle_port):
    rng = np.random.default_rng(0)
    x = rng.random((5, 40))
    x /= x.sum(0)
    m = rng.random((5, 40)) + 0.5
    y = oracle_port.proj_simplex_metric(x.ravel(order="F"), m.ravel(order="F"),
                                        5, 40, 40, np.ones(1), 1)
    assert np.allclose(y, x.ravel(order="F"), atol=1e-12)


def test_projection_identity_metric_matches_sort_projection(oracle_port):
    """metric = 1: the classic sort-based Euclidean projection"""
    rng = np.random.default_rng(1)
    D, N = 9, 60
    x = rng.normal(size=(D, N))
    y = oracle_port.proj_simplex_metric(x.ravel(order="F"), np.ones(D), D, N, 1,
                                        np.ones(1), 1).reshape(D, N, order="F")
    for n in range(N):
        u = np.sort(x[:, n])[::-1]
        css = np.cumsum(u) - 1.0
        r = np.nonzero(u - css / np.arange(1, D + 1) > 0)[0][-1]
        theta = css[r] / (r + 1.0)
        assert np.allclose(y[:, n], np.maximum(x[:, n] - theta, 0), atol=1e-12)


def _random_case(seed, dt):
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, uniform
    Eu, Ev = grid_graph((9, 7, 3), 26)
    V = 189
    Y = (uniform(seed, np.arange(V)) * 2 - 1).astype(dt)
    La = (0.05 + 0.1 * uniform(seed + 1, np.arange(Eu.size))).astype(dt)
    L1 = (0.01 * uniform(seed + 2, np.arange(V))).astype(dt)
    return Y, Eu, Ev, La, L1


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_oracle_vs_reference_random(dt):
    """direct call of the compiled reference (skipped on the GPU box)."""
    import oracle
    if not oracle.available("ref"):
        pytest.skip("oracle/_ref not built (reference sources absent)")
    ref, port = oracle.Oracle("ref"), oracle.Oracle("port")
    for seed in range(3):
        Y, Eu, Ev, La, L1 = _random_case(10 * seed + 1, dt)
        for pos in (0, 1):
            a = ref.quadratic_d1_l1(np.zeros_like(Y), Y, None, 0, Eu, Ev, La, L1,
                                    pos, 0, None, 1.3, 1e-2, 1e-3, 1e-6, 400, dif=True)
            b = port.quadratic_d1_l1(np.zeros_like(Y), Y, None, 0, Eu, Ev, La, L1,
                                     pos, 0, None, 1.3, 1e-2, 1e-3, 1e-6, 400, dif=True)
            assert a[1] == b[1] and np.array_equal(a[0], b[0]) and np.array_equal(a[3], b[3])
        a = ref.quadratic_d1_bounds(np.zeros_like(Y), Y, None, 0, Eu, Ev, La, -0.3, 0.4,
                                    difTol=1e-6, difRcd=1e-4, itMax=400)
        b = port.quadratic_d1_bounds(np.zeros_like(Y), Y, None, 0, Eu, Ev, La, -0.3, 0.4,
                                     difTol=1e-6, difRcd=1e-4, itMax=400)
        assert a[1] == b[1] and np.array_equal(a[0], b[0])
