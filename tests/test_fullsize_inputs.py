"""CPU checks of the full-size reference pins (tests/golden/fullsize/):
every BASELINE configuration has one, and the native generators reproduce
the pinned inputs bit for bit (cheap cases here; the GPU test checks every
case's input digest on the box before comparing outputs)."""
import os

import numpy as np
import pytest

import fullsize_cases as F

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize")


@pytest.mark.parametrize("name", F.CASES)
def test_pin_present_and_sane(name):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    assert bool(g["finite"]) and int(g["it"]) >= 1
    assert g["idx"].size == g["sample"].size > 0
    assert np.all(np.diff(g["idx"]) > 0) and g["idx"][-1] < int(g["size"])
    assert len(str(g["sha256"])) == 64 and len(str(g["in_sha256"])) == 64
    assert g["Dif"].size == int(g["it"])


@pytest.mark.parametrize("name", ["c1_fixk25", "c1_conv", "headline_k3"])
def test_generators_reproduce_pinned_inputs(name):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    case = F.build(name)
    assert F.input_digest(case) == str(g["in_sha256"])


def test_dense_generators_deterministic():
    """the C3 generators are thread-count independent: the matvec sums each
    row in double in column order (checked against numpy float64)"""
    from cp_pfdr_graph_d1_amd import pfdr
    N, V = 37, 1001
    A = pfdr.gen_uniform(3, N * V, -0.5, 0.5, np.float32)
    assert np.array_equal(A, pfdr.gen_uniform(3, N * V, -0.5, 0.5, np.float32))
    x = pfdr.gen_uniform(4, V, -1, 1, np.float32)
    y = pfdr.gen_matvec(A, N, V, x)
    ref = np.zeros(N)
    A2 = A.reshape(V, N).astype(np.float64)
    for v in range(V):
        ref += A2[v] * float(x[v])
    assert np.array_equal(y, ref.astype(np.float32))
    G = pfdr.gen_symmetric(50, 33, 0.1, 1.0, np.float32).reshape(50, 50)
    assert np.array_equal(G, G.T) and np.all(np.diag(G) == 1.0)
