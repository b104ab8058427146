"""GPU: the edge cases of tests/edge_cases.py (no edges, one vertex with a
self-loop, isolated vertices, zero-weight edges with the reference's 0/0
NaNs, duplicate and mirrored edges, zero iterations, a zero-width box,
K = 1..3 labels) through the C ABI against the restatement, which
tests/test_edge_cases.py pins to the reference: X, it and Dif bit for bit,
NaNs included; and invalid inputs fail with an error status, not a crash."""
import numpy as np
import pytest

import edge_cases as EC
import golden_io as G

pytestmark = pytest.mark.gpu

CASES = EC.cases()


@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_matches_restatement_on_edge_cases(gpu_lib, oracle_port, name):
    c = CASES[name]
    a = G.replay(gpu_lib, c, False, obj=False, dif=True)
    b = G.replay(oracle_port, c, False, obj=False, dif=True)
    assert EC.same(a, b), (name, a[1], b[1], a[0][:4], b[0][:4])


def test_invalid_inputs_fail_cleanly(gpu_lib):
    from cp_pfdr_graph_d1_amd import pfdr
    V = 4
    Y = np.zeros(V, np.float32)
    La = np.full(3, 0.1, np.float32)
    for Eu, Ev in (([0, 1, 4], [1, 2, 3]), ([0, -1, 2], [1, 2, 3])):
        with pytest.raises(pfdr.PFDRError):
            gpu_lib.quadratic_d1_l1(np.zeros(V, np.float32), Y, None, 0,
                                    np.asarray(Eu, np.int32), np.asarray(Ev, np.int32), La,
                                    None, 0, 0, None, 1.5, 1e-3, 0.0, 0.0, 5)
    # a negative loss parameter (the reference's al is >= 0); any K is served
    K = 1025
    Q = np.full(2 * K, 1.0 / K, np.float32)
    with pytest.raises(pfdr.PFDRError):
        gpu_lib.loss_d1_simplex(Q.copy(), Q, K, np.array([0], np.int32), np.array([1], np.int32),
                                np.array([0.1], np.float32), -0.5, None, 1.5, 1e-3, 0.0, 0.0, 3)
    # the library still works afterwards
    X, it, _, _ = gpu_lib.quadratic_d1_l1(np.zeros(V, np.float32), np.ones(V, np.float32), None,
                                          0, np.array([0, 1, 2], np.int32),
                                          np.array([1, 2, 3], np.int32), La, None, 0, 0, None,
                                          1.5, 1e-3, 0.0, 0.0, 5)
    assert it == 5 and np.all(np.isfinite(X))
