"""CPU: the restatement (oracle/) against the REFERENCE (oracle/_ref, its own
sources compiled single-threaded here) on the edge cases of
tests/edge_cases.py -- no edges, one vertex, isolated vertices, zero-weight
edges (0/0 NaNs), duplicate / mirrored edges, zero iterations, a zero-width
box, K = 1..3 labels: X, it and Dif bit for bit, NaNs included (the
restatement sums Dif sequentially, like the reference)."""
import numpy as np
import pytest

import edge_cases as EC
import golden_io as G
import oracle

CASES = EC.cases()


@pytest.mark.skipif(not oracle.available("ref"), reason="reference build absent (oracle/_ref)")
@pytest.mark.parametrize("name", sorted(CASES))
def test_restatement_matches_reference_on_edge_cases(oracle_port, name):
    c = CASES[name]
    ref = oracle.Oracle("ref")
    a = G.replay(oracle_port, c, False, obj=False, dif=True)
    b = G.replay(ref, c, False, obj=False, dif=True)
    assert EC.same(a, b, exact_dif=True), (name, a[1], b[1], a[0][:4], b[0][:4])
