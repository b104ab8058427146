"""GPU: the internal kernel variants chosen by the sessions give the same
iterates bit for bit, so none of them can drift from the reference.

Quadratic solvers: split incidence / CSR gather in the vertex sweep, u ends
staged in LDS / Eu streamed in the edge sweep (PFDR_SPLIT, PFDR_USTAGE),
amplitude sum by the workgroup binade scan / one lane (PFDR_SEQSUM), the
pipelined (chunked) iteration schedule (PFDR_CHUNKS).
Simplex: two (edge, label) entries per lane / one (PFDR_SX_PAIR), prox
weights recomputed from the factored splitting weights / stored
(PFDR_SX_PW).  Every golden case of the reference, with reconditioning where
the case has it, at the fixed iteration count and converged."""
import os

import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

QUAD = [n for n in G.names() if n.startswith(("l1_", "bounds_"))
        and "direct" not in n and "AtA" not in n]
SIMPLEX = [n for n in G.names() if n.startswith("simplex_")]


def _replay(lib, c, fixed, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return G.replay(lib, c, fixed)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _same(a, b):
    X0, it0, _, D0 = a
    X1, it1, _, D1 = b
    assert it0 == it1
    assert np.array_equal(X0, X1)
    if D0 is not None and D1 is not None:
        assert np.array_equal(D0[:it0], D1[:it1])


@pytest.mark.parametrize("name", QUAD)
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
def test_quadratic_variants_identical(gpu_lib, name, fixed):
    c, g = G.load(name)
    base = _replay(gpu_lib, c, fixed, {"PFDR_SPLIT": "1", "PFDR_USTAGE": "1"})
    for env in ({"PFDR_SPLIT": "0", "PFDR_USTAGE": "1"}, {"PFDR_SPLIT": "1", "PFDR_USTAGE": "0"},
                {"PFDR_SPLIT": "0", "PFDR_USTAGE": "0"}, {"PFDR_SEQSUM": "lane"},
                {"PFDR_TINY": "0", "PFDR_CHUNKS": "3"}, {"PFDR_TINY": "0", "PFDR_CHUNKS": "2"}):
        _same(base, _replay(gpu_lib, c, fixed, env))
    if fixed and base[0].dtype == np.float64:
        assert np.array_equal(base[0], g["fixk_X"])


@pytest.mark.parametrize("name", SIMPLEX)
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
def test_simplex_variants_identical(gpu_lib, name, fixed):
    c, g = G.load(name)
    base = _replay(gpu_lib, c, fixed, {"PFDR_SX_PAIR": "1", "PFDR_SX_PW": "0"})
    for env in ({"PFDR_SX_PAIR": "1", "PFDR_SX_PW": "1"}, {"PFDR_SX_PAIR": "0", "PFDR_SX_PW": "1"},
                {"PFDR_SX_PAIR": "0", "PFDR_SX_PW": "0"}):
        _same(base, _replay(gpu_lib, c, fixed, env))
    if fixed and base[0].dtype == np.float64:
        assert np.array_equal(base[0], g["fixk_X"])
