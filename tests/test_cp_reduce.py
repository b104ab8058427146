"""CP reduced-problem builder (reference
src/CP_PFDR_graph_quadratic_d1_l1.cpp:663-841).

CPU: the C restatement (oracle/cp_reduce_body.h) against a float64 numpy
statement of the same algebra (rA = A R, rAA = rA^t rA, rY = rA^t Y with R
the vertex-to-component indicator).  GPU: pfdr_cp_reduce against the
restatement, bit for bit on rA, rAA, rY and the equilibration factors (every
sum sequential in the reference's order); L = l^2 c against the exact
squared norm of the equilibrated matrix within 10 nTol.  The reference
never exposes these arrays (they live inside CP), so the restatement is
the pin ("parity pinned to the restatement")."""
import numpy as np
import pytest

from cp_pfdr_graph_d1_amd.graphs import uniform


def components(V, rV, seed):
    """random partition of V vertices into rV non-empty components, each
    listed in a scrambled order (as CP's DFS lists them)"""
    u = uniform(seed, np.arange(V))
    lab = np.r_[np.arange(rV), (u[rV:] * rV).astype(np.int64)] if V > rV else np.arange(V)
    order = np.argsort(uniform(seed + 1, np.arange(V)), kind="stable")
    Vc = np.concatenate([order[lab[order] == r] for r in range(rV)]).astype(np.int32)
    ptr = np.r_[0, np.cumsum(np.bincount(lab, minlength=rV))].astype(np.int32)
    return ptr, Vc, lab


def problem(kind, dt, V=60, rV=9, N=17, seed=3):
    ptr, Vc, lab = components(V, rV, seed)
    if kind == "direct":
        A = ((uniform(seed + 2, np.arange(N * V)) - 0.5).reshape(N, V)).astype(dt)
        Y = (uniform(seed + 3, np.arange(N)) - 0.5).astype(dt)
        return N, A, Y, ptr, Vc, lab
    if kind == "ata":
        B = ((uniform(seed + 2, np.arange(N * V)) - 0.5).reshape(N, V)).astype(np.float64)
        return -V, (B.T @ B).astype(dt), (uniform(seed + 3, np.arange(V)) - 0.5).astype(dt), ptr, Vc, lab
    A = (0.5 + uniform(seed + 2, np.arange(V))).astype(dt) if kind == "diag" else None
    return 0, A, (uniform(seed + 3, np.arange(V)) - 0.5).astype(dt), ptr, Vc, lab


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("kind", ["direct", "ata", "diag", "ident"])
def test_restatement_matches_numpy_algebra(oracle_port, dt, kind):
    N, A, Y, ptr, Vc, lab = problem(kind, dt)
    V, rV = Vc.size, ptr.size - 1
    R = np.zeros((V, rV))
    R[np.arange(V), lab] = 1.0
    o = oracle_port.cp_reduce(N, A, Y, ptr, Vc, preAt=True)
    tol = 1e-5 if dt == np.float32 else 1e-12
    rel = lambda a, b: np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-300)
    if kind == "direct":
        rA = A.astype(np.float64) @ R
        assert rel(o["rA"], rA) <= tol
        assert rel(o["rAA"], rA.T @ rA) <= tol
        assert rel(o["rY"], rA.T @ Y.astype(np.float64)) <= tol
        assert np.allclose(o["Leq"], np.sqrt(np.diag(rA.T @ rA)), rtol=tol)
    elif kind == "ata":
        assert rel(o["rAA"], R.T @ A.astype(np.float64) @ R) <= tol
        assert rel(o["rY"], R.T @ Y.astype(np.float64)) <= tol
    else:
        d = A.astype(np.float64) if A is not None else np.ones(V)
        assert rel(o["rAA"], R.T @ d) <= tol
        assert rel(o["rY"], R.T @ Y.astype(np.float64)) <= tol


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("kind,preAt", [("direct", True), ("direct", False), ("ata", True),
                                        ("diag", True), ("ident", True)])
@pytest.mark.parametrize("size", [(60, 9, 17), (3000, 257, 300)])
def test_gpu_builder_bitexact(gpu_lib, oracle_port, dt, kind, preAt, size):
    from cp_pfdr_graph_d1_amd import pfdr
    V, rV, N = size
    N, A, Y, ptr, Vc, lab = problem(kind, dt, V, rV, N)
    g = pfdr.cp_reduce(N, A, Y, ptr, Vc, preAt=preAt, normTol=1e-6, normItMax=500)
    o = oracle_port.cp_reduce(N, A, Y, ptr, Vc, preAt=preAt)
    for k in ("rA", "rAA", "rY", "Leq"):
        if o[k] is None:
            continue
        assert np.array_equal(g[k], o[k]), k
    if N == 0:
        assert np.array_equal(g["L"], o["rAA"])
        return
    l = o["Leq"].astype(np.float64)
    if kind == "direct" and not preAt:
        Meq = o["rA"].astype(np.float64) / l
        c = np.linalg.norm(Meq, 2) ** 2
    else:
        Meq = o["rAA"].astype(np.float64) / np.outer(l, l)
        c = np.linalg.eigvalsh(Meq).max()
    # the power method stops on a relative evolution below nTol: without a
    # spectral gap it can stop short of the top eigenvalue
    assert np.allclose(g["L"], l * l * c, rtol=2e-2)


# ---- pinned to the REFERENCE: the dense reduced problems its cut pursuit
# handed to PFDR (tests/golden/make_cp_dense_golden.py, N > 0 direct and
# premultiplied branches, N < 0), iteration by iteration
import os  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DENSE_PINS = sorted(f[:-4] for f in os.listdir(GOLD) if f.startswith("cp_dense_"))


def _pinned_iterations(name):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    N, V = int(g["in_N"]), int(g["in_Y"].size if int(g["in_N"]) <= 0 else g["in_La_l1"].size)
    A = g["in_A"]
    Am = A.reshape(V, N).T if N > 0 else A.reshape(V, V)
    ks = sorted({int(k.split("_")[0][1:]) for k in g.files if k.startswith("k") and "_red_" in k})
    return g, N, V, Am, ks


def _check_pin(out, g, k, N):
    n = int(g["k%d_red_n" % k])
    A, Y = g["k%d_red_A" % k], g["k%d_red_Y" % k]
    if n > 0:   # direct reduced matrix rA (N x rV, column major), original Y
        assert np.array_equal(out["rA"].T.ravel(), A), "rA"
        assert np.array_equal(Y, g["in_Y"])
    else:       # premultiplied: rAA (rV x rV) and rY
        assert np.array_equal(np.asarray(out["rAA"]).ravel(), A), "rAA"
        assert np.array_equal(out["rY"], Y), "rY"
    return n


@pytest.mark.parametrize("name", DENSE_PINS)
def test_restatement_pinned_to_reference_dense(oracle_port, name):
    """the restatement rebuilds, from the components the reference used,
    the exact arrays the reference handed to PFDR, and the reference's L is
    Leq^2 times one operator-norm estimate c"""
    g, N, V, Am, ks = _pinned_iterations(name)
    assert ks, "no recorded PFDR call"
    branches = set()
    for k in ks:
        n = int(g["k%d_red_n" % k])
        o = oracle_port.cp_reduce(N, Am, g["in_Y"], g["k%d_rVc" % k], g["k%d_Vc" % k],
                                  preAt=n < 0)
        branches.add(_check_pin(o, g, k, N) > 0)
        L = g["k%d_red_L" % k].astype(np.float64)
        c = L / o["Leq"].astype(np.float64) ** 2
        assert np.allclose(c, c.mean(), rtol=1e-5), "L = Leq^2 c with one c"
    if "direct_few" in name:
        assert branches == {True}
    else:
        assert branches == {False}


@pytest.mark.gpu
@pytest.mark.parametrize("name", DENSE_PINS)
def test_gpu_builder_pinned_to_reference_dense(gpu_lib, name):
    """pfdr_cp_reduce on the reference's recorded components: rA / rAA / rY
    bit for bit as the reference built them; L within the power method's
    tolerance of the reference's (its starts are time-seeded, ours fixed)"""
    from cp_pfdr_graph_d1_amd import pfdr
    g, N, V, Am, ks = _pinned_iterations(name)
    for k in ks:
        n = int(g["k%d_red_n" % k])
        out = pfdr.cp_reduce(N, Am, g["in_Y"], g["k%d_rVc" % k], g["k%d_Vc" % k], preAt=n < 0)
        _check_pin(out, g, k, N)
        L_ref = g["k%d_red_L" % k].astype(np.float64)
        assert np.allclose(out["L"], L_ref, rtol=2e-2), (k, np.max(np.abs(out["L"] / L_ref - 1)))
