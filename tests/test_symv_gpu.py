"""GPU: A^tA mode (N = -V) with the products taken from the block upper
triangle of an exactly symmetric matrix (k_symv_tiles / k_symv_finish,
PFDR_SYMV) against the reference's golden iterates, against the column-dot
path (k_col_dot, which reads the whole matrix as given) and against the C
restatement (oracle/) on larger, ragged sizes.

(The sequential-order path that small dense problems take by default,
PFDR_DENSE_EXACT, is turned off here; test_parity_gpu.py covers it.)
Both dense paths regroup the reference's dot products
(src/PFDR_graph_quadratic_d1_l1.cpp:368-376, :432-440, :462-464), so they
are held to the dense tolerance of test_parity_gpu.py: relative l2 <= 2e-5
(f32) / 1e-12 (f64) at a fixed iteration count, 1e-5 / 1e-9 converged."""
import os

import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

ATA = [n for n in G.names() if "AtA" in n]


@pytest.fixture(autouse=True)
def _tree_reduced_products(monkeypatch):
    """these problems are small enough for the sequential-order dense path
    (PFDR_DENSE_EXACT, default up to a chain of 8192): off here, so the
    tree-reduced products under test (upper triangle vs column dots) run"""
    monkeypatch.setenv("PFDR_DENSE_EXACT", "0")


class _env:
    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kw}
        os.environ.update(self.kw)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _tol(dt, fixed):
    if fixed:
        return 2e-5 if dt == np.float32 else 1e-12
    return 1e-5 if dt == np.float32 else 1e-9


def _session(c, **kw):
    from cp_pfdr_graph_d1_amd import pfdr
    kind = pfdr.PFDR_KIND_L1 if str(c["solver"]) == "l1" else pfdr.PFDR_KIND_BOUNDS
    X0 = np.asarray(c["X0"])
    extra = dict(La_l1=c.get("La_l1"), positivity=int(c.get("positivity", 0)))
    if kind == pfdr.PFDR_KIND_BOUNDS:
        extra = dict(lo=float(c["lo"]), hi=float(c["hi"]))
    return pfdr.Session(kind, X0.dtype, X0.size, c["Eu"].size, c["Eu"], c["Ev"], c["La_d1"],
                        X0, c["Y"], N=int(c["N"]), A=c["A"], Ltype=int(c["Ltype"]), L=c["L"],
                        rho=float(c["rho"]), condMin=float(c["condMin"]), **extra, **kw)


@pytest.mark.parametrize("name", ATA)
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
def test_symv_matches_reference(gpu_lib, name, fixed):
    c, g = G.load(name)
    tag = "fixk" if fixed else "conv"
    gX, git = g[tag + "_X"], int(g[tag + "_it"])
    with _env(PFDR_SYMV="1"):
        s = _session(c, itMax=1)
        assert s.query("symv") == 1, "golden A^tA is exactly symmetric: upper-triangle path expected"
        s.close()
        X1, it1, Obj1, Dif1 = G.replay(gpu_lib, c, fixed)
    with _env(PFDR_SYMV="0"):
        s = _session(c, itMax=1)
        assert s.query("symv") == 0
        s.close()
        X0, it0, _, _ = G.replay(gpu_lib, c, fixed)
    dt = X1.dtype
    e1, e0 = G.rel_l2(X1, gX), G.rel_l2(X0, gX)
    print("%s %s symv rel_l2=%.3e it=%d | col-dot %.3e it=%d | ref it=%d"
          % (name, tag, e1, it1, e0, it0, git))
    assert np.all(np.isfinite(X1))
    assert e1 <= _tol(dt, fixed)
    assert G.rel_l2(X1, X0) <= _tol(dt, fixed)
    if fixed:
        assert it1 == git
        go = g["fixk_Obj"][: it1 + 1]
        assert np.allclose(Obj1[: it1 + 1], go, rtol=(1e-4 if dt == np.float32 else 1e-10),
                           atol=1e-6 * np.abs(go).max())
    else:
        assert abs(it1 - git) <= 2


def _problem(V, dt, seed, nx):
    from cp_pfdr_graph_d1_amd import pfdr
    rng = np.random.default_rng(seed)
    M = 64
    B = rng.standard_normal((M, V)) / np.sqrt(M)
    G64 = B.T @ B
    G64 = (G64 + G64.T) * 0.5  # exactly symmetric
    A = np.asfortranarray(G64.astype(dt))
    x0 = np.where(np.arange(V) < V // 2, 1.0, -0.5)
    Y = (G64 @ x0).astype(dt)
    Eu, Ev = pfdr.gen_grid_edges((nx, V // nx), 4)
    L = np.array([np.linalg.eigvalsh(G64)[-1]], dt)
    return A, Y, Eu.astype(np.int32), Ev.astype(np.int32), L


# ragged tiles (V not a multiple of the 128 / 64 tile), several tile rows
@pytest.mark.parametrize("V,nx", [(1000, 40), (2048, 64), (1540, 44)])
@pytest.mark.parametrize("dt", [np.float32, np.float64], ids=["f32", "f64"])
def test_symv_matches_oracle(gpu_lib, oracle_port, V, nx, dt):
    A, Y, Eu, Ev, L = _problem(V, dt, V, nx)
    La = np.full(Eu.size, 0.05, dt)
    L1 = np.full(V, 0.01, dt)
    X0 = np.zeros(V, dt)
    kw = dict(La_l1=L1, positivity=0, Ltype=0, L=L, rho=1.5, condMin=1e-3, difRcd=0.0,
              difTol=0.0, itMax=30, obj=True, dif=True)
    ref = oracle_port.quadratic_d1_l1(X0, Y, A.ravel(order="F"), -V, Eu, Ev, La, **kw)
    with _env(PFDR_SYMV="1"):
        got = gpu_lib.quadratic_d1_l1(X0, Y, A.ravel(order="F"), -V, Eu, Ev, La, **kw)
    with _env(PFDR_SYMV="0"):
        cold = gpu_lib.quadratic_d1_l1(X0, Y, A.ravel(order="F"), -V, Eu, Ev, La, **kw)
    e = G.rel_l2(got[0], ref[0])
    print("V=%d %s symv vs oracle rel_l2=%.3e, col-dot %.3e" % (V, np.dtype(dt).name, e,
                                                                  G.rel_l2(cold[0], ref[0])))
    assert got[1] == ref[1] == 30
    assert e <= _tol(dt, True)
    assert np.allclose(got[2], ref[2], rtol=(1e-4 if dt == np.float32 else 1e-10))


def test_symv_not_taken_for_asymmetric_or_ragged_vectors(gpu_lib):
    from cp_pfdr_graph_d1_amd import pfdr
    for V, asym in ((1000, True), (1002, False)):
        A, Y, Eu, Ev, L = _problem(V, np.float32, 5, 2 if V == 1002 else 40)
        if asym:
            A[3, 700] = np.nextafter(A[3, 700], np.float32(np.inf))
        with _env(PFDR_SYMV="1"):
            s = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, Eu.size, Eu, Ev,
                             np.full(Eu.size, 0.05, np.float32), np.zeros(V, np.float32), Y,
                             N=-V, A=A.ravel(order="F"), L=L, itMax=5)
            assert s.query("symv") == 0
            s.run(5)
            X, it, _, _ = s.result()
            s.close()
        assert it == 5 and np.all(np.isfinite(X))
