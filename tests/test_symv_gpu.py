"""GPU: A^tA mode (N = -V) past the sequential-order range of small dense
problems (V > 8192, test_parity_gpu.py covers the small ones): the products
taken from the block upper triangle of an exactly symmetric matrix
(k_symv_tiles / k_symv_finish), or, for a matrix that is not exactly
symmetric or a V off the 16-byte vector, by full column dots (k_col_dot,
which reads the whole matrix as given) -- against the C restatement
(oracle/) on ragged sizes.  Both regroup the reference's dot products
(src/PFDR_graph_quadratic_d1_l1.cpp:368-376, :432-440, :462-464), so they
are held to the dense tolerance of test_parity_gpu.py: relative l2 <= 2e-5
(f32) / 1e-12 (f64) at a fixed iteration count."""
import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

def _tol(dt, fixed):
    if fixed:
        return 2e-5 if dt == np.float32 else 1e-12
    return 1e-5 if dt == np.float32 else 1e-9


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


# V = 8320 (whole 128 / 64 tiles), 8452 (ragged tiles); 8450 / 8449: V off
# the 16-byte vector (f32 / f64) and an asymmetric matrix: column dots
CASES = [(8320, 64, np.float32, False, 1), (8452, 2, np.float32, False, 1),
         (8450, 2, np.float32, False, 0), (8452, 2, np.float32, True, 0),
         (8320, 64, np.float64, False, 1), (8449, 7, np.float64, False, 0)]


@pytest.mark.parametrize("V,nx,dt,asym,symv", CASES,
                         ids=["%d-%s%s" % (c[0], np.dtype(c[2]).name, "-asym" if c[3] else "")
                              for c in CASES])
def test_dense_ata_matches_oracle(gpu_lib, oracle_port, V, nx, dt, asym, symv):
    from cp_pfdr_graph_d1_amd import pfdr
    A, Y, Eu, Ev, L = _problem(V, dt, V, nx)
    if asym:
        A[3, 700] = np.nextafter(A[3, 700], dt(np.inf))
    La = np.full(Eu.size, 0.05, dt)
    L1 = np.full(V, 0.01, dt)
    X0 = np.zeros(V, dt)
    Af = A.ravel(order="F")
    s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, La, X0, Y, N=-V, A=Af, L=L,
                     itMax=1)
    assert s.query("symv") == symv and s.query("dense_exact") == 0
    s.close()
    kw = dict(La_l1=L1, positivity=0, Ltype=0, L=L, rho=1.5, condMin=1e-3, difRcd=0.0,
              difTol=0.0, itMax=20, obj=True, dif=True)
    ref = oracle_port.quadratic_d1_l1(X0, Y, Af, -V, Eu, Ev, La, **kw)
    got = gpu_lib.quadratic_d1_l1(X0, Y, Af, -V, Eu, Ev, La, **kw)
    e = G.rel_l2(got[0], ref[0])
    print("V=%d %s symv=%d vs oracle rel_l2=%.3e" % (V, np.dtype(dt).name, symv, e))
    assert got[1] == ref[1] == 20
    assert e <= _tol(dt, True)
    assert np.allclose(got[2], ref[2], rtol=(1e-4 if dt == np.float32 else 1e-10))


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_dense_ata_symv_converged_matches_oracle(gpu_lib, oracle_port, dt):
    """the upper-triangle products run to the tolerance (reconditioning on
    the way): the stopping iteration within 2 of the restatement's and the
    converged iterate within the converged dense tolerance (the full-size
    A^tA pin, c3_ata_k3 at V = 32,768 against the reference's f64 run, is
    tests/test_fullsize_pin_gpu.py)"""
    V = 8320
    A, Y, Eu, Ev, L = _problem(V, dt, 17, 64)
    La = np.full(Eu.size, 0.05, dt)
    L1 = np.full(V, 0.01, dt)
    X0 = np.zeros(V, dt)
    Af = A.ravel(order="F")
    kw = dict(La_l1=L1, positivity=0, Ltype=0, L=L, rho=1.5, condMin=1e-3, difRcd=1e-2,
              difTol=2e-3, itMax=2000, dif=True)
    ref = oracle_port.quadratic_d1_l1(X0, Y, Af, -V, Eu, Ev, La, **kw)
    got = gpu_lib.quadratic_d1_l1(X0, Y, Af, -V, Eu, Ev, La, **kw)
    e = G.rel_l2(got[0], ref[0])
    print("V=%d %s converged: it %d / %d, rel_l2 %.3e" % (V, np.dtype(dt).name, got[1], ref[1], e))
    assert 0 < ref[1] < 2000 and abs(got[1] - ref[1]) <= 2
    if dt == np.float64:
        assert e <= _tol(dt, False)
        return
    # f32 over ~200 iterations: both runs regroup / accumulate rounding in
    # their own dot products; the yardstick is the f64 solve of the same
    # (exactly widened) problem, as for the full-size dense pins: the GPU
    # iterate at least as close to it as the restatement's f32 run
    w = lambda a: None if a is None else np.asarray(a, np.float64)
    kw64 = dict(kw, La_l1=w(L1), L=w(L))
    r64 = oracle_port.quadratic_d1_l1(w(X0), w(Y), w(Af), -V, Eu, Ev, w(La), **kw64)
    e_gpu, e_ref = G.rel_l2(got[0], r64[0]), G.rel_l2(ref[0], r64[0])
    print("  vs f64: GPU %.3e, restatement f32 %.3e (it %d)" % (e_gpu, e_ref, r64[1]))
    assert e_gpu <= 1.5 * e_ref + 1e-6
