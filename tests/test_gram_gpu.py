"""GPU: Gram matrices on the matrix cores and the operator norm (SURVEY.md
§8(f) rank 1, reference src/operator_norm_matrix.cpp), against float64
numpy and the reference's own power method (where built).

Tolerances: the exact-f32 MFMA chain rounds once per product
(≈1e-7 relative per element, cdna_hip_programming.md §3), so the f32 Gram
is held to 2e-6 relative Frobenius error, f64 to 1e-13, and it must be
exactly symmetric.  The power method stops on a relative evolution below
nTol, so the squared norm is held to 10 nTol of the SVD value."""
import numpy as np
import pytest

from cp_pfdr_graph_d1_amd import pfdr

pytestmark = pytest.mark.gpu


def _mat(M, N, seed, dt):
    rng = np.random.default_rng(seed)
    return rng.uniform(-1, 1, (M, N)).astype(dt)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
# (64, 3000) / (96, 4096) with which = 0: hundreds of output tiles and one
# contraction chunk -- every XCD takes an eighth of the tiles (gram_block),
# ragged (300 tiles over 8 x 38 slots) and even (528 over 8 x 66)
# (256, 1024), (384, 4096): whole 128-wide tiles, one and many contraction
# chunks
@pytest.mark.parametrize("shape", [(100, 37), (333, 129), (64, 300), (1000, 257), (20000, 96),
                                   (64, 3000), (96, 4096), (256, 1024), (384, 4096)])
@pytest.mark.parametrize("which", [0, 1])
def test_gram_matches_numpy(gpu_lib, dt, shape, which):
    A = _mat(*shape, seed=sum(shape) + which, dt=dt)
    G, ms = pfdr.gram(A, which)
    A64 = A.astype(np.float64)
    ref = A64.T @ A64 if which == 0 else A64 @ A64.T
    err = np.linalg.norm(G - ref) / np.linalg.norm(ref)
    print("gram %s %s which=%d err=%.2e %.3f ms" % (dt.__name__, shape, which, err, ms))
    assert G.shape == ref.shape
    assert np.array_equal(G, G.T)
    assert err <= (2e-6 if dt == np.float32 else 1e-13)


def test_gram_short_last_chunk(gpu_lib):
    """A A^t of a 2048 x 20000 f32 A: 16 contraction chunks of 1280, the
    last one 800 long (20000 = 15 x 1280 + 800)"""
    A = _mat(2048, 20000, seed=7, dt=np.float32)
    G, ms = pfdr.gram(A, 1)
    A64 = A.astype(np.float64)
    ref = A64 @ A64.T
    err = np.linalg.norm(G - ref) / np.linalg.norm(ref)
    print("gram 2048 x 20000 err=%.2e %.3f ms" % (err, ms))
    assert np.array_equal(G, G.T)
    assert err <= 2e-6


@pytest.mark.parametrize("which", [0, 1])
def test_gram_huge_entries(gpu_lib, which):
    """an entry past the largest bf16 (3.4e38) is split by truncation, not
    rounded to inf: its finite products stay finite and exact to f32.  A
    product that overflows f32 is +inf, as in the reference's f32 sums: the
    split tile's pieces would overflow with both signs (NaN), so its NaN
    flag sends the Gram to the exact-f32 tile (pfdr_gram.hip gram())"""
    rng = np.random.default_rng(3)
    B = rng.uniform(-1, 1, (128, 64)).astype(np.float32)  # rows = Gram index
    B[:, 0] = 0.0
    B[0, 0] = np.float32(3.4e38)
    B[1, 0] = np.float32(1e-30)  # (normal: MFMA inputs may flush subnormals)
    A = B if which == 1 else np.ascontiguousarray(B.T)  # A A^t of B, or A^t A of B^t
    G, _ = pfdr.gram(A, which)
    B64 = B.astype(np.float64)
    ref = B64 @ B64.T
    assert np.isposinf(G[0, 0])
    assert abs(G[0, 1] - ref[0, 1]) <= 1e-6 * abs(ref[0, 1]) and G[0, 1] == G[1, 0]
    sub, rsub = G[1:, 1:].astype(np.float64), ref[1:, 1:]
    assert np.linalg.norm(sub - rsub) <= 2e-6 * np.linalg.norm(rsub)
    assert np.all(np.isfinite(G[0, 1:]))



@pytest.mark.parametrize("which", [0, 1])
def test_gram_infinite_entry(gpu_lib, which):
    """an infinite entry gives the exact-f32 tile's signed infinities (the
    split would give NaN: h = inf, m = inf - inf); rows and columns away from
    it stay finite and accurate"""
    rng = np.random.default_rng(4)
    B = rng.uniform(0.5, 1.0, (96, 48)).astype(np.float32)
    B *= np.where(rng.random(B.shape) < 0.5, -1, 1).astype(np.float32)
    B[2, 5] = np.inf
    A = B if which == 1 else np.ascontiguousarray(B.T)
    G, _ = pfdr.gram(A, which)
    want = np.sign(B[:, 5]).astype(np.float32) * np.float32(np.inf)
    want[2] = np.inf
    assert np.array_equal(G[2], want) and np.array_equal(G[:, 2], want)
    keep = np.arange(96) != 2
    sub = G[np.ix_(keep, keep)].astype(np.float64)
    B64 = B[keep].astype(np.float64)
    ref = B64 @ B64.T
    assert np.all(np.isfinite(sub))
    assert np.linalg.norm(sub - ref) <= 2e-6 * np.linalg.norm(ref)


def _spectral(M, N, s, seed, dt):
    """A = U diag(s) V^t with orthonormal U, V: ||A||^2 = max(s)^2"""
    rng = np.random.default_rng(seed)
    U, _ = np.linalg.qr(rng.standard_normal((M, len(s))))
    V, _ = np.linalg.qr(rng.standard_normal((N, len(s))))
    return ((U * s) @ V.T).astype(dt)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("shape,itMax", [((300, 200), 200), ((2000, 64), 400), ((64, 5000), 200),
                                         ((40, 30), 1)])
def test_operator_norm_matches_svd(gpu_lib, dt, shape, itMax):
    M, N = shape
    k = min(M, N)
    s = np.linspace(0.2, 1.0, k) ** 2
    s[-1] = 2.0  # clear spectral gap: 4 vs 1
    A = _spectral(M, N, s, 5, dt)
    exact = float(np.linalg.norm(A.astype(np.float64), 2) ** 2)
    tol = 1e-6
    got, gms = pfdr.operator_norm(A, nTol=tol, itMax=itMax, nbInit=10)
    print("opnorm %s %s got %.7g exact %.7g gram %.3f ms" % (dt.__name__, shape, got, exact, gms))
    if itMax > 1:
        assert abs(got - exact) / exact <= (1e-4 if dt == np.float32 else 1e-5)
    else:  # one iteration: a lower estimate
        assert 0 < got <= exact * (1 + 1e-5)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_operator_norm_symmetric_input(gpu_lib, dt):
    """M = 0: A is A^tA itself (reference :95-103)"""
    B = _spectral(50, 40, np.linspace(0.5, 3.0, 40), 9, np.float64)
    AtA = (B.T @ B).astype(dt)
    exact = float(np.linalg.eigvalsh(B.T @ B).max())
    got, _ = pfdr.operator_norm(AtA, nTol=1e-7, itMax=500, nbInit=4, symmetric=True)
    assert abs(got - exact) / exact <= (1e-4 if dt == np.float32 else 1e-6)


def test_operator_norm_vs_reference_power_method(gpu_lib):
    """the reference's own estimate (time-seeded) and ours agree within the
    CP settings' tolerance (nTol = 1e-3, 100 iterations, 10 starts)"""
    import oracle
    if not oracle.available("ref_omp"):
        pytest.skip("reference OpenMP build absent")
    A = _spectral(400, 300, np.r_[np.linspace(0.1, 1.0, 299), 1.5], 3, np.float64)
    ref = oracle.Oracle("ref_omp").operator_norm(A.T.copy(), 400, 300, 1e-3, 100, 10)
    got, _ = pfdr.operator_norm(A, nTol=1e-3, itMax=100, nbInit=10)
    exact = 2.25
    assert abs(ref - exact) / exact < 1e-2
    assert abs(got - exact) / exact < 1e-2
