"""GPU: the simplex beyond K = 64 labels (groups of vertices with their
columns in LDS, or past the LDS one wave per vertex with the projection on
the whole wave, pfdr_proj.hpp) at sizes where the evolution
is summed in the reference's sequential rounding and the session decides
speculatively (P and (P, step) ping-ponged): the stopping iteration, every
Dif and P equal the restatement's (itself pinned to the reference on the
golden cases simplex_k65 .. simplex_k1500), for the l1 evolution and the
label-change count, with K in registers (K = 130) and in memory (K = 1100).
Also the partitioned wide-K session (K-wide halos) against one GPU, and
speculating over 3 ranks (both concurrency modes) against the restatement."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _problem(n, K, dt, seed=4, weak=False):
    """K-label 8-neighbour grid; weak: a faint block signal in uniform noise,
    so that labels keep changing for tens of iterations"""
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, simplex_observation, uniform
    Eu, Ev = grid_graph((n, n), 8)
    V = n * n
    v = np.arange(V)
    lab = (((v % n) * 3 // n) + 3 * ((v // n) * 2 // n)) * (K // 6)
    if weak:
        Q = uniform(9, np.arange(V * K)).reshape(V, K)
        Q[v, lab] += 0.1
        Q = (Q / Q.sum(1, keepdims=True)).ravel().astype(dt)
    else:
        Q = simplex_observation(V, K, seed, lab, dt)
    return V, Eu.astype(np.int32), Ev.astype(np.int32), Q


@pytest.mark.parametrize("K,n,dt", [(130, 40, np.float32), (1100, 12, np.float32),
                                    (2000, 9, np.float64), (3500, 7, np.float32)],
                         ids=["K130", "K1100", "K2000-f64", "K3500"])
@pytest.mark.parametrize("difTol", [1e-3, 1.0], ids=["l1", "labels"])
def test_wide_speculative_matches_restatement(gpu_lib, K, n, dt, difTol):
    """K = 130 and 1,100: groups of vertices with their columns in LDS (16
    and 4 per group, SxGroup::nv_for); K = 2,000 (f64) and 3,500 (f32): past
    the LDS, one wave per vertex with the columns and active sets in memory"""
    import oracle
    from cp_pfdr_graph_d1_amd import pfdr
    labels = difTol >= 1
    V, Eu, Ev, Q = _problem(n, K, dt, weak=labels)
    La = np.full(Eu.size, 0.3 if labels else 0.05, dt)
    s = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev, La, Q.copy(), Q,
                     K=K, al=0.1, rho=1.0, condMin=0.1, difRcd=0.0, difTol=difTol, itMax=300,
                     record_dif=True, evolution=pfdr.EVOLUTION_SEQUENTIAL)
    try:
        assert s.query("speculative") == 1 and s.query("seqdif") == 1
        for m in (5, 33, 300):
            s.prepare(m)
            s.run(m)
        P, it, _, Dif = s.result()
    finally:
        s.close()
    Po, ito, _, Difo = oracle.Oracle("port").loss_d1_simplex(
        Q.copy(), Q, K, Eu, Ev, La, 0.1, None, 1.0, 0.1, 0.0, difTol, 300, dif=True)
    print("K %d difTol %g: it %d / %d" % (K, difTol, it, ito))
    assert 20 < it == ito < 300
    assert np.array_equal(Dif[:it], Difo[:ito])
    assert np.array_equal(P, Po)


@pytest.mark.parametrize("K,n", [(100, 24), (1030, 9), (3500, 6)], ids=["K100", "K1030", "K3500"])
@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_wide_partitioned_matches_single(gpu_lib, K, n, dt):
    """3 loopback ranks with K-wide halos (the pushed W*Z packed per label,
    received ends summed in the wide sweep), fixed iterations with a
    reconditioning on the way, against the single-GPU session"""
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    V, Eu, Ev, Q = _problem(n, K, dt)
    La = np.full(Eu.size, 0.05, dt)
    kw = dict(rho=1.0, condMin=0.1, difRcd=1e-2, difTol=0.0, itMax=30, record_dif=True)
    s = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev, La, Q.copy(), Q, K=K,
                     al=0.1, **kw)
    s.run(30)
    X1, it1, _, D1 = s.result()
    s.close()
    X, it, _, D, _ = P.solve_loopback(3, pfdr.PFDR_KIND_SIMPLEX, dt, Eu, Ev, La, Q.copy(), Q,
                                      K=K, al=0.1, **kw)
    assert it == it1 == 30
    assert np.array_equal(X, X1)


@pytest.mark.parametrize("K,n", [(130, 40), (1100, 12)], ids=["K130", "K1100"])
@pytest.mark.parametrize("spec", [0, 1], ids=["overlapped", "serial"])
def test_wide_partitioned_speculative_matches_restatement(gpu_lib, K, n, spec):
    """3 loopback ranks, difRcd = 0 and the sequential evolution: the
    partition decides four iterations deep (depth 4 from 3 ranks), the chain
    on a second stream over the split transport (overlapped) or on the session
    stream (serial, PFDR_SPEC_SERIAL) -- the group sweep's K-wide halos and the
    speculative pipeline together: stopping iteration, every Dif and P equal
    the restatement's"""
    import oracle
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    dt = np.float32
    V, Eu, Ev, Q = _problem(n, K, dt)
    La = np.full(Eu.size, 0.05, dt)
    X, it, _, D, info = P.solve_loopback(3, pfdr.PFDR_KIND_SIMPLEX, dt, Eu, Ev, La, Q.copy(), Q,
                                         K=K, al=0.1, rho=1.0, condMin=0.1, difRcd=0.0,
                                         difTol=1e-3, itMax=300, record_dif=True,
                                         evolution=pfdr.EVOLUTION_SEQUENTIAL, spec=spec)
    assert all(q["speculative"] == spec + 1 for q in info["queries"])
    Po, ito, _, Difo = oracle.Oracle("port").loss_d1_simplex(
        Q.copy(), Q, K, Eu, Ev, La, 0.1, None, 1.0, 0.1, 0.0, 1e-3, 300, dif=True)
    print("K %d spec %d: it %d / %d" % (K, spec, it, ito))
    assert 20 < it == ito < 300
    assert np.array_equal(D[:it], Difo[:ito])
    assert np.array_equal(X, Po)


@pytest.mark.parametrize("D", [3, 7, 31, 64, 100, 1024, 1025, 4000])
def test_projection_random_matches_restatement(gpu_lib, D):
    """proj_simplex_metric at every segment / register / memory width
    against the restatement, on columns with many active-set events"""
    import oracle
    rng = np.random.default_rng(D)
    N = 257
    X = (rng.standard_normal(D * N) * 0.5 + 1.0 / D).astype(np.float64)
    M = rng.random(D * 50) + 0.2
    A = rng.random(31) + 0.5
    got = gpu_lib.proj_simplex_metric(X, M, D, N, 50, A, 31)
    ref = oracle.Oracle("port").proj_simplex_metric(X, M, D, N, 50, A, 31)
    assert np.array_equal(got, ref)
