"""The iterate-evolution statistic with the reference's sequential rounding
(PFDR_EVOLUTION_SEQUENTIAL, include/pfdr_mi355x.h).

The reference adds the evolution terms one by one in `real`
(src/PFDR_graph_quadratic_d1_l1.cpp:514-529: sum (X_ - X)^2 and sum X^2;
src/PFDR_graph_loss_d1_simplex.cpp:653-691: sum |P_ - P| over V K terms, or
the count of changed labels).  The sequential mode stores the terms in the
reference's order and sums them with the binade scan of pfdr_monosum.hpp,
which rounds exactly as that loop -- so Dif is the reference's bit for bit,
and with it the stopping / reconditioning iterations:

  * every golden case (fixed-k and converged) forced through the sequential
    mode: X, it and Dif equal to the reference's fixtures, bit for bit;
  * AUTO picks it on its own for sums of >= 2^17 terms outside the
    small-graph paths (a 640^2 grid: 1,600 vertex blocks, past the fused
    range of 1,024; a simplex with 2^17 (vertex, label) entries), checked
    against the single-threaded C restatement (whose sums are the
    reference's loops);
  * a relabelled session (random labels, internal breadth-first order) still
    sums in the caller's vertex order.
"""
import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

CASES = [n for n in G.names() if not n.startswith("proj_")]


def _session_replay(c, fixed, evolution, reorder=0):
    from cp_pfdr_graph_d1_amd import pfdr
    kw = dict(difTol=0.0, difRcd=0.0, itMax=G.FIXED_K) if fixed else {}
    a = dict(c, **kw)
    s = str(a["solver"])
    dt = a["Y"].dtype if s != "simplex" else a["Q"].dtype
    common = dict(rho=float(a["rho"]), condMin=float(a["condMin"]),
                  difRcd=float(a["difRcd"]), difTol=float(a["difTol"]),
                  itMax=int(a["itMax"]), record_dif=True, evolution=evolution,
                  reorder=reorder)
    if s == "simplex":
        K = int(a["K"])
        V = a["Q"].size // K
        ses = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, dt, V, a["Eu"].size, a["Eu"], a["Ev"],
                           a["La_d1"], a["P0"], a["Q"], K=K, al=float(a["al"]),
                           La_l1=a["La_f"], **common)
    else:
        V = a["X0"].size
        kind = pfdr.PFDR_KIND_L1 if s == "l1" else pfdr.PFDR_KIND_BOUNDS
        extra = dict(La_l1=a["La_l1"], positivity=int(a["positivity"])) if s == "l1" else \
            dict(lo=float(a["lo"]), hi=float(a["hi"]))
        ses = pfdr.Session(kind, dt, V, a["Eu"].size, a["Eu"], a["Ev"], a["La_d1"], a["X0"],
                           a["Y"], N=int(a["N"]), A=a["A"], Ltype=int(a["Ltype"]), L=a["L"],
                           **extra, **common)
    try:
        ses.run(int(a["itMax"]))
        X, it, _, Dif = ses.result()
        seq = ses.query("seqdif")
    finally:
        ses.close()
    return X, it, Dif, seq


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
def test_sequential_evolution_matches_reference_bitexact(gpu_lib, name, fixed):
    from cp_pfdr_graph_d1_amd import pfdr
    c, g = G.load(name)
    X, it, Dif, seq = _session_replay(c, fixed, pfdr.EVOLUTION_SEQUENTIAL)
    tag = "fixk" if fixed else "conv"
    gX, git, gD = g[tag + "_X"], int(g[tag + "_it"]), g[tag + "_Dif"]
    print("%s %s it=%d/%d seqdif=%d" % (name, tag, it, git, seq))
    assert seq == 1
    assert it == git
    assert np.array_equal(Dif[:it], gD[:it]), "Dif differs from the reference's sequential sums"
    if not any(d in name for d in ("direct", "AtA")) or np.array_equal(X, gX):
        assert np.array_equal(X, gX)


def _grid_problem(n, dt, seed=3):
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph
    Eu, Ev = grid_graph((n, n), 4)
    V = n * n
    Y = pfdr.gen_piecewise(n, V, seed, dt, 0.2)
    return V, Eu.astype(np.int32), Ev.astype(np.int32), Y


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_auto_sequential_at_size_matches_restatement(gpu_lib, dt):
    """V = 640^2 (AUTO takes the sequential sums): converged X, it and every
    Dif equal to the single-threaded restatement's"""
    import oracle
    from cp_pfdr_graph_d1_amd import pfdr
    V, Eu, Ev, Y = _grid_problem(640, dt)
    La = np.full(Eu.size, 0.1, dt)
    L1 = np.full(V, 0.01, dt)
    args = (np.zeros(V, dt), Y, None, 0, Eu, Ev, La, L1, 0, pfdr.SCAL, None, 1.5, 1e-3, 0.0,
            1e-4 if dt == np.float32 else 1e-5, 3000)
    X, it, _, Dif = gpu_lib.quadratic_d1_l1(*args, dif=True)
    Xo, ito, _, Difo = oracle.Oracle("port").quadratic_d1_l1(*args, dif=True)
    print("it %d/%d" % (it, ito))
    assert it == ito
    assert np.array_equal(Dif[:it], Difo[:it])
    assert np.array_equal(X, Xo)


def test_auto_sequential_simplex_matches_restatement(gpu_lib):
    """simplex, V K = 2^17 * 2.5 terms (AUTO sequential): l1 evolution and
    label-change count both equal the restatement's"""
    import oracle
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, simplex_observation
    n, K = 256, 5
    Eu, Ev = grid_graph((n, n), 8)
    V = n * n
    v = np.arange(V)
    lab = ((v % n) * 3 // n) + 3 * ((v // n) * 2 // n)
    Q = simplex_observation(V, K, 4, lab, np.float32)
    La = np.full(Eu.size, 0.05, np.float32)
    for difTol in (1e-3, 1.0):
        args = (Q.copy(), Q, K, Eu.astype(np.int32), Ev.astype(np.int32), La, 0.1, None, 1.0,
                0.1, 0.0, difTol, 400)
        P, it, _, Dif = gpu_lib.loss_d1_simplex(*args, dif=True)
        Po, ito, _, Difo = oracle.Oracle("port").loss_d1_simplex(*args, dif=True)
        print("difTol %g: it %d/%d" % (difTol, it, ito))
        assert it == ito
        assert np.array_equal(Dif[:it], Difo[:it])
        assert np.array_equal(P, Po)


@pytest.mark.parametrize("pieces", [(3000,), (7, 50, 3000), (31, 1, 32, 3000)],
                         ids=["one-run", "runs-7-50", "runs-31-1-32"])
def test_speculative_decision_matches_restatement(gpu_lib, pieces):
    """difRcd = 0 at size: the evolution sums and the decision on iteration t
    run beside the sweeps of t + 1 (speculative session, X ping-ponged); the
    stopping iteration, every Dif and X equal the restatement's whatever the
    run lengths (chunks of 32 replayed, partial chunks launched, prepared
    tails replayed) and wherever in a chunk the stop falls"""
    import oracle
    from cp_pfdr_graph_d1_amd import pfdr
    dt = np.float32
    V, Eu, Ev, Y = _grid_problem(600, dt, seed=4)  # 1,407 blocks: past the fused range
    La = np.full(Eu.size, 0.1, dt)
    L1 = np.full(V, 0.01, dt)
    s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, La, np.zeros(V, dt), Y,
                     La_l1=L1, rho=1.5, condMin=1e-3, difRcd=0.0, difTol=1e-4, itMax=3000,
                     record_dif=True)
    try:
        assert s.query("speculative") == 1 and s.query("seqdif") == 1
        for n in pieces:
            s.prepare(n)
            s.run(n)
        X, it, _, Dif = s.result()
    finally:
        s.close()
    Xo, ito, _, Difo = oracle.Oracle("port").quadratic_d1_l1(
        np.zeros(V, dt), Y, None, 0, Eu, Ev, La, L1, 0, pfdr.SCAL, None, 1.5, 1e-3, 0.0, 1e-4,
        3000, dif=True)
    print("pieces %s: it %d / %d" % (pieces, it, ito))
    assert it == ito < 3000
    assert np.array_equal(Dif[:it], Difo[:ito])
    assert np.array_equal(X, Xo)


@pytest.mark.parametrize("difTol", [1e-3, 1.0], ids=["l1", "labels"])
def test_speculative_simplex_matches_restatement(gpu_lib, difTol):
    """the simplex session's speculative decision (P and (P, step)
    ping-ponged), run in pieces: it, Dif and P equal the restatement's
    (384^2 vertices: AUTO's 2^17 terms for the label count too)"""
    import oracle
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, simplex_observation
    n, K = 384, 5
    Eu, Ev = grid_graph((n, n), 8)
    V = n * n
    v = np.arange(V)
    lab = ((v % n) * 3 // n) + 3 * ((v // n) * 2 // n)
    Q = simplex_observation(V, K, 4, lab, np.float32)
    La = np.full(Eu.size, 0.05, np.float32)
    Eu, Ev = Eu.astype(np.int32), Ev.astype(np.int32)
    s = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, np.float32, V, Eu.size, Eu, Ev, La, Q.copy(), Q,
                     K=K, al=0.1, rho=1.0, condMin=0.1, difRcd=0.0, difTol=difTol, itMax=400,
                     record_dif=True)
    try:
        assert s.query("speculative") == 1
        for m in (5, 33, 400):
            s.prepare(m)
            s.run(m)
        P, it, _, Dif = s.result()
    finally:
        s.close()
    Po, ito, _, Difo = oracle.Oracle("port").loss_d1_simplex(
        Q.copy(), Q, K, Eu, Ev, La, 0.1, None, 1.0, 0.1, 0.0, difTol, 400, dif=True)
    print("difTol %g: it %d / %d" % (difTol, it, ito))
    assert it == ito
    assert np.array_equal(Dif[:it], Difo[:ito])
    assert np.array_equal(P, Po)


@pytest.mark.parametrize("difRcd", [1e-2, 0.0], ids=["recond", "speculative"])
def test_relabelled_session_sums_in_caller_order(gpu_lib, difRcd):
    """random vertex labels, relabelling forced on: the terms are stored at
    the caller's labels, so Dif equals the plain (unrelabelled) session's
    and the restatement's, bit for bit"""
    import oracle
    from cp_pfdr_graph_d1_amd import pfdr
    dt = np.float32
    V, Eu, Ev, Y = _grid_problem(384, dt, seed=5)
    rng = np.random.default_rng(7)
    perm = rng.permutation(V).astype(np.int32)
    Eu, Ev = perm[Eu], perm[Ev]
    Yp = np.empty_like(Y)
    Yp[perm] = Y
    La = np.full(Eu.size, 0.1, dt)
    c = dict(solver="l1", X0=np.zeros(V, dt), Y=Yp, A=None, N=0, Eu=Eu, Ev=Ev, La_d1=La,
             La_l1=np.full(V, 0.01, dt), positivity=0, Ltype=pfdr.SCAL, L=None, rho=1.5,
             condMin=1e-3, difRcd=difRcd, difTol=1e-4, itMax=2000)
    X1, it1, D1, s1 = _session_replay(c, False, pfdr.EVOLUTION_SEQUENTIAL, pfdr.REORDER_ON)
    X0, it0, D0, s0 = _session_replay(c, False, pfdr.EVOLUTION_SEQUENTIAL, pfdr.REORDER_OFF)
    Xo, ito, _, Do = oracle.Oracle("port").quadratic_d1_l1(
        c["X0"], Yp, None, 0, Eu, Ev, La, c["La_l1"], 0, pfdr.SCAL, None, 1.5, 1e-3, difRcd,
        1e-4, 2000, dif=True)
    print("it %d / %d / %d" % (it1, it0, ito))
    assert s1 == s0 == 1
    assert it1 == it0 == ito
    assert np.array_equal(D1[:it1], Do[:ito]) and np.array_equal(D0[:it0], Do[:ito])
    assert np.array_equal(X1, Xo) and np.array_equal(X0, Xo)
