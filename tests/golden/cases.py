"""Input recipes of the golden fixtures (shared by make_golden.py and tests).

Each case is a dict with a ``solver`` in {"l1", "bounds", "simplex", "proj"}
plus the solver arguments as numpy arrays / scalars.  Sizes are chosen so the
single-threaded oracle finishes each in well under a second.

The values mirror the reference's own usage:
* l22 cases follow octave/mex/PFDR_graph_l22_d1_l1_mex.cpp:54-64 (Y <- La_l2*Y,
  N = 0, A = La_l2, Ltype DIAG, L = La_l2);
* AtA cases follow octave/mex/PFDR_graph_quadratic_d1_l1_AtA_mex.cpp:53 (N = -V);
* simplex cases follow octave/mex/PFDR_graph_loss_d1_simplex_mex.cpp:33,46
  (P0 = Q, La_f = NULL) and the CP caller (La_f = component sizes,
  src/CP_PFDR_graph_loss_d1_simplex.cpp:764).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from cp_pfdr_graph_d1_amd.graphs import (grid_graph, knn_jitter_grid,  # noqa: E402
                                        piecewise_observation,
                                        simplex_observation, uniform)


def _l1_base(dt, shape, conn, seed, la_d1=0.1, la_l1=0.01):
    Eu, Ev = grid_graph(shape, conn)
    V = int(np.prod(shape))
    return dict(solver="l1", X0=np.zeros(V, dt),
                Y=piecewise_observation(shape, seed, dt), A=None, N=0,
                Eu=Eu, Ev=Ev, La_d1=np.full(Eu.size, la_d1, dt),
                La_l1=np.full(V, la_l1, dt), positivity=0, Ltype=0, L=None,
                rho=1.5, condMin=1e-3, difRcd=0.0, difTol=1e-6, itMax=3000)


def _dense(dt, shape, N, seed):
    """Compressed-sensing style A ~ U(-.5,.5)/sqrt(N)*sqrt(12) col-major N x V,
    observation of a 3-block signal."""
    V = int(np.prod(shape))
    A = ((uniform(seed, np.arange(N * V)) - 0.5) * np.sqrt(12.0 / N))
    A = A.reshape(V, N)  # row v = column v of the column-major N x V matrix
    x = np.zeros(V)
    x[: V // 3] = 1.0
    x[V // 3: 2 * V // 3] = -0.5
    y = A.T @ x
    L = np.linalg.norm(A, 2) ** 2
    return A, y, L


def make_cases():
    cases = {}
    # --- KAT: 1-D chain, closed form [1.1, 1.6, -0.6, 2.9]
    for dt, nm in ((np.float64, "f64"), (np.float32, "f32")):
        cases["l1_chain_kat_" + nm] = dict(
            solver="l1", X0=np.zeros(4, dt), Y=np.array([1, 2, -1, 3], dt),
            A=None, N=0, Eu=np.array([0, 1, 2], np.int32),
            Ev=np.array([1, 2, 3], np.int32),
            La_d1=np.array([0.1, 0.3, 0.1], dt), La_l1=None, positivity=0,
            Ltype=0, L=None, rho=1.5, condMin=1e-3, difRcd=0.0, difTol=1e-8,
            itMax=1000)
    # --- identity A (config C1 shape, reduced): 2-D 4-NN
    for dt, nm in ((np.float64, "f64"), (np.float32, "f32")):
        c = _l1_base(dt, (32, 32), 4, 1)
        cases["l1_grid2d_" + nm] = c
    c = _l1_base(np.float32, (10, 10, 10), 6, 2)
    c.update(positivity=1, difTol=1e-5)
    cases["l1_grid3d_pos_f32"] = c
    c = _l1_base(np.float32, (24, 24), 8, 3)
    c.update(La_l1=None, difRcd=1e-3, difTol=1e-6)
    cases["l1_grid2d8_recond_f32"] = c
    c = _l1_base(np.float64, (24, 24), 4, 4)
    c.update(difRcd=1e-2, difTol=1e-7, condMin=1e-2)
    cases["l1_grid2d_recond_f64"] = c
    # --- l22 (diagonal A) semantics
    for dt, nm in ((np.float64, "f64"), (np.float32, "f32")):
        c = _l1_base(dt, (20, 30), 4, 5)
        V = 600
        la_l2 = (0.5 + uniform(11, np.arange(V))).astype(dt)
        c.update(Y=(la_l2 * c["Y"]).astype(dt), A=la_l2, Ltype=1, L=la_l2)
        cases["l1_l22_" + nm] = c
    # --- headline-style k-NN jittered grid, random relabelling
    Eu, Ev = knn_jitter_grid((8, 8, 8), 6, seed=6)
    perm = np.argsort(uniform(7, np.arange(512)), kind="stable").astype(np.int32)
    inv = np.empty_like(perm)
    inv[perm] = np.arange(512, dtype=np.int32)
    eperm = np.argsort(uniform(8, np.arange(Eu.size)), kind="stable")
    Eu, Ev = inv[Eu][eperm], inv[Ev][eperm]
    Y = piecewise_observation((8, 8, 8), 9, np.float32)[perm]
    cases["l1_knn_shuffled_f32"] = dict(
        solver="l1", X0=np.zeros(512, np.float32), Y=Y, A=None, N=0,
        Eu=Eu.astype(np.int32), Ev=Ev.astype(np.int32),
        La_d1=np.full(Eu.size, 0.1, np.float32),
        La_l1=np.full(512, 0.01, np.float32), positivity=0, Ltype=0, L=None,
        rho=1.5, condMin=1e-3, difRcd=0.0, difTol=1e-5, itMax=3000)
    # --- direct A (N > 0) and precomputed A^tA (N < 0)
    for dt, nm in ((np.float32, "f32"), (np.float64, "f64")):
        A, y, L = _dense(dt, (16, 16), 64, 3)
        Eu, Ev = grid_graph((16, 16), 4)
        base = dict(solver="l1", X0=np.zeros(256, dt), Eu=Eu, Ev=Ev,
                    La_d1=np.full(Eu.size, 0.05, dt),
                    La_l1=np.full(256, 0.005, dt), positivity=0, Ltype=0,
                    L=np.array([L], dt), rho=1.5, condMin=1e-3, difRcd=0.0,
                    difTol=1e-6, itMax=2000)
        c = dict(base, Y=y.astype(dt), A=A.ravel().astype(dt), N=64)
        cases["l1_direct_" + nm] = c
        AtA = (A @ A.T).astype(dt)
        AtY = (A @ y).astype(dt)
        c = dict(base, Y=AtY, A=AtA.ravel(), N=-256, positivity=1)
        cases["l1_AtA_" + nm] = c
    # --- bounds
    for dt, nm in ((np.float32, "f32"), (np.float64, "f64")):
        b = _l1_base(dt, (12, 12, 6), 6, 5)
        c = dict(solver="bounds", X0=b["X0"], Y=b["Y"], A=None, N=0,
                 Eu=b["Eu"], Ev=b["Ev"], La_d1=b["La_d1"], lo=0.0, hi=1.0,
                 Ltype=0, L=None, rho=1.5, condMin=1e-3, difRcd=0.0,
                 difTol=1e-6, itMax=3000)
        cases["bounds_box_" + nm] = c
    b = cases["bounds_box_f32"]
    cases["bounds_lower_f32"] = dict(b, lo=0.0, hi=float("inf"))
    cases["bounds_upper_recond_f32"] = dict(b, lo=-float("inf"), hi=0.5,
                                            difRcd=1e-3)
    d = cases["l1_AtA_f64"]
    cases["bounds_AtA_f64"] = dict(
        solver="bounds", X0=d["X0"], Y=d["Y"], A=d["A"], N=d["N"], Eu=d["Eu"],
        Ev=d["Ev"], La_d1=d["La_d1"], lo=-0.25, hi=0.75, Ltype=0, L=d["L"],
        rho=1.5, condMin=1e-3, difRcd=0.0, difTol=1e-6, itMax=2000)
    # --- simplex (config C4 shape, reduced): K labels, 8-neighbour grid
    shape, K = (20, 20), 10
    Eu, Ev = grid_graph(shape, 8)
    V = 400
    v = np.arange(V)
    lab = (v % 20 >= 10).astype(int) + 2 * (v // 20 >= 10) + 4 * ((v % 20) < 4)
    for dt, nm in ((np.float32, "f32"), (np.float64, "f64")):
        Q = simplex_observation(V, K, 4, lab, dt)
        base = dict(solver="simplex", K=K, P0=Q.copy(), Q=Q, Eu=Eu, Ev=Ev,
                    La_d1=np.full(Eu.size, 0.05, dt), La_f=None, al=0.1,
                    rho=1.0, condMin=0.1, difRcd=0.0, difTol=1e-4,
                    itMax=2000)
        cases["simplex_kl_" + nm] = base
        cases["simplex_linear_" + nm] = dict(base, al=0.0, difTol=1e-5)
        laf = (1.0 + np.floor(4 * uniform(12, v))).astype(dt)
        cases["simplex_quad_laf_" + nm] = dict(base, al=1.0, La_f=laf,
                                             difRcd=1e-2)
        cases["simplex_kl_laf_recond_" + nm] = dict(base, La_f=laf,
                                                  difRcd=1e-2, difTol=1e-5)
        cases["simplex_labels_" + nm] = dict(base, al=0.5, difTol=1.0,
                                           difRcd=8.0,
                                           P0=np.full(V * K, 1.0 / K, dt))
    # --- edge cases of the graph as CP builds it: self-loops (CP links every
    # isolated component to itself with weight eps,
    # src/CP_PFDR_graph_quadratic_d1_l1.cpp:642-645) and repeated edges
    # (reduced edges may repeat pairs; the headline graph keeps mirrored
    # duplicates)
    Eu = np.array([0, 0, 1, 2, 2, 3, 4, 5, 5, 6, 7], np.int32)
    Ev = np.array([1, 0, 2, 3, 3, 4, 5, 6, 5, 7, 7], np.int32)
    V = 8
    for dt, nm in ((np.float64, "f64"), (np.float32, "f32")):
        eps = np.finfo(dt).eps
        La = np.array([0.2, eps, 0.3, 0.1, 0.15, 0.25, 0.2, 0.05, eps, 0.3, eps], dt)
        Y = (np.array([1.0, 1.2, -0.5, 0.3, 2.0, 2.1, -1.0, 0.4]) * 1.5).astype(dt)
        cases["l1_selfloops_" + nm] = dict(
            solver="l1", X0=np.zeros(V, dt), Y=Y, A=None, N=0, Eu=Eu, Ev=Ev,
            La_d1=La, La_l1=np.full(V, 0.05, dt), positivity=0, Ltype=0, L=None,
            rho=1.5, condMin=1e-3, difRcd=1e-2, difTol=1e-7, itMax=5000)
        cases["bounds_selfloops_" + nm] = dict(
            solver="bounds", X0=np.zeros(V, dt), Y=Y, A=None, N=0, Eu=Eu, Ev=Ev,
            La_d1=La, lo=-0.5, hi=1.5, Ltype=0, L=None, rho=1.5, condMin=1e-3,
            difRcd=0.0, difTol=1e-7, itMax=5000)
        # one component: CP's reduced problem of a constant solution
        cases["l1_one_vertex_" + nm] = dict(
            solver="l1", X0=np.zeros(1, dt), Y=np.array([0.7], dt), A=None, N=0,
            Eu=np.array([0], np.int32), Ev=np.array([0], np.int32),
            La_d1=np.array([eps], dt), La_l1=np.array([0.1], dt), positivity=1,
            Ltype=0, L=None, rho=1.5, condMin=1e-3, difRcd=0.0, difTol=1e-8,
            itMax=500)
        Ks = 3
        Qs = simplex_observation(V, Ks, 21, np.arange(V) % Ks, dt)
        cases["simplex_selfloops_" + nm] = dict(
            solver="simplex", K=Ks, P0=Qs.copy(), Q=Qs, Eu=Eu, Ev=Ev, La_d1=La,
            La_f=(1.0 + np.arange(V) % 3).astype(dt), al=0.2, rho=1.0, condMin=0.1,
            difRcd=0.0, difTol=1e-6, itMax=3000)
    # --- standalone metric simplex projection (D = 7, nm < N, na < N)
    for dt, nm in ((np.float32, "f32"), (np.float64, "f64")):
        D, N = 7, 300
        X = (3.0 * uniform(13, np.arange(D * N)) - 1.0).astype(dt)
        M = (0.1 + uniform(14, np.arange(D * 200))).astype(dt)
        Asum = (0.5 + uniform(15, np.arange(120))).astype(dt)
        cases["proj_simplex_" + nm] = dict(solver="proj", X=X, M=M, D=D, N=N,
                                           nm=200, A=Asum, na=120)
    cases.update(make_wide_cases())
    return cases


def _grid_labels(shape, K):
    """block labels of a 2-D grid: quadrants, a left band, spread over K"""
    nx, ny = shape
    v = np.arange(nx * ny)
    lab = (v % nx >= nx // 2).astype(int) + 2 * (v // nx >= ny // 2) + 4 * ((v % nx) < nx // 5)
    return (lab * max(1, K // 7) + v // (2 * nx)) % K


def make_wide_cases():
    """Round 5: the simplex and the metric projection beyond K = 10 / D = 7
    (every label count the K-generic code paths take: the fused vertex
    sweep's upper range K <= 64, odd K with stored prox weights, the
    wave-per-vertex path from K = 65, and K, D > 1024 with the active set
    outside registers).  The reference handles any K (alloca(D),
    src/proj_simplex_metric.cpp:38, called with D = K from
    src/PFDR_graph_loss_d1_simplex.cpp:651)."""
    cases = {}
    # (K, grid, loss variants) -- sizes keep V*K <= ~30K so the reference's
    # single-threaded converged run finishes in about a second
    plan = [
        (16, (12, 12), [("kl", {})]),
        (33, (10, 10), [("quad_laf_recond", dict(al=1.0, laf=True, difRcd=1e-2))]),
        (63, (8, 8), [("linear", dict(al=0.0, difTol=1e-5))]),
        (64, (8, 8), [("kl_recond", dict(difRcd=1e-2, difTol=1e-5))]),
        (65, (8, 8), [("kl", {}), ("labels", dict(al=0.5, difTol=1.0, difRcd=8.0, uniform0=True))]),
        (128, (8, 6), [("quad_laf", dict(al=1.0, laf=True)), ("linear", dict(al=0.0, difTol=1e-5))]),
        (1024, (4, 4), [("kl", {})]),
        (1500, (5, 4), [("kl_laf_recond", dict(laf=True, difRcd=1e-2, difTol=1e-5)),
                        ("linear", dict(al=0.0, difTol=1e-5))]),
    ]
    for K, shape, variants in plan:
        Eu, Ev = grid_graph(shape, 8)
        V = int(np.prod(shape))
        v = np.arange(V)
        lab = _grid_labels(shape, K)
        for tag, opt in variants:
            dts = ((np.float32, "f32"), (np.float64, "f64"))
            if tag in ("labels",) or (K == 128 and tag == "linear"):
                dts = ((np.float32, "f32"),)
            for dt, nm in dts:
                Q = simplex_observation(V, K, 40 + K, lab, dt)
                laf = (1.0 + np.floor(4 * uniform(41 + K, v))).astype(dt)
                c = dict(solver="simplex", K=K, P0=Q.copy(), Q=Q, Eu=Eu, Ev=Ev,
                         La_d1=np.full(Eu.size, 0.05, dt), La_f=None, al=0.1,
                         rho=1.0, condMin=0.1, difRcd=0.0, difTol=1e-4,
                         itMax=2000)
                for k in ("al", "difRcd", "difTol"):
                    if k in opt:
                        c[k] = opt[k]
                if opt.get("laf"):
                    c["La_f"] = laf
                if opt.get("uniform0"):
                    c["P0"] = np.full(V * K, 1.0 / K, dt)
                cases["simplex_k%d_%s_%s" % (K, tag, nm)] = c
    # metric projection: one segment of G lanes per column (D <= 64), J
    # registers per lane (D <= 1024), the active set in scratch (D > 1024);
    # nm, na < N as in proj_simplex_D7
    for D, N, nm, na in ((16, 90, 70, 33), (33, 80, 50, 21), (64, 60, 41, 17), (65, 60, 41, 17),
                         (1024, 40, 30, 17), (2000, 30, 22, 9)):
        for dt, tnm in ((np.float32, "f32"), (np.float64, "f64")):
            X = (3.0 * uniform(50 + D, np.arange(D * N)) - 1.0).astype(dt)
            M = (0.1 + uniform(51 + D, np.arange(D * nm))).astype(dt)
            Asum = (0.5 + uniform(52 + D, np.arange(na))).astype(dt)
            cases["proj_simplex_D%d_%s" % (D, tnm)] = dict(solver="proj", X=X, M=M, D=D, N=N,
                                                          nm=nm, A=Asum, na=na)
    # adversarial order: ascending columns (every coordinate enters the
    # first pass, most leave again in the second) and a column of equal values
    for D in (200, 1500):
        N = 6
        X = np.concatenate([np.sort(uniform(60 + D + n, np.arange(D)) * (n + 1)) for n in range(N - 1)]
                           + [np.full(D, 0.25)])
        M = (0.5 + uniform(61 + D, np.arange(D))).astype(np.float64)
        cases["proj_simplex_sorted_D%d_f64" % D] = dict(solver="proj", X=X, M=M, D=D, N=N,
                                                      nm=1, A=np.ones(1), na=1)
    return cases


FIXED_K = 25  # iterations of the "fixed k" record (difTol = difRcd = 0)
