"""TEST INFRASTRUCTURE — cut-pursuit problems for the reference's four CP
drivers (oracle/harness/cp_drivers.cpp, binaries oracle/_ref/cp_<kind>_ref
and cp_<kind>_mi355x): writer of the driver's input file, reader of its
output, and the problem set of tests/test_dropin_cp.py.

Each problem is a 2-D 4-neighbour grid with a piecewise-constant truth
(three vertical bands) observed through
  * N = 0 : a diagonal A^tA (l22-style weights, Y = A^t y),
  * N > 0 : a dense N-by-V matrix (column major), Y = A x0 + noise — CP
            then solves its reduced problems both premultiplied (PFDR with
            n = -rV, rV small) and direct (PFDR with N, rV large),
            src/CP_PFDR_graph_quadratic_d1_l1.cpp:671, :848-858,
  * N < 0 : the V-by-V A^tA itself with A^t y,
  * simplex: K-class probabilities Q (src/CP_PFDR_graph_loss_d1_simplex.cpp).
"""
import os

import numpy as np

KINDS = {"l1": 0, "duplex": 1, "bounds": 2, "simplex": 3}


def _grid(nx, ny):
    from cp_pfdr_graph_d1_amd.graphs import grid_graph
    Eu, Ev = grid_graph((nx, ny), 4)
    return Eu.astype(np.int32), Ev.astype(np.int32)


def _bands(nx, ny):
    x = np.arange(nx * ny) % nx
    return np.where(x < nx // 3, 1.0, np.where(x < 2 * nx // 3, -0.5, 0.25))


def problem(kind, mode, dt, nx=48, ny=36, seed=7, **over):
    """-> dict of the driver's fields (see write())"""
    from cp_pfdr_graph_d1_amd.graphs import uniform
    V = nx * ny
    Eu, Ev = _grid(nx, ny)
    E = Eu.size
    x0 = _bands(nx, ny)
    noise = lambda n, s: (2 * uniform(seed + s, np.arange(n)) - 1)
    p = dict(kind=kind, V=V, E=E, N=0, K=0, dtype=dt, CP_itMax=8, PFDR_itMax=2000,
             positivity=0, CP_difTol=1e-4, PFDR_difTol=1e-5, rho=1.5, condMin=1e-3,
             difRcd=0.0, lo=-np.inf, hi=np.inf, al=0.0, Y=None, A=None,
             Eu=Eu, Ev=Ev, La_d1=np.full(E, 0.3, dt), La_l1=None)
    if kind == "simplex":
        K = 4
        lab = (np.arange(V) % nx) * K // nx
        Q = 0.2 * (1 + noise(K * V, 1).reshape(V, K))
        Q[np.arange(V), lab] += 1.0
        Q /= Q.sum(1, keepdims=True)
        p.update(K=K, Y=Q.astype(dt).ravel(), La_d1=np.full(E, 0.1, dt), al=0.1,
                 condMin=0.1, rho=1.0, PFDR_difTol=1e-4)
    elif mode == "diag":
        a = (0.5 + uniform(seed + 1, np.arange(V))).astype(dt)
        y = x0 + 0.4 * noise(V, 2)
        p.update(Y=(a * y).astype(dt), A=a)
    elif mode == "identity":
        p.update(Y=(x0 + 0.4 * noise(V, 2)).astype(dt), A=None)
    elif mode == "direct":  # N > 0
        N = over.pop("N", 24)
        A = (noise(N * V, 3) * np.sqrt(3.0 / N)).reshape(V, N)  # row v = column v
        Y = A.T @ x0 + 0.05 * noise(N, 4)
        p.update(N=N, Y=Y.astype(dt), A=A.astype(dt).ravel(), La_d1=np.full(E, 0.05, dt))
    elif mode == "AtA":  # N < 0
        N = 2 * V
        A = (noise(N * V, 3) * np.sqrt(3.0 / N)).reshape(V, N)
        y = A.T @ x0 + 0.05 * noise(N, 4)
        p.update(N=-V, Y=(A @ y).astype(dt), A=(A @ A.T).astype(dt).ravel(),
                 La_d1=np.full(E, 0.05, dt))
    else:
        raise ValueError(mode)
    if kind in ("l1", "duplex"):
        p["La_l1"] = np.full(V, 0.02, dt)
    if kind == "bounds":
        p.update(lo=-0.3, hi=0.8)
    p.update(over)
    return p


def write(path, p):
    dt = np.dtype(p["dtype"])
    flags = (1 if p["A"] is not None else 0) | (2 if p["La_l1"] is not None else 0)
    with open(path, "wb") as f:
        np.array([KINDS[p["kind"]], p["V"], p["E"], p["N"], p["K"],
                  1 if dt == np.float64 else 0, p["CP_itMax"], p["PFDR_itMax"],
                  p["positivity"], flags], np.int32).tofile(f)
        np.array([p["CP_difTol"], p["PFDR_difTol"], p["rho"], p["condMin"], p["difRcd"],
                  p["lo"], p["hi"], p["al"]], np.float64).tofile(f)
        np.ascontiguousarray(p["Y"], dt).tofile(f)
        if p["A"] is not None:
            np.ascontiguousarray(p["A"], dt).tofile(f)
        np.ascontiguousarray(p["Eu"], np.int32).tofile(f)
        np.ascontiguousarray(p["Ev"], np.int32).tofile(f)
        np.ascontiguousarray(p["La_d1"], dt).tofile(f)
        if p["La_l1"] is not None:
            np.ascontiguousarray(p["La_l1"], dt).tofile(f)


def read(path, p):
    """-> (rV, CP_it, Cv[V], rX[rV] or rP[K rV])"""
    dt = np.dtype(p["dtype"])
    raw = open(path, "rb").read()
    h = np.frombuffer(raw[:8], np.int32)
    V = p["V"]
    Cv = np.frombuffer(raw[8:8 + 4 * V], np.int32)
    rX = np.frombuffer(raw[8 + 4 * V:], dt)
    assert rX.size == h[0] * max(p["K"], 1)
    return int(h[0]), int(h[1]), Cv, rX


def driver(kind, provider, ref_dir):
    return os.path.join(ref_dir, "cp_%s_%s" % (kind, provider))
