"""Edge-case problems for the three PFDR solvers, in golden_io.replay's case
format: no edges, one vertex with a self-loop, isolated vertices,
zero-weight edges (the reference's 0/0 NaNs), duplicate and mirrored
edges, zero iterations, a zero-width box, K = 1 and K = 2 labels.  The
reference's own outputs on them pin the restatement (tests/test_edge_cases.py,
CPU, where oracle/_ref is built); the GPU must equal the restatement bit for
bit, NaNs included (tests/test_edge_cases_gpu.py)."""
import numpy as np

GRAPHS = {
    "no_edges": (5, [], [], []),
    "one_vertex_selfloop": (1, [0], [0], [0.1]),
    "isolated_vertices": (6, [0, 1, 2], [1, 2, 3], [0.1, 0.1, 0.1]),
    "zero_weight_edge": (4, [0, 1, 2], [1, 2, 3], [0.1, 0.0, 0.1]),
    "duplicate_edges": (4, [0, 0, 1, 2], [1, 1, 2, 3], [0.1, 0.1, 0.1, 0.1]),
    "mirrored_edges": (4, [0, 1, 1, 2], [1, 0, 2, 3], [0.1, 0.2, 0.1, 0.1]),
}


def _base(V, Eu, Ev, La, dt, itMax, difTol):
    return dict(Eu=np.asarray(Eu, np.int32), Ev=np.asarray(Ev, np.int32),
                La_d1=np.asarray(La, dt), rho=1.5, condMin=1e-3, difRcd=0.0, difTol=difTol,
                itMax=itMax)


def cases():
    out = {}
    for dt, nm in ((np.float32, "f32"), (np.float64, "f64")):
        for g, (V, Eu, Ev, La) in GRAPHS.items():
            Y = np.linspace(-1, 1, V).astype(dt) if V > 1 else np.array([0.7], dt)
            for itMax, difTol, tag in ((0, 0.0, "it0"), (1, 0.0, "it1"), (40, 1e-4, "conv")):
                b = _base(V, Eu, Ev, La, dt, itMax, difTol)
                out["l1_%s_%s_%s" % (g, tag, nm)] = dict(
                    b, solver="l1", X0=np.zeros(V, dt), Y=Y, A=None, N=0,
                    La_l1=np.full(V, 0.05, dt), positivity=0, Ltype=0, L=None)
                out["bounds_%s_%s_%s" % (g, tag, nm)] = dict(
                    b, solver="bounds", X0=np.zeros(V, dt), Y=Y, A=None, N=0, lo=-0.3, hi=0.4,
                    Ltype=0, L=None)
                for K in (1, 2, 3):
                    rng = np.random.default_rng(K + V)
                    Q = rng.random((V, K))
                    Q = (Q / Q.sum(axis=1, keepdims=True)).reshape(-1).astype(dt)
                    out["simplex_K%d_%s_%s_%s" % (K, g, tag, nm)] = dict(
                        b, solver="simplex", K=K, P0=Q.copy(), Q=Q, al=0.1, La_f=None)
        # a zero-width box and the unbounded box on a path graph
        V = 8
        Eu, Ev = list(range(7)), list(range(1, 8))
        b = _base(V, Eu, Ev, [0.1] * 7, dt, 30, 0.0)
        Y = np.linspace(-1, 1, V).astype(dt)
        for lo, hi, tag in ((0.25, 0.25, "zero_width_box"), (-np.inf, np.inf, "no_bounds"),
                            (-np.inf, 0.1, "upper_only")):
            out["bounds_path_%s_%s" % (tag, nm)] = dict(
                b, solver="bounds", X0=np.zeros(V, dt), Y=Y, A=None, N=0, lo=lo, hi=hi,
                Ltype=0, L=None)
    return out


def same(a, b, exact_dif=False):
    """outputs of golden_io.replay (X, it, Obj, Dif): X and it bit-equal,
    NaNs equal; Dif (the stopping statistic, tree-reduced on the GPU, a
    sequential sum in the reference: DESIGN §2) to the parity tests'
    tolerance, 1e-4 (f32) / 1e-9 (f64) relative, or bit-equal"""
    Xa, ita, Oa, Da = a
    Xb, itb, Ob, Db = b
    eq = lambda x, y: np.array_equal(np.asarray(x), np.asarray(y), equal_nan=True)
    if ita != itb or not eq(Xa, Xb):
        return False
    Da, Db = np.asarray(Da)[:ita], np.asarray(Db)[:itb]
    if exact_dif or eq(Da, Db):
        return eq(Da, Db)
    tol = 1e-4 if np.asarray(Xa).dtype == np.float32 else 1e-9
    d = np.abs(Da.astype(np.float64) - Db.astype(np.float64))
    return bool(np.all(np.isnan(Da) == np.isnan(Db)) and
                np.all(d[~np.isnan(d)] <= tol * np.maximum(np.abs(Db[~np.isnan(d)]), 1e-30)))
