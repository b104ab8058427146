"""GPU: small single-GPU graphs take the loop decision on iteration t inside
the edge sweep of iteration t + 1 (FuseDecide, pfdr_quadratic_kernels.hpp):
every workgroup repeats k_reduce_decide's loop and tree on the vertex
sweep's partials, the decisions alternate between two control blocks, and
the chunk closes with one k_decide_fused launch.  Fused sessions of at most
512 vertex blocks, each holding at most 4096 CSR entries, also store their
contributions in per-block lists (k_vertex_sweep_pad; a block past that cap
keeps the gathered sweep), and in f32 stream the endpoint data as per-edge
copies (k_edge_sweep_ends).

Checked against the reference and against the multi-launch loop:
  * every graph-mode golden case through the fused path (the one-workgroup
    path off, PFDR_TINY=0): iterates bit-exact at fixed k, Dif within the
    tree / sequential bound, converged iteration counts within 2 and
    bit-exact iterates when they agree;
  * grids across the fused range (16 to 1024 vertex blocks, just past it:
    not fused), stopping at a tolerance, at itMax inside a chunk, after
    reconditionings, with the run split into calls of odd and even lengths
    (partial chunks launched, whole ones replayed as hipGraphs): the fused
    session against the multi-launch loop with the reference's sequential
    evolution sums (PFDR_EVOLUTION_SEQUENTIAL) -- the same iterates bit for
    bit whenever the two decisions agree, which the tree's accuracy makes
    the rule (their Dif values agree to the tree/sequential bound)."""
import os

import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

QUAD = [n for n in G.names() if n.startswith(("l1_", "bounds_"))
        and "direct" not in n and "AtA" not in n]


class _env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("name", QUAD)
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
def test_fused_golden_matches_reference(gpu_lib, name, fixed):
    c, g = G.load(name)
    with _env(PFDR_TINY="0"):
        X, it, _, D = G.replay(gpu_lib, c, fixed, obj=False, dif=True)
    tag = "fixk" if fixed else "conv"
    gX, git, gD = g[tag + "_X"], int(g[tag + "_it"]), g[tag + "_Dif"]
    n = min(it, git)
    assert G.rel_l2(D[:n], gD[:n]) <= (1e-4 if X.dtype == np.float32 else 1e-9)
    if fixed:
        assert it == git
    assert abs(it - git) <= 2
    if it == git:
        assert np.array_equal(X, gX)


def _session(pfdr, shape, dt, kind, diag, itMax, difTol, difRcd, evolution=0):
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    Eu, Ev = grid_graph(shape, 4)
    V = int(np.prod(shape))
    Y = piecewise_observation(shape, 1, dt)
    rng = np.random.default_rng(V)
    A = (0.5 + rng.random(V)).astype(dt) if diag else None
    kw = dict(A=A, rho=1.5, condMin=1e-3, difRcd=difRcd, difTol=difTol, itMax=itMax,
              record_dif=True, evolution=evolution)
    if kind == "l1":
        return pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
                            np.zeros(V, dt), Y, La_l1=np.full(V, 0.01, dt), **kw)
    return pfdr.Session(pfdr.PFDR_KIND_BOUNDS, dt, V, Eu.size, Eu, Ev,
                        np.full(Eu.size, 0.1, dt), np.zeros(V, dt), Y, lo=0.1, hi=0.7, **kw)


CASES = [  # shape, dtype, kind, diagonal A, itMax, difTol, difRcd, run() lengths
    ((64, 64), np.float32, "l1", False, 3000, 1e-5, 1e-2, (3000,)),
    ((256, 256), np.float64, "l1", True, 3000, 1e-6, 0.0, (3000,)),      # C1's shape
    ((256, 256), np.float32, "bounds", False, 70, 0.0, 1e-1, (70,)),     # itMax inside a chunk
    ((200, 300), np.float64, "l1", False, 500, 1e-7, 1e-1, (7, 33, 1, 64, 500)),
    ((512, 512), np.float32, "l1", False, 200, 1e-9, 1e-2, (31, 200)),  # 1024 blocks
    ((513, 512), np.float32, "l1", False, 40, 1e-9, 0.0, (40,)),        # past the fused range
]


def _agree(fused, seq, dt):
    """fused (tree-summed decisions) against the multi-launch loop with the
    sequential sums: equal iterates when the iteration counts agree"""
    (X0, it0, _, D0), (X1, it1, _, D1) = fused, seq
    n = min(it0, it1)
    assert G.rel_l2(D0[:n], D1[:n]) <= (1e-4 if dt == np.float32 else 1e-9)
    assert abs(it0 - it1) <= 1
    if it0 == it1:
        assert np.array_equal(X0, X1)
    return it0 == it1


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%dx%d-%s-%s%s" % (
    c[0][0], c[0][1], np.dtype(c[1]).name, c[2], "-diag" if c[3] else ""))
def test_fused_sessions_match_multilaunch(gpu_lib, case):
    from cp_pfdr_graph_d1_amd import pfdr
    shape, dt, kind, diag, itMax, difTol, difRcd, runs = case
    V = int(np.prod(shape))
    nb = (V + 255) // 256
    res = []
    for evo in (pfdr.EVOLUTION_AUTO, pfdr.EVOLUTION_SEQUENTIAL):
        with _env(PFDR_TINY="0"):
            s = _session(pfdr, shape, dt, kind, diag, itMax, difTol, difRcd, evo)
        try:
            fused = evo == pfdr.EVOLUTION_AUTO and nb <= 1024
            assert s.query("fused") == (1 if fused else 0)
            assert s.query("padded") == (1 if fused and nb <= 512 else 0)  # kPadBlocks
            for n in runs:
                s.run(n)
            res.append(s.result())
        finally:
            s.close()
    assert 0 < res[0][1] <= itMax
    assert _agree(res[0], res[1], dt), "decisions differ on this case: pick another"


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_padded_cap(gpu_lib, dt):
    """A vertex block past the per-block list cap (a hub with 5000 incident
    edges) keeps the gathered vertex sweep; smaller graphs of the same law
    are padded.  Both equal the multi-launch loop bit for bit."""
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    for hub in (5000, 1000):
        Eu, Ev = grid_graph((96, 96), 4)
        V = 96 * 96
        extra = np.arange(1, hub + 1, dtype=np.int32) * 7 % V
        extra[extra == 0] = 1
        Eu = np.concatenate([np.zeros(hub, np.int32), Eu.astype(np.int32)])
        Ev = np.concatenate([extra, Ev.astype(np.int32)])
        Y = piecewise_observation((96, 96), 1, dt)
        res = []
        for evo in (pfdr.EVOLUTION_AUTO, pfdr.EVOLUTION_SEQUENTIAL):
            with _env(PFDR_TINY="0"):
                s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev,
                                 np.full(Eu.size, 0.1, dt), np.zeros(V, dt), Y,
                                 La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3,
                                 difRcd=1e-2, difTol=1e-6, itMax=600, record_dif=True,
                                 evolution=evo)
            try:
                if evo == pfdr.EVOLUTION_AUTO:
                    assert s.query("fused") == 1
                    assert s.query("padded") == (0 if hub > 4096 else 1)
                s.run(600)
                res.append(s.result())
            finally:
                s.close()
        assert 0 < res[0][1]
        assert _agree(res[0], res[1], dt), "decisions differ on this case: pick another"
