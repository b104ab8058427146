"""GPU: small single-GPU graphs take the loop decision on iteration t inside
the edge sweep of iteration t + 1 (FuseDecide, pfdr_quadratic_kernels.hpp;
PFDR_FUSE = 0 off): every workgroup repeats k_reduce_decide's loop and tree
on the vertex sweep's partials, the decisions alternate between two control
blocks, and the chunk closes with one k_decide_fused launch.  Iterates,
iteration counts and the evolution record must be identical bit for bit to
the three-launch loop -- and, for f64 at a fixed iteration count, to the
reference's golden iterates -- on every graph-mode golden case (fixed-k and
converged, reconditioning where the case has it) and on grids across the
fused range (16 to 1024 vertex blocks, just past it: not fused), stopping
at a tolerance, at itMax inside a chunk, after reconditionings, with the
run split into calls of odd and even lengths, with and without hipGraph
replay.  Fused sessions of at most 512 vertex blocks, each holding at most
4096 CSR entries, also store their contributions in per-block lists
(k_vertex_sweep_pad; PFDR_PAD = 0 off, 1 on across the fused range):
identical as well, and a block past that cap keeps the gathered sweep; with
the endpoint data streamed as per-edge copies (k_edge_sweep_ends; f32 up to
512 blocks by default, PFDR_PAD_ENDS = 0 off, 1 on for every padded session)
as well."""
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
def test_fused_golden_identical(gpu_lib, name, fixed):
    c, g = G.load(name)
    res = []
    for env in ({"PFDR_TINY": "0", "PFDR_FUSE": "1"}, {"PFDR_TINY": "0", "PFDR_FUSE": "0"},
                {"PFDR_TINY": "0", "PFDR_FUSE": "1", "PFDR_GRAPH": "0"},
                {"PFDR_TINY": "0", "PFDR_FUSE": "1", "PFDR_PAD": "0"},
                {"PFDR_TINY": "0", "PFDR_FUSE": "1", "PFDR_PAD_ENDS": "0"},
                {"PFDR_TINY": "0", "PFDR_FUSE": "1", "PFDR_PAD_ENDS": "1"}):
        with _env(**env):
            res.append(G.replay(gpu_lib, c, fixed, obj=False, dif=True))
    X0, it0, _, D0 = res[0]
    for X1, it1, _, D1 in res[1:]:
        assert it1 == it0
        assert np.array_equal(X1, X0)
        assert np.array_equal(D1[:it1], D0[:it0])
    if fixed and X0.dtype == np.float64:
        assert np.array_equal(X0, g["fixk_X"])


def _session(pfdr, shape, dt, kind, diag, itMax, difTol, difRcd):
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    Eu, Ev = grid_graph(shape, 4)
    V = int(np.prod(shape))
    Y = piecewise_observation(shape, 1, dt)
    rng = np.random.default_rng(V)
    A = (0.5 + rng.random(V)).astype(dt) if diag else None
    kw = dict(A=A, rho=1.5, condMin=1e-3, difRcd=difRcd, difTol=difTol, itMax=itMax,
              record_dif=True)
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


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%dx%d-%s-%s%s" % (
    c[0][0], c[0][1], np.dtype(c[1]).name, c[2], "-diag" if c[3] else ""))
def test_fused_sessions_identical(gpu_lib, case):
    from cp_pfdr_graph_d1_amd import pfdr
    shape, dt, kind, diag, itMax, difTol, difRcd, runs = case
    V = int(np.prod(shape))
    fusable = (V + 255) // 256 <= 1024
    res = []
    for env in ({"PFDR_FUSE": "1"}, {"PFDR_FUSE": "0"}, {"PFDR_FUSE": "1", "PFDR_GRAPH": "0"},
                {"PFDR_FUSE": "1", "PFDR_PAD": "0"}, {"PFDR_FUSE": "1", "PFDR_PAD": "1"},
                {"PFDR_FUSE": "1", "PFDR_PAD_ENDS": "0"},
                {"PFDR_FUSE": "1", "PFDR_PAD": "1", "PFDR_PAD_ENDS": "1"}):
        with _env(PFDR_TINY="0", **env):
            s = _session(pfdr, shape, dt, kind, diag, itMax, difTol, difRcd)
        try:
            fused = fusable and env["PFDR_FUSE"] == "1"
            assert s.query("fused") == (1 if fused else 0)
            pad = env.get("PFDR_PAD", "1" if (V + 255) // 256 <= 512 else "0")  # kPadBlocks
            assert s.query("padded") == (1 if fused and pad == "1" else 0)
            for n in runs:
                s.run(n)
            res.append(s.result())
        finally:
            s.close()
    X0, it0, _, D0 = res[0]
    assert 0 < it0 <= itMax
    for X1, it1, _, D1 in res[1:]:
        assert it1 == it0
        assert np.array_equal(X1, X0)
        assert np.array_equal(D1[:it1], D0[:it0])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_padded_cap(gpu_lib, dt):
    """A vertex block past the per-block list cap (a hub with 5000 incident
    edges) keeps the gathered vertex sweep; smaller graphs of the same law
    are padded.  Both equal the unfused three-launch loop bit for bit."""
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
        for env in ({"PFDR_FUSE": "1"}, {"PFDR_FUSE": "0"}):
            with _env(PFDR_TINY="0", **env):
                s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev,
                                 np.full(Eu.size, 0.1, dt), np.zeros(V, dt), Y,
                                 La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3,
                                 difRcd=1e-2, difTol=1e-6, itMax=600, record_dif=True)
            try:
                if env["PFDR_FUSE"] == "1":
                    assert s.query("fused") == 1
                    assert s.query("padded") == (0 if hub > 4096 else 1)
                s.run(600)
                res.append(s.result())
            finally:
                s.close()
        (X0, it0, _, D0), (X1, it1, _, D1) = res
        assert it0 == it1 and 0 < it0
        assert np.array_equal(X0, X1)
        assert np.array_equal(D0[:it0], D1[:it1])
