"""GPU: the split incidence of the vertex sweep (csrc/pfdr_quadratic_kernels.hpp
split_sum) and the u-staged edge sweep (k_edge_sweep_us).  When the edges
are sorted by their u end, each vertex's u-end contributions are a
contiguous run and only the other entries are gathered; a per-vertex code
keeps the reference's (e, side) summation order.  Blocks that do not
qualify (hubs, unsorted edges) keep the CSR gather.  Every path must equal
the restatement of the reference (oracle) bit for bit: iterates, iteration
counts and Dif (the sessions here sum the evolution sequentially, like the
reference, so reconditioning and stopping decisions are the reference's)."""
import numpy as np
import pytest

from cp_pfdr_graph_d1_amd import pfdr
from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation, uniform

pytestmark = pytest.mark.gpu


def _solve(V, Eu, Ev, Y, dt, it, reorder=pfdr.REORDER_OFF, difRcd=0.0, difTol=0.0):
    s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
                     np.zeros(V, dt), Y, La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3,
                     itMax=it, reorder=reorder, difRcd=difRcd, difTol=difTol, record_dif=True,
                     evolution=pfdr.EVOLUTION_SEQUENTIAL)
    try:
        nsplit = s.query("split_blocks")
        s.run(it)
        X, its, _, Dif = s.result()
    finally:
        s.close()
    return X, its, Dif, nsplit


def _oracle(oracle_port, V, Eu, Ev, Y, dt, it, difRcd=0.0, difTol=0.0):
    return oracle_port.quadratic_d1_l1(np.zeros(V, dt), Y, None, 0, Eu, Ev,
                                       np.full(Eu.size, 0.1, dt), np.full(V, 0.01, dt), 0, 0,
                                       None, 1.5, 1e-3, difRcd, difTol, it, dif=True)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_split_natural_grid_matches_oracle(gpu_lib, oracle_port, dt):
    """3-D 6-neighbour grid in emission order: every block takes the split
    path; with reconditioning and a tolerance, iterates, iteration count and
    Dif equal the restatement's"""
    shape = (48, 40, 24)
    Eu, Ev = grid_graph(shape, 6)
    Eu, Ev = Eu.astype(np.int32), Ev.astype(np.int32)
    V = int(np.prod(shape))
    Y = piecewise_observation(shape, 3, dt)
    kw = dict(difRcd=1e-1, difTol=1e-5)
    Xs, its, Ds, ns = _solve(V, Eu, Ev, Y, dt, 400, **kw)
    Xo, ito, _, Do = _oracle(oracle_port, V, Eu, Ev, Y, dt, 400, **kw)
    assert ns == (V + 255) // 256
    assert its == ito
    assert np.array_equal(Xs, Xo)
    assert np.array_equal(Ds[:its], Do[:ito])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_split_mixed_blocks_with_hubs(gpu_lib, oracle_port, dt):
    """A 2-D grid plus hub vertices of degree > 32 and zero-out-degree runs:
    the hubs' blocks fall back to the CSR gather, the others split; results
    equal the oracle bit for bit at a fixed k."""
    shape = (96, 80)
    V = int(np.prod(shape))
    Eu0, Ev0 = grid_graph(shape, 8)
    rng_t = uniform(5, np.arange(4000))
    hubs = np.array([17, 3000, 3001, 7000], np.int64)
    extra_u = np.repeat(hubs, 40)
    extra_v = (rng_t[: extra_u.size] * V).astype(np.int64)
    extra_v[extra_v == extra_u] += 1
    Eu = np.concatenate([Eu0.astype(np.int64), extra_u])
    Ev = np.concatenate([Ev0.astype(np.int64), extra_v % V])
    # drop the out-edges of a band of vertices (a zero out-degree run longer
    # than the edge sweep's staged u span: those blocks read Eu)
    keep = ~((Eu >= 5000) & (Eu < 6500))
    Eu, Ev = Eu[keep], Ev[keep]
    order = np.argsort(Eu, kind="stable")
    Eu, Ev = Eu[order].astype(np.int32), Ev[order].astype(np.int32)
    Y = piecewise_observation(shape, 4, dt)
    k = 25
    Xs, _, _, ns = _solve(V, Eu, Ev, Y, dt, k)
    nb = (V + 255) // 256
    assert 0 < ns < nb
    Xo, ito, _, _ = _oracle(oracle_port, V, Eu, Ev, Y, dt, k)
    assert ito == k
    assert np.array_equal(Xs, Xo)


def test_split_unsorted_edges_keep_the_gather(gpu_lib, oracle_port):
    """Edges out of u order: no split blocks, the CSR gather and the Eu
    stream everywhere (the summation order is the edge order); equal to the
    oracle bit for bit"""
    shape = (64, 64)
    Eu, Ev = grid_graph(shape, 4)
    V = int(np.prod(shape))
    p = np.argsort(uniform(9, np.arange(Eu.size)), kind="stable")
    Eu, Ev = Eu[p].astype(np.int32), Ev[p].astype(np.int32)
    Y = piecewise_observation(shape, 6, np.float32)
    Xs, _, _, ns = _solve(V, Eu, Ev, Y, np.float32, 10)
    Xo, _, _, _ = _oracle(oracle_port, V, Eu, Ev, Y, np.float32, 10)
    assert ns == 0
    assert np.array_equal(Xs, Xo)


def test_relabelled_large_graph_equals_plain_solve(gpu_lib):
    """Randomly labelled grid (V >= 2^20): the relabelled session renumbers
    its vertices and, being large, takes the tile order (no split blocks:
    test_tiled_gpu.py covers that path), and stays bit-identical to the
    plain solve in the caller's labels."""
    shape = (128, 128, 64)
    Eu, Ev = grid_graph(shape, 6)
    V = int(np.prod(shape))
    new_of = np.empty(V, np.int64)
    new_of[np.argsort(uniform(11, np.arange(V)), kind="stable")] = np.arange(V)
    Eu, Ev = new_of[Eu].astype(np.int32), new_of[Ev].astype(np.int32)
    Y = piecewise_observation(shape, 7, np.float32)
    Xs, _, _, ns = _solve(V, Eu, Ev, Y, np.float32, 12, reorder=pfdr.REORDER_ON)
    Xg, _, _, ng = _solve(V, Eu, Ev, Y, np.float32, 12, reorder=pfdr.REORDER_OFF)
    assert ns == 0 and ng == 0
    assert np.array_equal(Xs, Xg)
