"""CPU: the per-rank inputs bench.py builds for N > 1 (tools/workloads.py) are
slabs of ONE global problem: concatenated over the ranks they equal the
global generation, and each rank's vtx_begin / e_offset are the global ids of
its first vertex and first edge.  (That the partitioned solve of such slabs
equals the single-GPU solve is tests/test_partition_gpu.py's and
test_fullsize_gpu.py's job.)"""
import os
import sys

import numpy as np
import pytest

from cp_pfdr_graph_d1_amd import pfdr

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import workloads  # noqa: E402


class SmallHeadline(workloads.Headline):
    SHAPE = (9, 8, 5)


@pytest.mark.parametrize("world", [2, 3])
def test_headline_weak_slabs_form_the_global_graph(world):
    ranks = [SmallHeadline().inputs(r, world, strong=False) for r in range(world)]
    nx, ny, nz = SmallHeadline.SHAPE

    class Global(workloads.Headline):
        SHAPE = (nx, ny, nz * world)
    g = Global().inputs(0, 1, strong=False)
    V, E = g["V"], g["E"]
    assert sum(d["V"] for d in ranks) == V and sum(d["E"] for d in ranks) == E
    v0 = e0 = 0
    for d in ranks:
        assert d["vtx_begin"] == v0 and d["e_offset"] == e0
        v0 += d["V"]
        e0 += d["E"]
        assert np.all((d["kw"]["Eu"] >= d["vtx_begin"]) & (d["kw"]["Eu"] < v0))  # owner = Eu
    for key in ("Eu", "Ev", "Y", "La_d1", "La_l1", "X0"):
        assert np.array_equal(np.concatenate([d["kw"][key] for d in ranks]), g["kw"][key]), key


@pytest.mark.parametrize("shape,conn", [((7, 6, 9), 6), ((11, 12), 8), ((5, 4, 6), 26)])
def test_grid_slabs_and_edge_offsets(shape, conn):
    """the C2 / C4 / C5 slabs: edges of a vertex range and the number of
    edges emitted before it"""
    Eu, Ev = pfdr.gen_grid_edges(shape, conn)
    V = int(np.prod(shape))
    cuts = [0, V // 4, V // 2, V - 3, V]
    for a, b in zip(cuts[:-1], cuts[1:]):
        su, sv = pfdr.gen_grid_edges(shape, conn, (a, b))
        e0 = pfdr.grid_edge_count(shape, conn, a)
        assert e0 == int(np.count_nonzero(Eu < a))
        assert np.array_equal(su, Eu[e0:e0 + su.size]) and np.array_equal(sv, Ev[e0:e0 + su.size])
        assert np.all((su >= a) & (su < b))


def test_piecewise_observation_slabs():
    full = pfdr.gen_piecewise(10, 600, 5, np.float32, 0.2)
    parts = [pfdr.gen_piecewise(10, 600, 5, np.float32, 0.2, (a, b))
             for a, b in ((0, 250), (250, 251), (251, 600))]
    assert np.array_equal(np.concatenate(parts), full)


def _check_strong(wl, world, g):
    """the strong split: the ranks' slabs concatenate to the single-GPU inputs"""
    ranks = [wl.inputs(r, world, strong=True) for r in range(world)]
    assert sum(d["V"] for d in ranks) == g["V"] and sum(d["E"] for d in ranks) == g["E"]
    v0 = e0 = 0
    for d in ranks:
        assert d["vtx_begin"] == v0 and d["e_offset"] == e0
        v0 += d["V"]
        e0 += d["E"]
        assert np.all((d["kw"]["Eu"] >= d["vtx_begin"]) & (d["kw"]["Eu"] < v0))
    for key in ("Eu", "Ev", "Y", "La_d1", "X0"):
        assert np.array_equal(np.concatenate([d["kw"][key] for d in ranks]), g["kw"][key]), key
    return ranks


@pytest.mark.parametrize("world", [2, 3, 8])
def test_headline_strong_slabs_split_the_global_graph(world):
    _check_strong(SmallHeadline(), world, SmallHeadline().inputs(0, 1))


def test_headline_strong_split_full_size():
    """bench.py --gpus 8 (default strong scaling): eight z-slabs of the
    fixed 10M-vertex / 60M-edge graph, 1.25M vertices each"""
    wl = workloads.Headline()
    g = wl.inputs(0, 1)
    assert (g["V"], g["E"]) == (10_000_000, 60_000_000)
    ranks = _check_strong(wl, 8, g)
    assert {d["V"] for d in ranks} == {1_250_000}


def _gloo_worker(rank, world, port, out):
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import torch.distributed as dist
    import workloads as W

    class Small(W.Headline):
        SHAPE = (9, 8, 7)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=world)
    try:
        d = Small().inputs(rank, world, strong=True)
        t = torch.tensor([d["V"], d["E"], d["vtx_begin"], d["e_offset"]], dtype=torch.int64)
        allt = [torch.zeros(4, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allt, t)
        out[rank] = [x.tolist() for x in allt]
    finally:
        dist.destroy_process_group()


def test_strong_slabs_over_gloo():
    """world_size 2 over gloo (as bench.py's ranks): every rank builds its own
    slab; gathered, the slabs tile the vertices and the edge list"""
    import socket
    import torch.multiprocessing as mp
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_gloo_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)

    class Small(workloads.Headline):
        SHAPE = (9, 8, 7)
    g = Small().inputs(0, 1)
    for r in range(world):
        rows = res[r]
        assert sum(x[0] for x in rows) == g["V"] and sum(x[1] for x in rows) == g["E"]
        assert [x[2] for x in rows] == [0, rows[0][0]]
        assert [x[3] for x in rows] == [0, rows[0][1]]
