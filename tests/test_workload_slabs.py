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
    ranks = [SmallHeadline().inputs(r, world) for r in range(world)]
    nx, ny, nz = SmallHeadline.SHAPE

    class Global(workloads.Headline):
        SHAPE = (nx, ny, nz * world)
    g = Global().inputs(0, 1)
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
