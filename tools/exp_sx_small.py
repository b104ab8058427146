"""Small simplex problems (cut pursuit's reduced ones): microseconds per
iteration of PFDR_graph_loss_d1_simplex sessions on 8-neighbour grids, K = 4
smoothed KL, f32 / f64, difTol tiny (runs to itMax), with and without the
hipGraph replay of iteration chunks (PFDR_GRAPH = 1 / 0) or the fused
loop decision (PFDR_FUSE).  Usage: python tools/exp_sx_small.py [KNOB]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from cp_pfdr_graph_d1_amd import pfdr  # noqa: E402
from cp_pfdr_graph_d1_amd.graphs import grid_graph  # noqa: E402


KNOB = sys.argv[1] if len(sys.argv) > 1 else "PFDR_GRAPH"  # or PFDR_SX_TINY
ON = sys.argv[2] if len(sys.argv) > 2 else "1"  # the knob's "on" value


def us_per_it(shape, dt, graph, K=4, it=1000):
    os.environ[KNOB] = graph
    Eu, Ev = grid_graph(shape, 8)
    V = int(np.prod(shape))
    rng = np.random.default_rng(V)
    Q = rng.random((V, K))
    Q = (Q / Q.sum(axis=1, keepdims=True)).reshape(-1).astype(dt)
    s = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.05, dt),
                     Q.copy(), Q, K=K, al=0.1, rho=1.0, condMin=0.1, difRcd=0.0, difTol=1e-12,
                     itMax=it + 100)
    try:
        s.run(100)
        torch.cuda.synchronize()
        t = time.perf_counter()
        s.run(it)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / it * 1e6
    finally:
        s.close()


torch.cuda.init()
for dt in (np.float32, np.float64):
    for shape in ((8, 8), (16, 16), (24, 24), (32, 32), (40, 40), (64, 64), (100, 100)):
        r = {g: [us_per_it(shape, dt, g) for _ in range(2)] for g in (ON, "0")}
        print("%-4s %-8s %s on %7.2f %7.2f   off %7.2f %7.2f us/it" % (
            np.dtype(dt).name[5:], "%dx%d" % shape, KNOB, *r[ON], *r["0"]), flush=True)
