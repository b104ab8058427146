"""One-workgroup iterations (k_tiny_iterate) against the two-launch loop:
microseconds per iteration of l1 sessions on 4-NN grids of 1 to 32 vertex
blocks, f32 and f64, difTol tiny (runs to itMax).  PFDR_TINY = edge limit
(0: off); above 8 blocks the limit also lifts the block cap to 32.
Usage: python tools/exp_tiny.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from cp_pfdr_graph_d1_amd import pfdr  # noqa: E402
from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation  # noqa: E402


def us_per_it(shape, dt, tiny, it=2000):
    os.environ["PFDR_TINY"] = tiny
    Eu, Ev = grid_graph(shape, 4)
    V = int(np.prod(shape))
    Y = piecewise_observation(shape, 1, dt)
    s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
                     np.zeros(V, dt), Y, La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3,
                     difRcd=0.0, difTol=1e-30, itMax=it + 200)
    try:
        assert s.query("tiny") == (1 if tiny != "0" else 0), (shape, tiny)
        s.run(200)
        torch.cuda.synchronize()
        t = time.perf_counter()
        s.run(it)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / it * 1e6
    finally:
        s.close()


torch.cuda.init()
for dt in (np.float32, np.float64):
    for shape in ((16, 16), (32, 32), (45, 45), (64, 64), (90, 90)):
        r = {p: [us_per_it(shape, dt, p) for _ in range(2)] for p in ("100000", "0")}
        print("%-4s %-8s %3d blocks  tiny %6.2f %6.2f   launches %6.2f %6.2f us/it" % (
            np.dtype(dt).name[5:], "%dx%d" % shape, (shape[0] * shape[1] + 255) // 256,
            *r["100000"], *r["0"]), flush=True)
