"""A/B of the per-block contribution lists of fused (small) sessions
(PFDR_PAD = 1 / 0): microseconds per iteration of l1 sessions on 4-NN grids
across the fused range, f32 and f64, difTol tiny (runs to itMax), graph
replay on.  Usage: python tools/exp_pad.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402  (device init before timing)
from cp_pfdr_graph_d1_amd import pfdr  # noqa: E402
from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation  # noqa: E402


KNOB = sys.argv[1] if len(sys.argv) > 1 else "PFDR_PAD"  # or PFDR_PAD_ENDS


def us_per_it(shape, dt, pad, it=2000):
    os.environ[KNOB] = pad  # "1": on whatever the size
    Eu, Ev = grid_graph(shape, 4)
    V = int(np.prod(shape))
    Y = piecewise_observation(shape, 1, dt)
    s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
                     np.zeros(V, dt), Y, La_l1=np.full(V, 0.01, dt), rho=1.5, condMin=1e-3,
                     difRcd=0.0, difTol=1e-30, itMax=it + 200)
    try:
        if KNOB == "PFDR_PAD":
            assert s.query("padded") == (1 if pad == "1" else 0), s.query("padded")
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
    for shape in ((48, 48), (256, 256), (360, 360), (400, 400), (512, 512)):
        r = {p: [us_per_it(shape, dt, p) for _ in range(2)] for p in ("1", "0")}
        print("%-4s %-10s pad %6.2f %6.2f   gathered %6.2f %6.2f us/it" % (
            np.dtype(dt).name[5:], "%dx%d" % shape, *r["1"], *r["0"]), KNOB, flush=True)
