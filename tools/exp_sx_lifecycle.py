"""Where a CP-sized simplex PFDR call spends its time outside the
iterations: session create / run / result copy-out / close, in ms, for
grid sizes like cut pursuit's reduced simplex problems (copy_ms
~1.3 ms a call), with and without the chunk graph (PFDR_GRAPH).
Usage: python tools/exp_sx_lifecycle.py [SHAPES]   (e.g. 60x60,120x120;
other knobs, e.g. PFDR_SX_NT=64, from the environment)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from cp_pfdr_graph_d1_amd import pfdr  # noqa: E402
from cp_pfdr_graph_d1_amd.graphs import grid_graph  # noqa: E402


def phases(shape, graph, K=4, it=223, dt=np.float32):
    os.environ["PFDR_GRAPH"] = graph
    Eu, Ev = grid_graph(shape, 4)
    V = int(np.prod(shape))
    rng = np.random.default_rng(V)
    Q = rng.random((V, K))
    Q = (Q / Q.sum(axis=1, keepdims=True)).reshape(-1).astype(dt)
    La = np.full(Eu.size, 0.05, dt)
    t0 = time.perf_counter()
    s = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev, La, Q.copy(), Q, K=K,
                     al=0.1, rho=1.0, condMin=0.1, difRcd=0.0, difTol=1e-12, itMax=it)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    s.run(it)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    s.result()
    t3 = time.perf_counter()
    s.close()
    t4 = time.perf_counter()
    return [1e3 * (b - a) for a, b in ((t0, t1), (t1, t2), (t2, t3), (t3, t4))]


torch.cuda.init()
phases((16, 16), "1")
SHAPES = sys.argv[1] if len(sys.argv) > 1 else "120x120,240x240"
for shape in [tuple(int(n) for n in t.split("x")) for t in SHAPES.split(",")]:
    for g in ("1", "0"):
        for rep in range(3):
            c, r, o, d = phases(shape, g)
            print("%-8s graph=%s create %7.3f run %7.3f result %6.3f close %6.3f ms" % (
                "%dx%d" % shape, g, c, r, o, d), flush=True)
