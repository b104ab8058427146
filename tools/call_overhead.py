"""Per-call cost of the host-pointer drop-in (the view of a cut-pursuit
caller): repeated PFDR_graph_quadratic_d1_l1<float> calls on small grids,
with the library's own trace (PFDR_TRACE=1: setup / iterate / copy-back per
call on stderr) and the wall time around each call.

    python tools/call_overhead.py [--sizes 16 64 256] [--calls 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[16, 64, 256, 1024])
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--its", type=int, default=70)
    args = ap.parse_args()
    os.environ.setdefault("PFDR_TRACE", "1")
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    lib = pfdr.Lib()
    t_load = time.perf_counter()
    n_dev = lib.lib.pfdr_device_count()
    print(json.dumps({"device_count": n_dev, "first_hip_call_s": round(time.perf_counter() - t_load, 4)}),
          flush=True)
    for n in args.sizes:
        shape = (n, n)
        Eu, Ev = grid_graph(shape, 4)
        V = n * n
        Y = piecewise_observation(shape, 1, np.float32)
        for c in range(args.calls):
            t = time.perf_counter()
            X, it, _, _ = lib.quadratic_d1_l1(np.zeros(V, np.float32), Y, None, 0, Eu, Ev,
                                              np.full(Eu.size, 0.1, np.float32),
                                              np.full(V, 0.01, np.float32), 0, pfdr.DIAG, None,
                                              1.5, 1e-3, 0.0, 0.0, args.its)
            el = time.perf_counter() - t
            print(json.dumps({"V": V, "E": int(Eu.size), "call": c, "it": it,
                              "wall_ms": round(el * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
