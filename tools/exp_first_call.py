"""Where the first drop-in call's time goes: HIP start-up, code-object
loading, first-touch allocations.  Times (wall) the library load, the first
HIP call (pfdr_device_count), then three identical small
PFDR_graph_quadratic_d1_l1<float> calls (64x64 grid, 70 iterations).

    python tools/exp_first_call.py            (one JSON line)
Run it with HIP_ENABLE_DEFERRED_LOADING=0 to load every code object at HIP
start-up instead of at each module's first launch."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    t = {}
    t0 = time.perf_counter()
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    lib = pfdr.Lib()
    t["load_lib_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    n = pfdr.load().pfdr_device_count()
    t["first_hip_call_s"] = time.perf_counter() - t0
    shape = (64, 64)
    Eu, Ev = grid_graph(shape, 4)
    V = 64 * 64
    Y = piecewise_observation(shape, 1, np.float32)
    La = np.full(Eu.size, 0.1, np.float32)
    L1 = np.full(V, 0.01, np.float32)
    calls = []
    for _ in range(3):
        t0 = time.perf_counter()
        lib.quadratic_d1_l1(np.zeros(V, np.float32), Y, None, 0, Eu, Ev, La, L1, 0, 0, None,
                            1.5, 1e-3, 0.0, 0.0, 70)
        calls.append(time.perf_counter() - t0)
    t["calls_s"] = calls
    t["devices"] = n
    t["deferred_loading"] = os.environ.get("HIP_ENABLE_DEFERRED_LOADING", "default")
    print(json.dumps(t))


if __name__ == "__main__":
    main()
