"""Host-side timeline between the session setup and the first iteration
(the GPU idles there and its clock drops): ctor, input release, graph
capture, first iterations."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402,F401
from workloads import WORKLOADS  # noqa: E402
from cp_pfdr_graph_d1_amd import pfdr  # noqa: E402

wl = WORKLOADS["headline"]
inp = wl.inputs(0, 1)
T = [("start", time.perf_counter())]
s = pfdr.Session(wl.kind, wl.dtype, inp["V"], inp["E"], itMax=100, **inp["kw"])
T.append(("ctor", time.perf_counter()))
del inp
T.append(("del inputs", time.perf_counter()))
s.profile(False)
s.prepare(20)
T.append(("prepare(20)", time.perf_counter()))
s.run(5)
s.sync()
T.append(("run(5)+sync", time.perf_counter()))
for (a, ta), (b, tb) in zip(T, T[1:]):
    print("%-14s %8.2f ms" % (b, (tb - ta) * 1e3))
