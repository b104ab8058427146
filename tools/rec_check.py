"""Headline X after 20 iterations, single GPU and 2 loopback ranks, saved to
gpurun_out/<tag>_{single,k2}.npy: an A/B of two library builds
(PFDR_LIB_PATH) on the same inputs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from workloads import WORKLOADS  # noqa: E402
from cp_pfdr_graph_d1_amd import pfdr, partition as P  # noqa: E402

tag = sys.argv[1]
wl = WORKLOADS["headline"]
inp = wl.inputs(0, 1)
kw = inp["kw"]
s = pfdr.Session(wl.kind, wl.dtype, inp["V"], inp["E"], itMax=20, **kw)
s.run(20)
X = s.result()[0]
print(tag, "single: tiled", s.query("tiled_blocks"), "record", s.query("record_blocks"))
s.close()
np.save("gpurun_out/%s_single.npy" % tag, X)
r = P.solve_loopback(2, wl.kind, wl.dtype, kw["Eu"], kw["Ev"], kw["La_d1"], kw["X0"], kw["Y"],
                     La_l1=kw.get("La_l1"), rho=kw["rho"], condMin=kw["condMin"], itMax=20)
print(tag, "k2 queries", r[4]["queries"])
np.save("gpurun_out/%s_k2.npy" % tag, r[0])
