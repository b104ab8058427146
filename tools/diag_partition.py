import sys, os, numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
from workloads import WORKLOADS
from cp_pfdr_graph_d1_amd import pfdr, partition as P
wl = WORKLOADS["headline"]; inp = wl.inputs(0, 1); kw = inp["kw"]; ITS = int(sys.argv[1]) if len(sys.argv) > 1 else 12
def single():
    s = pfdr.Session(wl.kind, wl.dtype, inp["V"], inp["E"], itMax=ITS, **kw); s.run(ITS); X = s.result()[0]; s.close(); return X
def part(k):
    r = P.solve_loopback(k, wl.kind, wl.dtype, kw["Eu"], kw["Ev"], kw["La_d1"], kw["X0"], kw["Y"],
                         La_l1=kw.get("La_l1"), rho=kw["rho"], condMin=kw["condMin"], itMax=ITS)
    return r[0], r[4]
X1 = single(); X1b = single()
print("single vs single: ndiff", int((X1 != X1b).sum()))
V = X1.size
for t in range(3):
    X2, info = part(2)
    d = X2 != X1
    idx = np.nonzero(d)[0]
    print("part2 run %d: ndiff %d maxabs %.3e first %s last %s off %s q %s" % (t, d.sum(), np.abs(X2 - X1).max() if d.any() else 0,
          idx[:5], idx[-5:], info["off"], info["queries"]))
