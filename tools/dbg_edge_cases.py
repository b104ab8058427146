import sys, numpy as np
sys.path[:0] = ['.', 'oracle', 'tests', 'tests/golden']
import edge_cases as EC, golden_io as G, oracle
from cp_pfdr_graph_d1_amd import pfdr
lib = pfdr.Lib(); o = oracle.Oracle("port")
C = EC.cases()
bad = []
for name in sorted(C):
    a = G.replay(lib, C[name], False, obj=False, dif=True)
    b = G.replay(o, C[name], False, obj=False, dif=True)
    if not EC.same(a, b):
        bad.append(name)
        if len(bad) <= 6:
            print(name, "it", a[1], b[1])
            print("  X gpu", a[0].view(np.uint32 if a[0].dtype==np.float32 else np.uint64)[:8])
            print("  X ora", b[0].view(np.uint32 if b[0].dtype==np.float32 else np.uint64)[:8])
            print("  Dif gpu", np.asarray(a[3])[:a[1]])
            print("  Dif ora", np.asarray(b[3])[:b[1]])
print("bad", len(bad), "of", len(C)); print(bad)
