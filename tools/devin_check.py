"""Session on device-resident inputs vs host arrays: X after 12 iterations
must be identical (bench.py hands the session device inputs by default)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
from workloads import WORKLOADS  # noqa: E402
from cp_pfdr_graph_d1_amd import pfdr  # noqa: E402

for name in sys.argv[1:]:
    wl = WORKLOADS[name]
    inp = wl.inputs(0, 1)
    kw = inp["kw"]
    its = 12
    s = pfdr.Session(wl.kind, wl.dtype, inp["V"], inp["E"], itMax=its, **kw)
    s.run(its)
    Xh = s.result()[0]
    s.close()
    dkw = dict(kw, device=True)
    for k in ("Eu", "Ev", "La_d1", "X0", "Y", "La_l1", "A", "L"):
        a = kw.get(k)
        if a is not None:
            a = np.ascontiguousarray(a, np.int32 if k in ("Eu", "Ev") else wl.dtype)
            dkw[k] = torch.from_numpy(a).cuda()
    torch.cuda.synchronize()
    s = pfdr.Session(wl.kind, wl.dtype, inp["V"], inp["E"], itMax=its, **dkw)
    s.run(its)
    Xd = s.result()[0]
    s.close()
    print(name, "identical" if np.array_equal(Xh, Xd) else "DIFFER (%d)" % int((Xh != Xd).sum()),
          flush=True)
    assert np.array_equal(Xh, Xd)
