"""Kernel time of the amplitude sum: workgroup binade scan vs one lane."""
import numpy as np

from cp_pfdr_graph_d1_amd import pfdr

rng = np.random.default_rng(1)
for dt in (np.float32, np.float64):
    for n in (1 << 20, 10_000_000):
        a = np.abs(rng.normal(0, 1, n)).astype(dt)
        r = {}
        for m in (0, 1):
            best = min(pfdr.sequential_sum(a, 0.0, m)[1] for _ in range(3))
            r[m] = (pfdr.sequential_sum(a, 0.0, m)[0], best)
        assert r[0][0] == r[1][0] == np.cumsum(a)[-1]
        print("%s n=%d  scan %.3f ms  lane %.3f ms  (x%.1f)" % (
            np.dtype(dt).name, n, r[0][1], r[1][1], r[1][1] / r[0][1]), flush=True)
