"""Time the sequential-rounding sum (pfdr_monosum.hpp, C entry
pfdr_sequential_sum_*) on synthetic term sets shaped like the iterate
evolution's two sums, and count the binade crossings that force the walk
to scan term by term.  GPU: python tools/seqsum_bench.py [n]"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cp_pfdr_graph_d1_amd import pfdr


def crossings(a):
    c = np.add.accumulate(a)  # sequential f32 rounding
    e = np.frexp(c[c > 0])[1]
    return int(np.count_nonzero(np.diff(e))) + 1, c[-1]


def cases(n, rng):
    x = rng.random(n, dtype=np.float32)
    yield "X^2 uniform", (x * x).astype(np.float32)
    yield "loguniform 1e-20..1e-6", np.exp(rng.uniform(np.log(1e-20), np.log(1e-6), n)).astype(np.float32)
    d = (1e-4 * rng.standard_normal(n)).astype(np.float32)
    yield "dif gaussian 1e-4", d * d
    m = rng.random(n) < 0.01
    z = np.zeros(n, np.float32)
    z[m] = np.exp(rng.uniform(np.log(1e-30), np.log(1e-8), int(m.sum()))).astype(np.float32)
    yield "1% nonzero loguniform 1e-30..1e-8", z
    w = np.exp(rng.uniform(np.log(1e-30), np.log(1.0), n)).astype(np.float32)
    yield "loguniform 1e-30..1", w


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    rng = np.random.default_rng(3)
    for name, a in cases(n, rng):
        k, ref = crossings(a)
        ms = []
        for _ in range(5):
            s, t = pfdr.sequential_sum(a, 0.0, 0)
            ms.append(t)
        ok = s == ref
        print("%-36s crossings %4d  walk-sum %.3f ms (min of 5)  %s"
              % (name, k, min(ms), "equal" if ok else "DIFFERS %r %r" % (s, ref)), flush=True)


if __name__ == "__main__":
    main()
