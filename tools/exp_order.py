"""Experiment: how much does the vertex order of the headline graph matter
for the iteration (gather locality of the edge and vertex sweeps)?

Relabels the headline graph on the host with orders computed from its grid
coordinates (an upper bound for what a graph-only locality order could
reach), sorts the edges by their new u end, and times the iteration.

    python tools/exp_order.py [--orders natural tile8 tile16 morton]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def morton3(x, y, z, bits=10):
    code = np.zeros(x.shape, np.uint64)
    for b in range(bits):
        for i, c in enumerate((x, y, z)):
            code |= ((c.astype(np.uint64) >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b + i)
    return code


def order_keys(name, nx, ny, nz):
    v = np.arange(nx * ny * nz, dtype=np.int64)
    x, y, z = v % nx, (v // nx) % ny, v // (nx * ny)
    if name == "natural":
        return v
    if name.startswith("tile"):
        T = int(name[4:])
        return ((((z // T) * ((ny + T - 1) // T) + y // T) * ((nx + T - 1) // T) + x // T)
                * T ** 3 + ((z % T) * T + y % T) * T + x % T)
    if name == "morton":
        return morton3(x, y, z).astype(np.int64)
    if name.startswith("slab"):  # xy tiles of T x T, all z inside a tile column
        T = int(name[4:])
        return (((y // T) * ((nx + T - 1) // T) + x // T) * nz + z) * T * T + (y % T) * T + x % T
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--orders", nargs="+", default=["natural", "tile8", "tile16", "morton"])
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    import torch
    from cp_pfdr_graph_d1_amd import pfdr
    nx, ny, nz = 250, 200, 200
    V = nx * ny * nz
    Eu0, Ev0 = pfdr.gen_knn_jitter_grid((nx, ny, nz), 6, 6, 0.25)
    Y0 = pfdr.gen_piecewise(nx, V, 2, np.float32, 0.2)
    E = Eu0.size
    torch.cuda.set_device(0)
    for name in args.orders:
        t = time.perf_counter()
        key = order_keys(name, nx, ny, nz)
        inv = np.argsort(key, kind="stable")          # new position -> old vertex
        new = np.empty(V, np.int32)
        new[inv] = np.arange(V, dtype=np.int32)       # old vertex -> new id
        Eu, Ev = new[Eu0], new[Ev0]
        perm = np.argsort(Eu, kind="stable")
        Eu, Ev = Eu[perm], Ev[perm]
        Y = Y0[inv]
        prep = time.perf_counter() - t
        sess = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, E, Eu=Eu, Ev=Ev,
                            La_d1=np.full(E, 0.1, np.float32), X0=np.zeros(V, np.float32), Y=Y,
                            La_l1=np.full(V, 0.01, np.float32), rho=1.5, condMin=1e-3,
                            itMax=5 + args.steps, reorder=pfdr.REORDER_OFF)
        sess.run(5)
        sess.profile(True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        sess.run(args.steps)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        st = {k: round(sess.kernel_stats(k)[1], 4) for k in ("edge_sweep", "vertex_sweep")}
        sess.close()
        print(json.dumps({"order": name, "ms_per_iter": round(el / args.steps * 1e3, 4),
                          "kernels_ms": st, "prep_s": round(prep, 1)}), flush=True)


if __name__ == "__main__":
    main()
