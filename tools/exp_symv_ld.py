"""Experiment: does the power-of-two column stride of A^tA (V = 32,768 ->
128 KB between columns) cost the upper-triangle product bandwidth?  Times
the symmetric product (session kernel stats "symv") for V around 32,768 on
random exactly symmetric matrices.

    python tools/exp_symv_ld.py [--sizes 32768 32704 32832]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[32768, 32704, 32832])
    ap.add_argument("--its", type=int, default=30)
    args = ap.parse_args()
    import torch
    from cp_pfdr_graph_d1_amd import pfdr
    for V in args.sizes:
        g = torch.Generator(device="cuda")
        g.manual_seed(V)
        B = torch.rand((V, V), generator=g, device="cuda") - 0.5
        A = (B + B.t()) * 0.5
        del B
        nx = 64
        Eu, Ev = pfdr.gen_grid_edges((nx, V // nx), 4)
        E = Eu.size
        dev = lambda a, t=torch.float32: torch.as_tensor(a, dtype=t, device="cuda")
        Y = torch.rand(V, generator=g, device="cuda")
        L = torch.tensor([float(V)], device="cuda")
        s = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, E, dev(Eu, torch.int32), dev(Ev, torch.int32),
                         torch.full((E,), 0.05, device="cuda"), torch.zeros(V, device="cuda"), Y,
                         N=-V, A=A, La_l1=torch.full((V,), 0.005, device="cuda"), L=L,
                         itMax=args.its + 5, device=True)
        s.run(5)
        s.profile(True)
        s.run(args.its)
        n, ms = s.kernel_stats("symv")
        sym = s.query("symv")
        s.close()
        nb = (V + 127) // 128
        tile_bytes = nb * (nb + 1) // 2 * 128 * 128 * 4
        print(json.dumps({"V": V, "symv_path": sym, "launches": n, "symv_ms": round(ms, 4),
                          "tile_bytes": tile_bytes, "TBps": round(tile_bytes / (ms * 1e-3) / 1e12, 3)}),
              flush=True)
        del A
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
