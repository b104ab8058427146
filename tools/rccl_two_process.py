"""Experiment: the RCCL transport with two processes (torchrun, gloo for the
unique id), both ranks on cuda:0 -- the only way to run the multi-process
RCCL path on a one-GPU box.  RCCL may refuse two ranks on one device; then
this prints the refusal and exits 3.  Otherwise each rank solves its slab of
a jittered 6-NN grid through the RCCL halo and rank 0 compares the gathered
iterate with the single-GPU session (must be bit-identical).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 tools/rccl_two_process.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)

    def bcast(t):  # uint8 CPU tensor, broadcast through gloo
        dist.broadcast(t, 0)

    shape = (40, 30, 32)
    V = int(np.prod(shape))
    Eu, Ev = pfdr.gen_knn_jitter_grid(shape, 6, 6)
    Y = pfdr.gen_piecewise(40, V, 2, np.float32)
    La = np.full(Eu.size, 0.1, np.float32)
    L1 = np.full(V, 0.01, np.float32)
    X0 = np.zeros(V, np.float32)
    off = P.vertex_offsets(V, world)
    e = P.split_edges(Eu, off)[rank]
    v0, v1 = int(off[rank]), int(off[rank + 1])
    try:
        comm = P.comm_init(world, rank, bcast)
    except Exception as ex:
        print(json.dumps({"rank": rank, "rccl_init": "refused", "error": str(ex)[:300]}), flush=True)
        sys.exit(3)
    s = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, v1 - v0, e.size, Eu[e], Ev[e], La[e],
                     X0[v0:v1], Y[v0:v1], La_l1=L1[v0:v1], difTol=1e-5, itMax=300,
                     record_dif=True, nranks=world, rank=rank, comm=comm,
                     comm_kind=P.COMM_RCCL, vtx_begin=v0, V_global=V, e_global=e)
    s.run(300)
    Xr, it, _, _ = s.result()
    s.close()
    parts = [None] * world
    dist.all_gather_object(parts, (rank, Xr.tolist(), it))
    if rank == 0:
        parts.sort()
        X = np.concatenate([np.asarray(p[1], np.float32) for p in parts])
        its = {p[2] for p in parts}
        ss = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, Eu.size, Eu, Ev, La, X0, Y, La_l1=L1,
                          difTol=1e-5, itMax=300, record_dif=True)
        ss.run(300)
        Xs, its1, _, _ = ss.result()
        ss.close()
        ok = its == {its1} and np.array_equal(X, Xs)
        print(json.dumps({"ranks": world, "iterations": sorted(its), "single_gpu_iterations": its1,
                          "bit_identical": bool(np.array_equal(X, Xs)), "ok": bool(ok)}), flush=True)
        if not ok:
            sys.exit(1)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
