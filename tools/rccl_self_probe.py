"""Probe of the 1-rank RCCL self-call test flag (PFDR_RCCL_SELF): one
partitioned session on a 1-rank communicator, a few iterations, progress
printed before each step (run one process per flag value, each under its own
time limit)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cp_pfdr_graph_d1_amd import partition as P  # noqa: E402
from cp_pfdr_graph_d1_amd import pfdr  # noqa: E402
from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation  # noqa: E402


def main():
    lib = pfdr.load()
    shape = (128, 96)
    V = int(np.prod(shape))
    Eu, Ev = grid_graph(shape, 4)
    dt = np.float32
    print("flag", os.environ.get("PFDR_RCCL_SELF"), flush=True)
    idb = (C.c_char * 128)()
    assert lib.pfdr_comm_unique_id(idb) == 0
    comm = C.c_void_p()
    assert lib.pfdr_comm_init(C.byref(comm), 1, 0, idb) == 0, lib.pfdr_last_error()
    print("comm ok", flush=True)
    for spec in (pfdr.SPEC_OFF, pfdr.SPEC_SERIAL, pfdr.SPEC_AUTO):
        s = pfdr.Session(pfdr.PFDR_KIND_L1, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.1, dt),
                         np.zeros(V, dt), piecewise_observation(shape, 3, dt),
                         La_l1=np.full(V, 0.01, dt), difTol=1e-5, itMax=200, record_dif=True,
                         evolution=pfdr.EVOLUTION_SEQUENTIAL, nranks=1, rank=0, comm=comm.value,
                         comm_kind=P.COMM_RCCL, vtx_begin=0, V_global=V, spec=spec)
        print("session ok spec", spec, {k: s.query(k) for k in ("graphs", "speculative")},
              flush=True)
        s.run(200)
        X, it, _, _ = s.result()
        s.close()
        print("run ok it", it, float(np.abs(X).sum()), flush=True)
    lib.pfdr_comm_destroy(comm)
    print("done", flush=True)


if __name__ == "__main__":
    main()
