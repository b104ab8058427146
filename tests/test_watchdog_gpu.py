"""The partitioned path fails loudly instead of hanging (loopback transport:
k ranks as k threads on one GPU, the same session code as RCCL).

* a rank whose peer never joins: its collective times out after
  PFDR_COMM_TIMEOUT seconds and the call fails with the rank, the phase, the
  iteration and the last collective (peers, bytes);
* a rank that fails (bad input) wakes the others: solve_loopback raises that
  rank's error and returns, no thread is left waiting."""
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _graph():
    from cp_pfdr_graph_d1_amd import pfdr
    shape = (20, 16, 10)
    V = int(np.prod(shape))
    Eu, Ev = pfdr.gen_knn_jitter_grid(shape, 6, 6)
    Y = pfdr.gen_piecewise(20, V, 2, np.float32)
    return V, Eu, Ev, Y


def test_stalled_peer_times_out_with_diagnostic(gpu_lib, monkeypatch):
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    monkeypatch.setenv("PFDR_COMM_TIMEOUT", "3")
    V, Eu, Ev, Y = _graph()
    off = P.vertex_offsets(V, 2)
    e = P.split_edges(Eu, off)[0]
    lib = pfdr.load()
    import ctypes as C
    hub = C.c_void_p()
    pfdr._check(lib.pfdr_loopback_create(C.byref(hub), 2), "pfdr_loopback_create")
    err = {}

    def rank0():  # rank 1 never joins
        try:
            pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, int(off[1]), e.size, Eu[e], Ev[e],
                         np.full(e.size, 0.1, np.float32), np.zeros(int(off[1]), np.float32),
                         Y[:off[1]], nranks=2, rank=0, comm=hub.value,
                         comm_kind=P.COMM_LOOPBACK, vtx_begin=0, V_global=V, e_global=e)
        except Exception as ex:
            err["ex"] = ex

    t0 = time.time()
    th = threading.Thread(target=rank0)
    th.start()
    th.join(60)
    assert not th.is_alive(), "watchdog did not fire"
    el = time.time() - t0
    lib.pfdr_loopback_destroy(hub)
    msg = str(err.get("ex"))
    print(msg)
    assert "ex" in err and "stalled" in msg and "rank 0 of 2" in msg and "last collective" in msg
    assert 2.5 <= el < 30


def test_failing_rank_wakes_its_peers(gpu_lib, monkeypatch):
    from cp_pfdr_graph_d1_amd import partition as P
    monkeypatch.setenv("PFDR_COMM_TIMEOUT", "60")
    V, Eu, Ev, Y = _graph()
    Ev = Ev.copy()
    Ev[-1] = V + 7  # an edge of the last rank points outside the graph
    t0 = time.time()
    with pytest.raises(Exception) as ei:
        P.solve_loopback(2, 0, np.float32, Eu, Ev, np.full(Eu.size, 0.1, np.float32),
                         np.zeros(V, np.float32), Y, itMax=5)
    el = time.time() - t0
    print(ei.value)
    assert el < 30, "the healthy rank waited for the watchdog instead of being woken"


def test_rccl_abort_then_destroy_is_safe(gpu_lib, monkeypatch):
    """RCCL transport, one rank, a watchdog forced to fire (a timeout far
    below one iteration's GPU time): the library aborts the caller's
    communicator, the call fails with the diagnostic, a new session on the
    aborted handle is refused, and the owner's normal clean-up
    (pfdr_comm_destroy) returns without freeing the handle a second time"""
    import ctypes as C
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph
    lib = pfdr.load()
    idb = (C.c_char * 128)()
    assert lib.pfdr_comm_unique_id(idb) == 0
    comm = C.c_void_p()
    assert lib.pfdr_comm_init(C.byref(comm), 1, 0, idb) == 0, lib.pfdr_last_error()
    Eu, Ev = grid_graph((512, 512), 4)
    V = 512 * 512
    Y = pfdr.gen_piecewise(512, V, 2, np.float32)
    La = np.full(Eu.size, 0.1, np.float32)
    monkeypatch.setenv("PFDR_COMM_TIMEOUT", "1e-7")
    with pytest.raises(Exception) as ei:
        s = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, Eu.size, Eu, Ev, La,
                         np.zeros(V, np.float32), Y, difTol=1e-9, itMax=2000,
                         nranks=1, rank=0, comm=comm.value, comm_kind=P.COMM_RCCL,
                         vtx_begin=0, V_global=V)
        try:
            s.run(2000)
        finally:
            s.close()
    print(ei.value)
    assert "stalled" in str(ei.value)
    monkeypatch.setenv("PFDR_COMM_TIMEOUT", "60")
    with pytest.raises(Exception) as e2:
        pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, Eu.size, Eu, Ev, La,
                     np.zeros(V, np.float32), Y, itMax=5, nranks=1, rank=0, comm=comm.value,
                     comm_kind=P.COMM_RCCL, vtx_begin=0, V_global=V)
    assert "aborted" in str(e2.value)
    v = C.c_double(1.0)
    assert lib.pfdr_comm_allreduce_max_f64(comm, C.byref(v)) != 0
    assert lib.pfdr_comm_destroy(comm) == 0
