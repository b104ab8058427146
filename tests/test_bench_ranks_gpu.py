"""GPU: a rehearsal, on one GPU, of the driver's multi-GPU bench run
(`torch.distributed.run ... bench.py --gpus N`).  Every rank's inputs come
from bench.py's own workload classes (tools/workloads.py, `inputs(rank,
world, strong)`), and every rank's session is created with bench.py's own
arguments (nranks, rank, vtx_begin, e_offset -- no explicit global edge
ids, no V_global); only the transport differs: the ranks are threads on this
GPU exchanging through the loopback hub instead of processes over RCCL (two
RCCL ranks cannot share one GPU).  The gathered iterate after a fixed number
of iterations must equal, bit for bit, the single-GPU session of the same
global graph -- strong scaling at N = 2, 3 and 8 (the headline, C2, C5, and
the simplex C4 with K-wide halos, the randomly labelled headline split in
its locality order) and weak scaling at N = 3 (the stacked headline) -- at
reduced grid sizes."""
import os
import sys
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import workloads  # noqa: E402


class Headline(workloads.Headline):
    SHAPE = (30, 24, 16)


class HeadlineShuffled(workloads.HeadlineShuffled):
    SHAPE = (30, 24, 16)


class C2(workloads.C2):
    SHAPE = (20, 18, 24)


class C4(workloads.C4):
    SIDE = 48


class C5(workloads.C5):
    SHAPE = (22, 20, 16)


STEPS = 25


def _session(wl, inp, **extra):
    from cp_pfdr_graph_d1_amd import pfdr
    return pfdr.Session(wl.kind, wl.dtype, inp["V"], inp["E"], itMax=STEPS, **inp["kw"], **extra)


def _single(wl, world_for_graph, strong):
    """the single-GPU session of the graph the N ranks share"""
    if strong:
        inp = wl.inputs(0, 1, True)
    else:  # the N-times taller graph of weak scaling, as one problem
        class Tall(type(wl)):
            SHAPE = (wl.SHAPE[0], wl.SHAPE[1], wl.SHAPE[2] * world_for_graph)
        inp = Tall().inputs(0, 1, True)
    s = _session(wl, inp)
    s.run(STEPS)
    X, it, _, _ = s.result()
    s.close()
    return X, it


def _ranks(wl, world, strong):
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    import ctypes as C
    lib = pfdr.load()
    inps = [wl.inputs(r, world, strong) for r in range(world)]
    hub = C.c_void_p()
    pfdr._check(lib.pfdr_loopback_create(C.byref(hub), C.c_int(world)), "pfdr_loopback_create")
    res, err = [None] * world, [None] * world

    def main(r):
        try:
            inp = inps[r]
            s = _session(wl, inp, nranks=world, rank=r, comm=hub.value,
                         comm_kind=P.COMM_LOOPBACK, vtx_begin=inp["vtx_begin"],
                         e_offset=inp["e_offset"], e_global=inp.get("e_global"),
                         vtx_label=inp.get("vtx_label"))
            s.run(STEPS)
            res[r] = s.result()
            s.close()
        except Exception as ex:
            err[r] = ex
            lib.pfdr_loopback_abort(hub, ("rank %d: %s" % (r, ex))[:200].encode())

    th = [threading.Thread(target=main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    lib.pfdr_loopback_destroy(hub)
    for ex in [e for e in err if e is not None and "aborted" not in str(e)] or \
            [e for e in err if e is not None]:
        raise ex
    assert {r[1] for r in res} == {STEPS}
    assert sum(i["E"] for i in inps) == sum(len(i["kw"]["Eu"]) for i in inps)
    X = np.concatenate([r[0] for r in res])
    if inps[0].get("vtx_label") is not None:  # a relabelled split: back to the caller's labels
        lab = np.concatenate([i["vtx_label"] for i in inps])
        Xc = np.empty_like(X)
        Xc[lab] = X
        X = Xc
    return X


CASES = [(Headline(), 2, True), (Headline(), 3, True), (Headline(), 8, True),
         (Headline(), 3, False), (C2(), 8, True), (C5(), 8, True), (C4(), 3, True),
         (C4(), 8, True), (HeadlineShuffled(), 3, True), (HeadlineShuffled(), 8, True)]


@pytest.mark.parametrize("wl,world,strong", CASES,
                         ids=["%s-%d-%s" % (w.name, n, "strong" if s else "weak")
                              for w, n, s in CASES])
def test_bench_ranks_equal_single_gpu(gpu_lib, wl, world, strong):
    Xr = _ranks(wl, world, strong)
    Xs, its = _single(wl, world, strong)
    assert its == STEPS
    assert Xr.shape == Xs.shape
    assert np.array_equal(Xr, Xs)
