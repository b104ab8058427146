"""GPU: the partitioned solver (1-D vertex ranges, halo pull/push, chained
exact preconditioner sum) with k ranks as k threads on ONE GPU (loopback
transport: the same session code as RCCL, exchanges as device copies),
against the REFERENCE's golden outputs.  Expected bit-exact: partitioning
changes no arithmetic and no summation order (tests/test_partition_cpu.py)."""
import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

CASES = ["l1_grid2d_f64", "l1_grid2d_f32", "l1_knn_shuffled_f32", "l1_l22_f64",
         "l1_grid3d_pos_f32", "l1_grid2d_recond_f64", "bounds_box_f32",
         "bounds_upper_recond_f32", "l1_chain_kat_f64"]


def _solve(c, k, fixed):
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    a = dict(c)
    if fixed:
        a.update(difTol=0.0, difRcd=0.0, itMax=G.FIXED_K)
    kind = pfdr.PFDR_KIND_L1 if str(a["solver"]) == "l1" else pfdr.PFDR_KIND_BOUNDS
    X0 = a["X0"]
    return P.solve_loopback(
        k, kind, X0.dtype, a["Eu"], a["Ev"], a["La_d1"], X0, a["Y"], A=a["A"],
        La_l1=a.get("La_l1"), positivity=int(a.get("positivity", 0)),
        lo=float(a.get("lo", -np.inf)), hi=float(a.get("hi", np.inf)), Ltype=int(a["Ltype"]),
        L=a["L"], rho=float(a["rho"]), condMin=float(a["condMin"]),
        difRcd=float(a["difRcd"]), difTol=float(a["difTol"]), itMax=int(a["itMax"]),
        record_obj=True, record_dif=True)


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("k", [2, 3])
@pytest.mark.parametrize("fixed", [True, False], ids=["fixk", "conv"])
def test_partitioned_equals_reference(gpu_lib, name, k, fixed):
    c, g = G.load(name)
    if c["X0"].size < 4 * k:
        pytest.skip("graph too small for %d ranks" % k)
    X, it, Obj, Dif, info = _solve(c, k, fixed)
    tag = "fixk" if fixed else "conv"
    print("%s k=%d %s it=%d/%d edges/rank=%s bitexact=%s" % (
        name, k, tag, it, int(g[tag + "_it"]), info["edges"], np.array_equal(X, g[tag + "_X"])))
    assert it == int(g[tag + "_it"])
    assert np.array_equal(X, g[tag + "_X"])
    n = it
    assert G.rel_l2(Dif[:n], g[tag + "_Dif"][:n]) <= (1e-5 if X.dtype == np.float32 else 1e-12)
    if tag + "_Obj" in g:
        go = g[tag + "_Obj"][: n + 1]
        assert np.allclose(Obj[: n + 1], go, rtol=1e-5, atol=1e-6 * np.abs(go).max())


def test_partitioned_headline_slab_matches_single(gpu_lib):
    """weak-scaling geometry of bench.py at a small size: slabs of a jittered
    6-NN grid, 4 ranks, against the single-GPU session"""
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    shape = (40, 30, 32)
    V = 40 * 30 * 32
    Eu, Ev = pfdr.gen_knn_jitter_grid(shape, 6, 6)
    Y = pfdr.gen_piecewise(40, V, 2, np.float32)
    La = np.full(Eu.size, 0.1, np.float32)
    L1 = np.full(V, 0.01, np.float32)
    X0 = np.zeros(V, np.float32)
    s = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, Eu.size, Eu, Ev, La, X0, Y, La_l1=L1,
                     difTol=1e-5, itMax=300, record_dif=True)
    s.run(300)
    Xs, its, _, Difs = s.result()
    s.close()
    X, it, _, Dif, _ = P.solve_loopback(4, pfdr.PFDR_KIND_L1, np.float32, Eu, Ev, La, X0, Y,
                                        La_l1=L1, difTol=1e-5, itMax=300, record_dif=True)
    assert it == its
    assert np.array_equal(X, Xs)


def test_rccl_transport_single_rank(gpu_lib):
    """the RCCL transport code path (comm init, grouped send/recv, all-reduce,
    broadcast, chain) on a 1-rank communicator: equals the plain session"""
    import ctypes as C
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    lib = pfdr.load()
    idb = (C.c_char * 128)()
    assert lib.pfdr_comm_unique_id(idb) == 0
    comm = C.c_void_p()
    assert lib.pfdr_comm_init(C.byref(comm), 1, 0, idb) == 0, lib.pfdr_last_error()
    c, g = G.load("l1_grid2d_f32")
    a = dict(c, difTol=0.0, difRcd=0.0, itMax=G.FIXED_K)
    V = a["X0"].size
    s = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, a["Eu"].size, a["Eu"], a["Ev"],
                     a["La_d1"], a["X0"], a["Y"], La_l1=a["La_l1"], rho=float(a["rho"]),
                     condMin=float(a["condMin"]), itMax=G.FIXED_K, record_dif=True,
                     record_obj=True, nranks=1, rank=0, comm=comm.value,
                     comm_kind=P.COMM_RCCL, vtx_begin=0, V_global=V)
    s.run(G.FIXED_K)
    X, it, Obj, Dif = s.result()
    s.close()
    v = C.c_double(3.5)
    assert lib.pfdr_comm_allreduce_max_f64(comm, C.byref(v)) == 0 and v.value == 3.5
    lib.pfdr_comm_destroy(comm)
    assert it == G.FIXED_K and np.array_equal(X, g["fixk_X"])
