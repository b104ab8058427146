"""GPU: several devices behind ONE drop-in call (pfdr_set_devices,
csrc/pfdr_multidev.hip).  The reference's PFDR_* entry points are single
synchronous host calls (include/PFDR_graph_quadratic_d1_bounds.hpp:34-40,
called by src/CP_PFDR_graph_quadratic_d1_bounds.cpp:824-835); configured with
a device list, the library splits the caller's graph by vertex range, runs
one rank per device on its own host thread and copies every rank's slice of
X into the caller's array.  Expected bit-identical to the one-GPU drop-in:
X, iteration count and Dif (sequential-rounding evolution summed rank to
rank).

On a one-GPU box: a one-device group runs the RCCL partitioned session on a
1-rank communicator; a list repeating device 0 runs 2-3 ranks as threads on
it over the loopback transport (RCCL refuses two ranks on one GPU)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def one_gpu_after():
    from cp_pfdr_graph_d1_amd import pfdr
    yield
    pfdr.set_devices([])


def _l1_problem(shape=(700, 600), dt=np.float32):
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, piecewise_observation
    V = int(np.prod(shape))
    Eu, Ev = grid_graph(shape, 4)
    Y = piecewise_observation(shape, 3, dt)
    return V, Eu, Ev, Y


@pytest.mark.parametrize("devs", [[0], [0, 0], [0, 0, 0]], ids=["rccl1", "loop2", "loop3"])
@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_dropin_l1_partitioned_equals_one_gpu(gpu_lib, one_gpu_after, devs, dt):
    from cp_pfdr_graph_d1_amd import pfdr
    V, Eu, Ev, Y = _l1_problem(dt=dt)
    La = np.full(Eu.size, 0.1, dt)
    L1 = np.full(V, 0.01, dt)
    args = (np.zeros(V, dt), Y, None, 0, Eu, Ev, La, L1, 0, pfdr.SCAL, None, 1.5, 1e-3, 1e-2,
            1e-5, 2000)
    lib = pfdr.Lib()
    pfdr.set_devices([])
    X1, it1, _, D1 = lib.quadratic_d1_l1(*args, dif=True)
    pfdr.set_devices(devs, min_vertices=0)
    Xk, itk, _, Dk = lib.quadratic_d1_l1(*args, dif=True)
    print("devices %s: it %d / %d" % (devs, itk, it1))
    assert 0 < it1 < 2000 and itk == it1
    assert np.array_equal(Dk[:itk], D1[:it1])
    assert np.array_equal(Xk, X1)


def test_dropin_bounds_partitioned_equals_one_gpu(gpu_lib, one_gpu_after):
    """3-D 6-NN grid with a box constraint (C5's solver), 2 ranks"""
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import piecewise_observation
    shape = (80, 72, 64)
    V = int(np.prod(shape))
    Eu, Ev = pfdr.gen_grid_edges(shape, 6)
    dt = np.float32
    Y = piecewise_observation(shape, 5, dt)
    La = np.full(Eu.size, 0.1, dt)
    args = (np.zeros(V, dt), Y, None, 0, Eu, Ev, La, 0.0, 1.0, pfdr.SCAL, None, 1.5, 1e-3, 0.0,
            0.0, 40)
    lib = pfdr.Lib()
    pfdr.set_devices([])
    X1, it1, O1, _ = lib.quadratic_d1_bounds(*args, obj=True)
    pfdr.set_devices([0, 0], min_vertices=0)
    X2, it2, O2, _ = lib.quadratic_d1_bounds(*args, obj=True)
    assert it1 == it2 == 40
    assert np.array_equal(X2, X1)
    # the objective's partial sums meet across the ranks (a tree)
    assert np.allclose(O2[:41], O1[:41], rtol=1e-5)


@pytest.mark.parametrize("devs", [[0], [0, 0]], ids=["rccl1", "loop2"])
def test_dropin_simplex_partitioned_equals_one_gpu(gpu_lib, one_gpu_after, devs):
    from cp_pfdr_graph_d1_amd import pfdr
    from cp_pfdr_graph_d1_amd.graphs import grid_graph, simplex_observation
    n, K = 380, 4
    Eu, Ev = grid_graph((n, n), 8)
    V = n * n
    v = np.arange(V)
    lab = ((v % n) * 2 // n) + 2 * ((v // n) * 2 // n)
    Q = simplex_observation(V, K, 4, lab, np.float32)
    La = np.full(Eu.size, 0.05, np.float32)
    args = (Q.copy(), Q, K, Eu, Ev, La, 0.1, None, 1.0, 0.1, 0.0, 1e-4, 500)
    lib = pfdr.Lib()
    pfdr.set_devices([])
    P1, it1, _, D1 = lib.loss_d1_simplex(*args, dif=True)
    pfdr.set_devices(devs, min_vertices=0)
    Pk, itk, _, Dk = lib.loss_d1_simplex(*args, dif=True)
    print("devices %s: it %d / %d" % (devs, itk, it1))
    assert 0 < it1 < 500 and itk == it1
    assert np.array_equal(Dk[:itk], D1[:it1])
    assert np.array_equal(Pk, P1)


def test_dropin_small_calls_stay_on_one_gpu(gpu_lib, one_gpu_after):
    """below min_vertices (CP's reduced problems) the call is the one-GPU
    session: same result, and a bad configuration is refused"""
    from cp_pfdr_graph_d1_amd import pfdr
    V, Eu, Ev, Y = _l1_problem((64, 48))
    args = (np.zeros(V, np.float32), Y, None, 0, Eu, Ev, np.full(Eu.size, 0.1, np.float32),
            None, 0, pfdr.SCAL, None, 1.5, 1e-3, 0.0, 1e-4, 300)
    lib = pfdr.Lib()
    X1, it1, _, _ = lib.quadratic_d1_l1(*args)
    pfdr.set_devices([0, 0], min_vertices=1 << 20)
    X2, it2, _, _ = lib.quadratic_d1_l1(*args)
    assert it1 == it2 and np.array_equal(X1, X2)
    with pytest.raises(pfdr.PFDRError):
        pfdr.set_devices([0, 99])
