"""GPU: the stable LSD radix sort behind the incidence lists
(csrc/pfdr_sort.hip, pfdr_radix_sort_pairs_{u32,u64}) against numpy's stable
argsort on the masked keys: keys and values equal element for element --
random keys at every bit width the library uses, sizes around the 4096-key
tile and the scan chunk (ragged tails), all-equal keys, already sorted and
reversed inputs, one element, 2 x 10^7 pairs."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sort(lib, keys, vals, bits):
    k = np.ascontiguousarray(keys).copy()
    v = np.ascontiguousarray(vals, np.uint32).copy()
    fn = lib.pfdr_radix_sort_pairs_u32 if k.dtype == np.uint32 else lib.pfdr_radix_sort_pairs_u64
    ms = C.c_double()
    rc = fn(C.c_int64(k.size), k.ctypes.data_as(C.c_void_p), v.ctypes.data_as(C.c_void_p),
            C.c_int(bits), C.byref(ms))
    assert rc == 0
    return k, v, ms.value


def _ref(keys, vals, bits):
    mask = (1 << bits) - 1 if bits < 64 else (1 << 64) - 1
    kk = keys & keys.dtype.type(mask)
    o = np.argsort(kk, kind="stable")
    return keys[o], vals[o]


@pytest.fixture(scope="module")
def clib(gpu_lib):
    from cp_pfdr_graph_d1_amd import pfdr
    return pfdr.load()


@pytest.mark.parametrize("dt,bits", [(np.uint32, 3), (np.uint32, 8), (np.uint32, 17),
                                     (np.uint32, 24), (np.uint32, 32), (np.uint64, 40),
                                     (np.uint64, 57), (np.uint64, 64)])
@pytest.mark.parametrize("n", [1, 255, 4095, 4096, 4097, 70001, 1 << 20])
def test_sort_matches_numpy_stable(clib, dt, bits, n):
    rng = np.random.default_rng(n + bits)
    hi = (1 << bits) if bits < 64 else None
    if dt == np.uint64:
        keys = rng.integers(0, np.iinfo(np.uint64).max, n, dtype=np.uint64, endpoint=True)
        if hi:
            keys &= np.uint64(hi - 1)
    else:
        keys = rng.integers(0, hi, n, dtype=np.uint64).astype(np.uint32)
    # few distinct keys: long equal runs whose order the sort must keep
    keys[rng.random(n) < 0.5] = keys[0]
    vals = np.arange(n, dtype=np.uint32)
    k, v, _ = _sort(clib, keys, vals, bits)
    rk, rv = _ref(keys, vals, bits)
    assert np.array_equal(k, rk)
    assert np.array_equal(v, rv)


def test_sort_ignores_bits_above(clib):
    """keys equal in their low bits keep their input order whatever the high bits"""
    n = 50000
    rng = np.random.default_rng(1)
    keys = (rng.integers(0, 1 << 12, n).astype(np.uint32) << np.uint32(20)) | \
        rng.integers(0, 16, n).astype(np.uint32)
    vals = np.arange(n, dtype=np.uint32)
    k, v, _ = _sort(clib, keys, vals, 4)
    o = np.argsort(keys & np.uint32(15), kind="stable")
    assert np.array_equal(v, vals[o])
    assert np.array_equal(k, keys[o])


@pytest.mark.parametrize("order", ["equal", "sorted", "reversed"])
def test_sort_degenerate_orders(clib, order):
    n = 300000
    keys = {"equal": np.full(n, 7, np.uint32), "sorted": np.arange(n, dtype=np.uint32),
            "reversed": np.arange(n, dtype=np.uint32)[::-1].copy()}[order]
    vals = np.arange(n, dtype=np.uint32)[::-1].copy()
    k, v, _ = _sort(clib, keys, vals, 20)
    rk, rv = _ref(keys, vals, 20)
    assert np.array_equal(k, rk) and np.array_equal(v, rv)


def test_sort_large(clib):
    """the incidence size of a 10^7-edge graph: 2 x 10^7 slots, 24 bits"""
    n = 20_000_000
    rng = np.random.default_rng(9)
    keys = rng.integers(0, 10_000_000, n, dtype=np.uint32)
    vals = np.arange(n, dtype=np.uint32)
    k, v, ms = _sort(clib, keys, vals, 24)
    rk, rv = _ref(keys, vals, 24)
    print("2e7 pairs, 24 bits: %.3f ms" % ms)
    assert np.array_equal(k, rk) and np.array_equal(v, rv)
