"""GPU: the edge-block records of the tiled edge sweep (k_tile_erec,
csrc/pfdr_quadratic_kernels.hpp) on a partitioned rank's edge order, checked
deterministically through the C-ABI test hook pfdr_debug_tile_erec.

A partitioned rank sorts its edges by (u block, v block) with the edges that
have a ghost end after all the interior ones, so the edge block that
straddles the cut sees its u block DROP.  Round 3's kernel then indexed its
u-block starts below its own record (q = u / 256 - ub0 < 0) and wrote into an
earlier block's record while that block's own wave was building it: the
intermittent full-size 2-rank mismatch.  Here every other record is
pre-filled with a sentinel and only the straddling block is built -- the
sentinels must survive and the record must equal the host computation below
(the straddling block unstaged: the sweep reads Eu for it).  Edge sweep it
serves: reference src/PFDR_graph_quadratic_d1_l1.cpp:466-489."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SENT = 0x5A5A5A5A
INT_MAX = 0x7FFFFFFF


def _layout(lib):
    ints, runs, nost = C.c_int(), C.c_int(), C.c_int()
    assert lib.pfdr_debug_erec_layout(C.byref(ints), C.byref(runs), C.byref(nost)) == 0
    return ints.value, runs.value, nost.value


def _hook(lib, Eu, Ev, dtype_code, b0, nb, rec):
    fn = lib.pfdr_debug_tile_erec
    fn.argtypes = [C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                   C.c_int64]
    rc = fn(Eu.size, dtype_code, Eu.ctypes.data, Ev.ctypes.data, b0, nb, rec.ctypes.data,
            rec.size)
    assert rc == 0, lib.pfdr_last_error()


def erec_host(Eu, Ev, blk, EB, KEREC, RUNS, NOSTAGE):
    """the record k_tile_erec writes for edge block blk (see its comment)"""
    eb, ee = blk * EB, min(blk * EB + EB, Eu.size)
    u, v = Eu[eb:ee].astype(np.int64), Ev[eb:ee].astype(np.int64)
    ub, vb = u // 256, v // 256
    ub0 = int(ub[0])
    drop = bool(np.any(ub[1:] < ub[:-1]))
    nub = NOSTAGE if drop else int(ub[-1]) - ub0 + 1
    starts = [0] + [i for i in range(1, u.size) if vb[i] != vb[i - 1]]
    r = np.zeros(KEREC, np.int64)
    r[0], r[1] = ub0, nub
    r[2] = len(starts) if len(starts) <= RUNS else 0
    r[3] = int(u.min()) - ub0 * 256
    r[4] = int(u.max() - u.min()) + 1
    for q in range(1, 4):
        if drop or q >= nub:
            r[4 + q] = INT_MAX
        else:
            r[4 + q] = int(np.argmax(ub - ub0 >= q))
    for k in range(RUNS):
        if k < len(starts):
            r[8 + 2 * k], r[9 + 2 * k] = starts[k], int(vb[starts[k]]) * 256
        else:
            r[8 + 2 * k], r[9 + 2 * k] = INT_MAX, 0
    return r.astype(np.int32)


def _rank_edges(EB, nint_blocks, cut, lo_interior, drop_to, nbnd):
    """a rank's tile-ordered edges: interior edges [0, Eint) with u blocks
    rising from lo_interior, then boundary edges whose u blocks restart at
    drop_to; Eint = nint_blocks * EB + cut (the straddling block is
    nint_blocks).  v ends a few blocks above u (ghost range for the
    boundary part)."""
    Eint = nint_blocks * EB + cut
    i = np.arange(Eint)
    u_int = lo_interior * 256 + (i * 3) // 4           # 0.75 u per edge: blocks rise
    v_int = u_int + 300 + (i % 7)
    j = np.arange(nbnd)
    u_b = drop_to * 256 + (j * 3) // 4
    v_b = 10_000_000 + (j % 11) * 97                   # ghosts, far away
    Eu = np.concatenate([u_int, u_b]).astype(np.int32)
    Ev = np.concatenate([v_int, v_b]).astype(np.int32)
    return Eu, Ev, Eint


@pytest.mark.parametrize("dt,drop", [("f32", "far"), ("f32", "near"), ("f64", "far"),
                                     ("f64", "near")])
def test_straddling_block_writes_only_its_record(gpu_lib, dt, drop):
    from cp_pfdr_graph_d1_amd import pfdr
    lib = pfdr.load()
    KEREC, RUNS, NOSTAGE = _layout(lib)
    EB = 1024 if dt == "f32" else 512
    code = pfdr.PFDR_F32 if dt == "f32" else pfdr.PFDR_F64
    nint_blocks = 9
    # far: the boundary restarts ~40 u blocks below the straddling block's
    # first u block (round 3's write landed records before); near: one block
    # below, a span that would fit the LDS stage (the staged lookup would
    # then have read the wrong u end)
    lo = 10
    top_block = lo + (nint_blocks * EB * 3 // 4) // 256
    drop_to = lo if drop == "far" else top_block - 1
    Eu, Ev, Eint = _rank_edges(EB, nint_blocks, EB // 3, lo, drop_to, 4 * EB + 77)
    nblk = (Eu.size + EB - 1) // EB
    assert np.any(np.diff(Eu[nint_blocks * EB: (nint_blocks + 1) * EB] // 256) < 0)
    if drop == "far":
        assert top_block - drop_to > 4
    rec = np.full(nblk * KEREC, SENT, np.int32)
    _hook(lib, Eu, Ev, code, nint_blocks, 1, rec)
    R = rec.reshape(nblk, KEREC)
    for b in range(nblk):
        if b != nint_blocks:
            assert np.all(R[b] == SENT), "record of block %d touched" % b
    want = erec_host(Eu, Ev, nint_blocks, EB, KEREC, RUNS, NOSTAGE)
    assert want[1] == NOSTAGE
    assert np.array_equal(R[nint_blocks], want), (R[nint_blocks], want)
    # every block at once: each record is its host computation (monotone
    # blocks keep their staged u-block starts)
    rec2 = np.full(nblk * KEREC, SENT, np.int32)
    _hook(lib, Eu, Ev, code, 0, nblk, rec2)
    R2 = rec2.reshape(nblk, KEREC)
    for b in range(nblk):
        assert np.array_equal(R2[b], erec_host(Eu, Ev, b, EB, KEREC, RUNS, NOSTAGE)), b
    assert all(R2[b][1] < 4 for b in range(nint_blocks))  # interior blocks staged


def test_hook_rejects_mismatched_records(gpu_lib):
    from cp_pfdr_graph_d1_amd import pfdr
    lib = pfdr.load()
    KEREC, _, _ = _layout(lib)
    Eu = np.arange(3000, dtype=np.int32)
    Ev = Eu + 1
    rec = np.zeros(KEREC, np.int32)  # 3 blocks need 3 records
    fn = lib.pfdr_debug_tile_erec
    fn.argtypes = [C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                   C.c_int64]
    assert fn(Eu.size, pfdr.PFDR_F32, Eu.ctypes.data, Ev.ctypes.data, 0, 1, rec.ctypes.data,
              rec.size) != 0
