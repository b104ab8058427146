"""CPU, world_size 2 (gloo): the library's partition planner driven over
torch.distributed exactly as a partitioned session drives it over RCCL.

Checked per rank, against the unpartitioned graph:
  * ghosts = the non-owned endpoints of the rank's edges, grouped by owner;
  * pull: after packing owned values at PULL_INDEX and landing the peers'
    in the ghost range, every ghost holds its owner's value;
  * push + CSR: local slots plus the received items, sorted by key, list for
    every owned vertex exactly its global incidences in global (e, side)
    order, and a float32 sequential sum over them equals the unpartitioned
    sequential sum BIT FOR BIT (the property that makes a partitioned solve
    equal the single-GPU / reference one).
Graph: shuffled jittered-grid 6-NN with self-loops and duplicate edges.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _graph():
    import sys
    sys.path.insert(0, ROOT)
    from cp_pfdr_graph_d1_amd.graphs import knn_jitter_grid, uniform
    Eu, Ev = knn_jitter_grid((7, 6, 5), 6, seed=3)
    V = 210
    perm = np.argsort(uniform(11, np.arange(V)), kind="stable")
    inv = np.empty(V, np.int64)
    inv[perm] = np.arange(V)
    Eu, Ev = inv[Eu], inv[Ev]
    e = np.argsort(uniform(12, np.arange(Eu.size)), kind="stable")
    Eu, Ev = Eu[e], Ev[e]
    # self-loops and a duplicated edge
    Eu = np.concatenate([Eu, [5, 100, 7, Eu[3]]]).astype(np.int32)
    Ev = np.concatenate([Ev, [5, 100, 9, Ev[3]]]).astype(np.int32)
    return V, Eu, Ev


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    from cp_pfdr_graph_d1_amd import partition as P
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port,
                            rank=rank, world_size=world)
    try:
        V, Eu, Ev = _graph()
        off = P.vertex_offsets(V, world)
        parts = P.split_edges(Eu, off)
        mine = parts[rank]
        plan = P.Plan(world, rank, off, Eu[mine], Ev[mine], mine)
        msgs = {q: (plan.get(P.PLAN_PULL_REQUEST, q), plan.get(P.PLAN_PUSH_ITEMS, q))
                for q in range(world) if q != rank}
        allm = [None] * world
        dist.all_gather_object(allm, msgs)
        for q in range(world):
            if q != rank:
                req, items = allm[q][rank]
                plan.set_incoming(q, P.PLAN_PULL_REQUEST, req)
                plan.set_incoming(q, P.PLAN_PUSH_ITEMS, items)
        plan.finish()
        lo, hi = int(off[rank]), int(off[rank + 1])
        Vl, El = hi - lo, mine.size
        ghosts = plan.get(P.PLAN_GHOSTS)
        Eul, Evl = plan.get(P.PLAN_EU_LOCAL), plan.get(P.PLAN_EV_LOCAL)
        # --- ghosts and local ids
        ends = np.concatenate([Eu[mine], Ev[mine]]).astype(np.int64)
        want = np.unique(ends[(ends < lo) | (ends >= hi)])
        assert np.array_equal(ghosts, want)
        glob = np.concatenate([np.arange(lo, hi), ghosts])
        assert np.array_equal(glob[Eul], Eu[mine]) and np.array_equal(glob[Evl], Ev[mine])
        # --- pull: values of a global vector land in the ghost range
        g = np.random.default_rng(0).random(V).astype(np.float32)
        pidx, poff = plan.get(P.PLAN_PULL_INDEX), plan.get(P.PLAN_PULL_OFFSETS)
        goff = plan.get(P.PLAN_GHOST_OFFSETS)
        send = {q: g[lo:hi][pidx[poff[q]:poff[q + 1]]] for q in range(world) if q != rank}
        allm = [None] * world
        dist.all_gather_object(allm, send)
        ext = np.concatenate([g[lo:hi], np.zeros(ghosts.size, np.float32)])
        for q in range(world):
            if q != rank:
                ext[Vl + goff[q]: Vl + goff[q + 1]] = allm[q][rank]
        assert np.array_equal(ext[Vl:], g[ghosts])
        # --- push + keyed CSR: per-vertex sums in global (e, side) order
        c = np.random.default_rng(1).random(2 * Eu.size).astype(np.float32)  # per global slot
        wz = np.concatenate([c[2 * mine], c[2 * mine + 1]])  # side-major local layout
        padr, psoff = plan.get(P.PLAN_PUSH_ADDR), plan.get(P.PLAN_PUSH_OFFSETS)
        send = {q: wz[padr[psoff[q]:psoff[q + 1]]] for q in range(world) if q != rank}
        allm = [None] * world
        dist.all_gather_object(allm, send)
        roff = plan.get(P.PLAN_RECV_OFFSETS)
        tail = np.zeros(roff[-1], np.float32)
        for q in range(world):
            if q != rank:
                tail[roff[q]:roff[q + 1]] = allm[q][rank]
        vals = np.concatenate([wz, tail])
        keys = []
        for side, ends_l in ((0, Eul), (1, Evl)):
            for e in range(El):
                if ends_l[e] < Vl:
                    keys.append(((int(ends_l[e]) << 32) | (2 * int(mine[e]) + side),
                                 side * El + e))
        rk = plan.get(P.PLAN_RECV_KEYS)
        keys += [(int(k), 2 * El + j) for j, k in enumerate(rk)]
        keys.sort()
        sums = np.zeros(Vl, np.float32)
        orders = [[] for _ in range(Vl)]
        for k, a in keys:
            v = k >> 32
            orders[v].append(k & 0xffffffff)
            sums[v] = np.float32(sums[v] + vals[a])
        ref_sums = np.zeros(V, np.float32)
        ref_orders = [[] for _ in range(V)]
        for e in range(Eu.size):  # the reference's sequential scatter order
            for side, vv in ((0, Eu[e]), (1, Ev[e])):
                ref_sums[vv] = np.float32(ref_sums[vv] + c[2 * e + side])
                ref_orders[vv].append(2 * e + side)
        for v in range(Vl):
            assert orders[v] == ref_orders[lo + v], v
        assert np.array_equal(sums, ref_sums[lo:hi])
        out[rank] = 1
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
def test_partition_plan_gloo(world):
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world,
                       start_method="spawn", join=True)
    assert sorted(out.keys()) == list(range(world))
