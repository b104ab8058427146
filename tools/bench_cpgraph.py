"""Measure the cut-pursuit graph steps on the GPU (pfdr_cpgraph_*,
SURVEY.md §8(f) ranks 2-3) at the headline size, with the restatement
timed on the host beside it.

Graph: the headline jittered 250x200x200 6-NN graph (V = 10M, E = 60M),
La_d1 = 0.1, La_l1 = 0.01, Y the headline observation.  State: a mid-run
CP iteration — the activity of a synthetic cut (vertices split into 10^3-
vertex blocks, alternate blocks on the source side), its components, and
component values drawn at random and rounded (so the merge finds ties).
Each step is timed on that state (median of --reps, device-resident
inputs and outputs; activity restored between repetitions):

    gradient (N = 0, identity), capacities (cut 1 and 2), activate,
    components, reduced graph, merge; and the duplex driver's two-layer cut
    (capacities, activation)

plus the PCIe-inclusive capacities -> host copy a host maxflow needs.
CPU: oracle/liboracle_pfdr.so (single-threaded restatement of the same
reference lines) on the same state, when --cpu.  Prints one JSON line.

    python tools/bench_cpgraph.py [--shape 250 200 200] [--reps 5] [--cpu]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=3, default=(250, 200, 200))
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--block", type=int, default=10)
    ap.add_argument("--cpu", action="store_true")
    args = ap.parse_args()
    import torch
    from cp_pfdr_graph_d1_amd import pfdr
    lib = pfdr.load()
    nx, ny, nz = args.shape
    V = nx * ny * nz
    t = time.perf_counter()
    Eu, Ev = pfdr.gen_knn_jitter_grid((nx, ny, nz), 6, 6, 0.25)
    Y = pfdr.gen_piecewise(nx, V, 2, np.float32, 0.2)
    E = Eu.size
    La = np.full(E, 0.1, np.float32)
    L1 = np.full(V, 0.01, np.float32)
    b = args.block
    v = np.arange(V, dtype=np.int64)
    x, y, z = v % nx, (v // nx) % ny, v // (nx * ny)
    seg = (((x // b) + (y // b) + (z // b)) & 1).astype(np.uint8)
    gen_s = time.perf_counter() - t
    torch.cuda.set_device(0)
    g = pfdr.CPGraph(V, Eu, Ev, La, L1)
    h = g.h

    def call(name, *a):
        pfdr._check(getattr(lib, name)(h, *a), name)

    # the CP state: one cut from the single initial component
    g.set_values(np.array([0.25], np.float32))
    w = g.activate(seg)
    Cv, Vc, rVc = g.components()
    rV = rVc.size - 1
    rng = np.random.default_rng(3)
    rX = np.round(rng.standard_normal(rV), 1).astype(np.float32)
    g.set_values(rX)
    act0 = g.active()
    active_edges = int(act0.sum())
    dY = torch.from_numpy(Y).cuda()
    dtr = torch.empty(V, dtype=torch.float32, device="cuda")
    drc = torch.empty(E, dtype=torch.float32, device="cuda")
    dDf = torch.empty(V, dtype=torch.float32, device="cuda")
    dseg = torch.from_numpy(seg ^ (rng.random(V) < 0.01).astype(np.uint8)).cuda()
    # the duplex driver's two-layer cut (2V nodes)
    dtr2 = torch.empty(2 * V, dtype=torch.float32, device="cuda")
    dlink = torch.empty(V, dtype=torch.float32, device="cuda")
    seg2 = np.concatenate([seg, seg ^ (rng.random(V) < 0.01).astype(np.uint8)])
    dseg2 = torch.from_numpy(seg2).cuda()
    DEV = pfdr.PFDR_MEM_DEVICE
    rE = C.c_int()
    n = C.c_int()
    eps = float(np.finfo(np.float32).eps)
    vp = lambda t_: C.c_void_p(t_.data_ptr())

    def restore():
        g.set_active(act0)

    steps = {
        "gradient": lambda: call("pfdr_cpgraph_gradient", C.c_int(0), None, vp(dY), None, DEV,
                                 vp(dDf)),
        "capacities_cut1": lambda: call("pfdr_cpgraph_capacities", C.c_int(1), C.c_int(0),
                                        vp(dtr), vp(drc), DEV),
        "capacities_cut2": lambda: call("pfdr_cpgraph_capacities", C.c_int(2), C.c_int(0),
                                        vp(dtr), vp(drc), DEV),
        "activate": lambda: call("pfdr_cpgraph_activate", C.c_void_p(dseg.data_ptr()), DEV,
                                 C.byref(n)),
        "capacities_duplex": lambda: call("pfdr_cpgraph_capacities_duplex", C.c_int(0),
                                          vp(dtr2), vp(dlink), vp(drc), DEV),
        "activate_duplex": lambda: call("pfdr_cpgraph_activate_duplex",
                                        C.c_void_p(dseg2.data_ptr()), DEV, C.byref(n)),
        "components": lambda: call("pfdr_cpgraph_components", C.byref(C.c_int())),
        "reduced_graph": lambda: call("pfdr_cpgraph_reduced_graph", C.c_double(eps),
                                      C.byref(rE)),
        "merge": lambda: call("pfdr_cpgraph_merge", C.c_double(eps), C.c_double(1e-3),
                              C.byref(n)),
    }
    res = {}
    for name, fn in steps.items():
        ts = []
        for r in range(args.reps + 1):
            restore()
            if name in ("reduced_graph", "merge", "gradient", "capacities_cut1",
                        "capacities_cut2", "capacities_duplex"):
                call("pfdr_cpgraph_set_components", C.c_int(rV), C.c_void_p(Cv.ctypes.data),
                     C.c_void_p(Vc.ctypes.data), C.c_void_p(rVc.ctypes.data), pfdr.PFDR_MEM_HOST)
                g.set_values(rX)
            if name == "gradient" or name.startswith("capacities"):
                fn_grad = steps["gradient"]
                if name != "gradient":
                    fn_grad()
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            if r:  # first repetition warms up
                ts.append(time.perf_counter() - t)
        res[name] = round(float(np.median(ts)) * 1e3, 3)
    # PCIe-inclusive: capacities straight to host (what a host maxflow consumes)
    restore()
    g.set_values(rX)
    steps["gradient"]()
    ts = []
    for r in range(args.reps + 1):
        t = time.perf_counter()
        g.capacities(1, 0)
        if r:
            ts.append(time.perf_counter() - t)
    res["capacities_cut1_to_host"] = round(float(np.median(ts)) * 1e3, 3)
    # the reduced graph as produced
    restore()
    call("pfdr_cpgraph_set_components", C.c_int(rV), C.c_void_p(Cv.ctypes.data),
         C.c_void_p(Vc.ctypes.data), C.c_void_p(rVc.ctypes.data), pfdr.PFDR_MEM_HOST)
    rEu, rEv, rLa, rL1 = g.reduced_graph(eps)
    g.close()
    total = sum(v for k, v in res.items()
                if not k.endswith("_to_host") and not k.endswith("_duplex"))
    out = {
        "what": "CP graph steps (pfdr_cpgraph_*), one MI355X, device-resident",
        "graph": "jittered %dx%dx%d 6-NN (V=%d, E=%d)" % (nx, ny, nz, V, E),
        "state": {"cut_block": b, "activated_by_cut": w, "active_edges": active_edges,
                  "components": rV, "reduced_edges": int(rEu.size)},
        "gpu_ms": res,
        "gpu_ms_iteration_graph_steps": round(total, 3),
        "iteration_note": "the l1 driver's two-cut iteration; *_duplex: the duplex driver's "
                          "one two-layer cut instead of the two cuts",
        "input_generation_s": round(gen_s, 2),
    }
    if args.cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        o = oracle.Oracle("port")
        cpu = {}
        t = time.perf_counter()
        D = o.cp_gradient(0, V, None, Y, None, Eu, Ev, La, L1, act0, Cv, Vc, rVc, rX)
        cpu["gradient"] = time.perf_counter() - t
        t = time.perf_counter()
        o.cp_capacities(1, La, L1, 0, act0, Cv, rX, D)
        cpu["capacities_cut1"] = time.perf_counter() - t
        t = time.perf_counter()
        o.cp_capacities(2, La, L1, 0, act0, Cv, rX, D)
        cpu["capacities_cut2"] = time.perf_counter() - t
        sg = dseg.cpu().numpy()
        t = time.perf_counter()
        o.cp_activate(Eu, Ev, sg, act0)
        cpu["activate"] = time.perf_counter() - t
        t = time.perf_counter()
        o.cp_capacities_duplex(La, L1, 0, act0, Cv, rX, D)
        cpu["capacities_duplex"] = time.perf_counter() - t
        t = time.perf_counter()
        o.cp_activate_duplex(V, Eu, Ev, seg2, act0)
        cpu["activate_duplex"] = time.perf_counter() - t
        t = time.perf_counter()
        oCv, oVc, orVc = o.cp_components(V, Eu, Ev, act0)
        cpu["components"] = time.perf_counter() - t
        t = time.perf_counter()
        ored = o.cp_reduced_graph(V, Eu, Ev, La, L1, act0, oCv, oVc, orVc, eps)
        cpu["reduced_graph"] = time.perf_counter() - t
        t = time.perf_counter()
        o.cp_merge(Eu, Ev, oCv, rX, eps, 1e-3, act0)
        cpu["merge"] = time.perf_counter() - t
        out["cpu_ms"] = {k: round(v * 1e3, 1) for k, v in cpu.items()}
        out["cpu_ms_iteration_graph_steps"] = round(
            sum(v for k, v in cpu.items() if not k.endswith("_duplex")) * 1e3, 1)
        out["cpu"] = {"kind": "port", "cores": 1,
                      "note": "single-threaded C restatement (oracle/cp_graph_body.h); "
                              "components / reduced graph / gradient rebuild the maxflow "
                              "graph's arc lists per call (O(E)), which the reference keeps"}
        out["parity_full_size"] = bool(
            np.array_equal(oCv, Cv) and np.array_equal(oVc, Vc) and np.array_equal(orVc, rVc)
            and np.array_equal(ored[0], rEu) and np.array_equal(ored[1], rEv)
            and np.array_equal(ored[2].view(np.uint32), rLa.view(np.uint32)))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
