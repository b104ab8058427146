"""Measure the simplex driver's cut-pursuit graph steps on the GPU
(pfdr_cpgraph_simplex_*, src/CP_PFDR_graph_loss_d1_simplex.cpp) at C4's
size, with the single-threaded restatement timed beside it (--cpu).

Graph: C4's 2236 x 2236 8-neighbour grid (V = 5.0M, E = 20.0M), K = 10
labels, smoothed-KL loss al = 0.1, La_d1 = 0.05, Q random in the simplex.
State: a mid-run CP iteration -- the activity of a synthetic cut (alternate
10 x 10 vertex blocks), its components, label vectors drawn at random and
rounded (ties: merges, equal labels).  Steps (median of --reps,
device-resident, activity restored between repetitions):

    observations (reduced rQ / barycentre / rLa_f, :733-766), gradient +
    most confident labels (:327-376, :525-536), capacities of one
    alpha-expansion (:542-595), expansion (:600-604), activation
    (:608-618), merge (:782-803)

A whole CP iteration runs K - 1 = 9 capacity / expansion pairs.  --cpu also
checks the GPU results of every step against the restatement at this size
(bit for bit).  Prints one JSON line.

    python tools/bench_cpgraph_simplex.py [--side 2236] [--K 10] [--reps 5] [--cpu]
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
    ap.add_argument("--side", type=int, default=2236)
    ap.add_argument("--K", type=int, default=10)
    ap.add_argument("--al", type=float, default=0.1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--block", type=int, default=10)
    ap.add_argument("--cpu", action="store_true")
    args = ap.parse_args()
    import torch
    from cp_pfdr_graph_d1_amd import pfdr
    lib = pfdr.load()
    n, K = args.side, args.K
    V = n * n
    t = time.perf_counter()
    Eu, Ev = pfdr.gen_grid_edges((n, n), 8)
    E = Eu.size
    La = np.full(E, 0.05, np.float32)
    rng = np.random.default_rng(4)
    Q = rng.random((V, K), dtype=np.float32)
    Q = (Q / Q.sum(axis=1, keepdims=True)).reshape(-1).astype(np.float32)
    b = args.block
    v = np.arange(V, dtype=np.int64)
    seg = (((v % n) // b + (v // n) // b) & 1).astype(np.uint8)
    gen_s = time.perf_counter() - t
    torch.cuda.set_device(0)
    g = pfdr.CPGraph(V, Eu, Ev, La)
    g.simplex_setup(K, args.al, Q)
    h = g.h

    def call(name, *a):
        pfdr._check(getattr(lib, name)(h, *a), name)

    # the state: one cut of the initial component, its components, rounded labels
    g.activate(seg)
    Cv, Vc, rVc = g.components()
    rV = rVc.size - 1
    P = np.round(rng.random((rV, K)), 1) + 0.05
    P[rng.random(rV) < 0.2] = P[0]
    P = (P / P.sum(axis=1, keepdims=True)).reshape(-1).astype(np.float32)
    act0 = g.active()
    eps = float(np.finfo(np.float32).eps)
    DEV = pfdr.PFDR_MEM_DEVICE
    dP = torch.empty(rV * K, dtype=torch.float32, device="cuda")
    dQr = torch.empty(rV * K, dtype=torch.float32, device="cuda")
    dL = torch.empty(rV, dtype=torch.float32, device="cuda")
    dD = torch.empty(V * K, dtype=torch.float32, device="cuda")
    dtr = torch.empty(V, dtype=torch.float32, device="cuda")
    drc = torch.empty(E, dtype=torch.float32, device="cuda")
    dseg = torch.from_numpy((rng.random(V) < 0.3).astype(np.uint8)).cuda()
    vp = lambda t_: C.c_void_p(t_.data_ptr())
    cnt = C.c_int()

    def state():
        g.set_active(act0)
        call("pfdr_cpgraph_set_components", C.c_int(rV), C.c_void_p(Cv.ctypes.data),
             C.c_void_p(Vc.ctypes.data), C.c_void_p(rVc.ctypes.data), pfdr.PFDR_MEM_HOST)
        g.rV = rV
        g.simplex_set_values(P)

    grad = lambda: call("pfdr_cpgraph_simplex_gradient", C.c_double(eps), vp(dD), None, DEV)
    steps = {
        "observations": lambda: call("pfdr_cpgraph_simplex_observations", vp(dP), vp(dQr),
                                     vp(dL), DEV),
        "gradient": grad,
        "capacities_one_expansion": lambda: call("pfdr_cpgraph_simplex_capacities", C.c_int(1),
                                                 vp(dtr), vp(drc), DEV),
        "expand": lambda: call("pfdr_cpgraph_simplex_expand", C.c_int(1), vp(dseg), DEV),
        "activate": lambda: call("pfdr_cpgraph_simplex_activate", C.byref(cnt)),
        "merge": lambda: call("pfdr_cpgraph_simplex_merge", C.c_double(eps), C.byref(cnt)),
    }
    res = {}
    for name, fn in steps.items():
        ts = []
        for r in range(args.reps + 1):
            state()
            if name in ("capacities_one_expansion", "expand", "activate"):
                grad()
            if name == "activate":
                steps["expand"]()
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            if r:
                ts.append(time.perf_counter() - t)
        res[name] = round(float(np.median(ts)) * 1e3, 3)
    it_ms = (res["gradient"] + (K - 1) * (res["capacities_one_expansion"] + res["expand"])
             + res["activate"] + res["observations"] + res["merge"])
    out = {
        "what": "simplex CP graph steps (pfdr_cpgraph_simplex_*), one MI355X, device-resident",
        "graph": "%dx%d 8-neighbour grid (V=%d, E=%d), K=%d, al=%g" % (n, n, V, E, K, args.al),
        "state": {"cut_block": b, "active_edges": int(act0.sum()), "components": rV},
        "gpu_ms": res,
        "gpu_ms_iteration_graph_steps": round(it_ms, 3),
        "iteration_note": "gradient + (K-1) x (capacities + expand) + activate + observations "
                          "+ merge; components and reduced graph are the l1 driver's "
                          "(tools/bench_cpgraph.py); the K-1 maxflows are the caller's",
        "input_generation_s": round(gen_s, 2),
    }
    if args.cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        o = oracle.Oracle("port")
        cpu, ok = {}, {}
        state()
        t = time.perf_counter()
        oP, oQ, oL = o.cp_simplex_reduced(K, args.al, Q, Vc, rVc)
        cpu["observations"] = time.perf_counter() - t
        gP, gQ, gL = g.simplex_observations()
        ok["observations"] = bool(np.array_equal(gP, oP) and np.array_equal(gQ, oQ)
                                  and np.array_equal(gL, oL))
        g.simplex_set_values(P)
        t = time.perf_counter()
        oD, orDi = o.cp_simplex_gradient(K, args.al, Q, Eu, Ev, La, act0, Cv, P, eps)
        cpu["gradient"] = time.perf_counter() - t
        gD, grDi = g.simplex_gradient(eps)
        ok["gradient"] = bool(np.array_equal(gD.view(np.uint32), oD.view(np.uint32))
                              and np.array_equal(grDi, orDi))
        Djv = np.zeros(V, np.int32)
        t = time.perf_counter()
        otr, orc = o.cp_simplex_capacities(K, 1, Eu, Ev, La, act0, Vc, rVc, orDi, Djv, oD)
        cpu["capacities_one_expansion"] = time.perf_counter() - t
        gtr, grc = g.simplex_capacities(1)
        ok["capacities"] = bool(np.array_equal(gtr.view(np.uint32), otr.view(np.uint32))
                                and np.array_equal(grc.view(np.uint32), orc.view(np.uint32)))
        sg = dseg.cpu().numpy()
        t = time.perf_counter()
        Djv = o.cp_simplex_expand(1, sg, Djv)
        cpu["expand"] = time.perf_counter() - t
        g.simplex_expand(1, sg)
        t = time.perf_counter()
        oact, on = o.cp_simplex_activate(Eu, Ev, Djv, act0)
        cpu["activate"] = time.perf_counter() - t
        gn = g.simplex_activate()
        ok["activate"] = bool(gn == on and np.array_equal(g.active(), oact))
        t = time.perf_counter()
        oact2, om = o.cp_simplex_merge(K, Eu, Ev, Cv, P, eps, oact)
        cpu["merge"] = time.perf_counter() - t
        gm = g.simplex_merge(eps)
        ok["merge"] = bool(gm == om and np.array_equal(g.active(), oact2))
        cpu_it = (cpu["gradient"] + (K - 1) * (cpu["capacities_one_expansion"] + cpu["expand"])
                  + cpu["activate"] + cpu["observations"] + cpu["merge"])
        out["cpu_ms"] = {k: round(v * 1e3, 1) for k, v in cpu.items()}
        out["cpu_ms_iteration_graph_steps"] = round(cpu_it * 1e3, 1)
        out["cpu"] = {"kind": "port", "cores": 1,
                      "note": "single-threaded C restatement (oracle/cp_graph_body.h)"}
        out["parity_full_size"] = ok
    g.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
