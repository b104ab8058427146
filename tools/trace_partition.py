"""Host cost of a partitioned iteration (Next 4(b)).

Runs the headline graph split over N loopback ranks (N threads on this GPU,
the same session code as one RCCL process per GPU) for K untracked
iterations after a warm-up, and reports each rank's wall time.  Under
`rocprofv3 --hip-trace --kernel-trace` the HIP API records let
`python tools/trace_partition.py --analyse <dir>` split every rank thread's
host time into API calls (launches, event records / waits, copies) per
iteration -- the host enqueue cost per rank-iteration that has to stay below
the rank's GPU time per iteration for the driver's N-GPU run to stay
GPU-bound.

    python tools/trace_partition.py [N] [K] [--shape 250x200x200]
    python tools/trace_partition.py --analyse <rocprof output dir> [K]
"""
import csv
import glob
import os
import sys
import time
from collections import defaultdict

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def run(N, K, shape):
    import ctypes as C
    import threading
    from cp_pfdr_graph_d1_amd import partition as P
    from cp_pfdr_graph_d1_amd import pfdr
    import workloads

    class WL(workloads.Headline):
        SHAPE = shape

    wl = WL()
    inps = [wl.inputs(r, N, True) for r in range(N)]
    lib = pfdr.load()
    hub = C.c_void_p()
    pfdr._check(lib.pfdr_loopback_create(C.byref(hub), C.c_int(N)), "pfdr_loopback_create")
    warm = 10
    out = [None] * N
    bar = threading.Barrier(N)

    def main(r):
        inp = inps[r]
        s = pfdr.Session(wl.kind, wl.dtype, inp["V"], inp["E"], itMax=warm + K, **inp["kw"],
                         nranks=N, rank=r, comm=hub.value, comm_kind=P.COMM_LOOPBACK,
                         vtx_begin=inp["vtx_begin"], e_offset=inp["e_offset"])
        s.run(warm)
        s.sync()
        bar.wait()
        t0 = time.perf_counter()
        s.run(K)
        t1 = time.perf_counter()
        s.sync()
        t2 = time.perf_counter()
        out[r] = (inp["V"], inp["E"], s.query("ghosts"), s.query("interior_edges"),
                  t1 - t0, t2 - t0)
        s.close()

    th = [threading.Thread(target=main, args=(r,)) for r in range(N)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    lib.pfdr_loopback_destroy(hub)
    print("graph %s, N = %d loopback ranks on one GPU, K = %d iterations" % (
        "x".join(map(str, shape)), N, K))
    print("rank        V          E   ghosts  interior_E   enqueue_ms  wall_ms  enqueue_us/it")
    for r, (V, E, g, ie, te, tw) in enumerate(out):
        print("%4d %9d %10d %8d %11d %11.2f %8.2f %10.1f" % (r, V, E, g, ie, te * 1e3, tw * 1e3,
                                                               te / K * 1e6))


def analyse(d, K):
    """per host thread: HIP API time inside the timed run() calls"""
    files = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    by_tid = defaultdict(list)
    for r in rows:
        by_tid[r.get("Thread_Id")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                           r["Function"]))
    print("thread          api_calls  launches  api_ms  api_us_per_it (last %d its window)" % K)
    for tid, ev in sorted(by_tid.items(), key=lambda kv: -len(kv[1])):
        ev.sort()
        launches = [e for e in ev if "Launch" in e[2]]
        if len(launches) < 4 * K:
            continue
        # the window of the timed iterations: the last 4K+ launches of the thread
        # (up to the last launch: the session's teardown frees are not per iteration)
        lo, hi = launches[-4 * K][0], launches[-1][1]
        win = [e for e in ev if lo <= e[0] <= hi]
        api = sum(e[1] - e[0] for e in win)
        fn = defaultdict(float)
        for e in win:
            fn[e[2]] += (e[1] - e[0]) / 1e3
        top = ", ".join("%s %.0f" % (k, v) for k, v in sorted(fn.items(), key=lambda kv: -kv[1])[:5])
        print("%-14s %9d %9d %7.2f %9.1f   [%s us]" % (tid, len(win), len(launches), api / 1e6,
                                                     api / 1e3 / K, top))


if __name__ == "__main__":
    a = sys.argv[1:]
    if a and a[0] == "--analyse":
        analyse(a[1], int(a[2]) if len(a) > 2 else 40)
    else:
        shape = (250, 200, 200)
        if "--shape" in a:
            i = a.index("--shape")
            shape = tuple(int(x) for x in a[i + 1].split("x"))
            del a[i:i + 2]
        run(int(a[0]) if a else 8, int(a[1]) if len(a) > 1 else 40, shape)
