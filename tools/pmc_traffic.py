"""Summarise rocprofv3 PMC passes into per-launch HBM traffic per kernel.

Per MI355X_MICROARCH.md §HBM (gfx950): FETCH_SIZE (KiB) reads exactly half
the bytes of a wide coalesced streaming read, so read bytes = 2 x FETCH_SIZE
x 1024; WRITE_SIZE (KiB) reads the bytes of 16-B-per-lane streaming stores
exactly.  The sweeps stream 16 B per lane on every array, so the x2
correction applies to their streams; gathers are uncalibrated (the guide:
ratios between variants of one kernel are unaffected).  Infinity-Cache hits
are counted by these counters, not excluded.
Usage: python tools/pmc_traffic.py <dir with fetch/ and write/> [workload E V]
(the summary goes to stdout; bench.py reads profiles/pmc/<workload>.json)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def counter(dirname, name):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != name:
                continue
            kn = r.get("Kernel_Name", "")
            short = kn.split("(")[0].split("<")[0].split("::")[-1].strip()
            if short.startswith("void "):
                short = short[5:]
            vals[short].append(float(r["Counter_Value"]))
    return vals


def bench_size(root):
    """(E, V) of the run, from the bench line the profiled command printed
    (fetch.log / stats.log in the profile directory), or None"""
    import re
    for name in ("fetch.log", "write.log", "stats.log"):
        try:
            t = open(os.path.join(root, name)).read()
        except OSError:
            continue
        e = re.search(r'"E_per_gpu": (\d+)', t)
        v = re.search(r'"V_per_gpu": (\d+)', t)
        if e and v:
            return int(e.group(1)), int(v.group(1))
    return None


def main(root, workload="headline", E=60000000, V=10000000):
    size = bench_size(root)  # the run's own size wins over the defaults
    if size:
        E, V = size
    fetch = counter(os.path.join(root, "fetch"), "FETCH_SIZE")
    write = counter(os.path.join(root, "write"), "WRITE_SIZE")
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from kernel_hash import kernel_source_sha256
    from workloads import WORKLOADS
    solver = WORKLOADS[workload].pmc if workload in WORKLOADS else "quadratic"
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, kernel "
                     "trace only), bench.py --workload %s" % workload,
           "workload": workload, "workload_E": E, "workload_V": V,
           "solver_sources": solver,
           "kernel_source_sha256": kernel_source_sha256(solver), "kernels": {}}
    for k in sorted(set(fetch) & set(write)):
        if not k.startswith("k_"):
            continue
        f, w = fetch[k], write[k]
        fk, wk = sum(f) / len(f), sum(w) / len(w)
        rd = 2.0 * fk * 1024.0
        wr = wk * 1024.0
        out["kernels"][k] = {"FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
                             "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                             "hbm_bytes_per_launch": rd + wr, "launches": [len(f), len(w)]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], *(a[1:2] + [int(x) for x in a[2:4]]))
