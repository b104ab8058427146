"""Effective shader clock of every sweep launch along a run: GRBM_GUI_ACTIVE
(per-XCD busy cycles, summed over the 8 XCDs) / 8 / kernel duration, from a
rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace run; medians per window of
10 launches.  python tools/clock_trace.py <dir>"""
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1]
rows = []
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if r.get("Counter_Name") == "GRBM_GUI_ACTIVE"]
tr = {}
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        tr[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
for pat in ("k_edge_sweep_tl", "k_vertex_sweep"):
    sel = sorted((int(r["Dispatch_Id"]), float(r["Counter_Value"])) for r in rows
                 if pat in r["Kernel_Name"])
    ghz, dur = [], []
    for d, cyc in sel:
        t = tr.get(str(d))
        if t:
            ghz.append(cyc / 8.0 / t / 1e9)
            dur.append(t * 1e6)
    print(pat, len(ghz), "launches")
    print("  us  " + " ".join("%.0f" % statistics.median(dur[i:i + 10]) for i in range(0, len(dur), 10)))
    print("  GHz " + " ".join("%.2f" % statistics.median(ghz[i:i + 10]) for i in range(0, len(ghz), 10)))
