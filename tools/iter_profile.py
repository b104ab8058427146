"""Per-iteration durations of the two sweeps along a run, from a rocprofv3
kernel-trace CSV: medians per window of 10 launches (does an iteration's
cost depend on how far the solve has gone?)."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for pat in ("k_edge_sweep_tl", "k_vertex_sweep"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
         if pat in r["Kernel_Name"]]
    print(pat, len(d), "launches; median us per window of 10:")
    print("  " + " ".join("%.0f" % statistics.median(d[i:i + 10]) for i in range(0, len(d), 10)))
