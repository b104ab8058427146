"""Per-kernel mean of every rocprofv3 PMC counter found under a directory
(the passes of tools/counters.sh), as a markdown table: one row per kernel
whose name starts with k_, one column per counter, plus the kernel's mean
duration.  Usage: python tools/counter_summary.py <dir>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(kn):
    s = kn.split("(")[0].split("<")[0].split("::")[-1].strip()
    return s[5:] if s.startswith("void ") else s


def main(root):
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r.get("Kernel_Name", ""))
            if not k.startswith("k_"):
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"].startswith("SQ_WAVE_CYCLES"):
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    names = sorted({c for k in vals for c in vals[k]})
    print("| kernel | launches | us (profiled) | " + " | ".join(names) + " |")
    print("|---|---|---|" + "---|" * len(names))
    for k in sorted(vals):
        n = max(len(v) for v in vals[k].values())
        us = sum(dur[k]) / len(dur[k]) if dur[k] else float("nan")
        cells = []
        for c in names:
            v = vals[k].get(c)
            cells.append("%.4g" % (sum(v) / len(v)) if v else "")
        print("| %s | %d | %.1f | %s |" % (k, n, us, " | ".join(cells)))


if __name__ == "__main__":
    main(sys.argv[1])
