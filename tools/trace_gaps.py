"""Per-kernel durations and the gaps between consecutive kernels of a
rocprofv3 --kernel-trace CSV (one stream's iteration chain).
Usage: python tools/trace_gaps.py <run_kernel_trace.csv> [last N dispatches]"""
import csv
import sys
from collections import defaultdict


def main(path, last=2000):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-last:]
    dur = defaultdict(list)
    gap = defaultdict(list)
    prev = None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").split("::")[-1]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[name].append(e - s)
        if prev is not None:
            gap[(prev[0], name)].append(s - prev[1])
        prev = (name, e)
    print("kernel                          n     mean_us   min_us")
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print("%-30s %5d %9.2f %8.2f" % (k, len(v), sum(v) / len(v) / 1e3, min(v) / 1e3))
    print("gap (prev -> next)                                   n   mean_us  median_us")
    for k, v in sorted(gap.items(), key=lambda kv: -len(kv[1]))[:12]:
        v = sorted(v)
        print("%-50s %5d %8.2f %8.2f" % ("%s -> %s" % k, len(v), sum(v) / len(v) / 1e3,
                                        v[len(v) // 2] / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2000)
