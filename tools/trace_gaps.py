"""Idle time between consecutive kernels on each HW queue of a rocprofv3
kernel-trace CSV: median / mean gap per (previous kernel -> next kernel)
pair, over the steady part of the run (after the first `skip` kernels).
python tools/trace_gaps.py trace.csv [skip]"""
import collections
import csv
import statistics
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").replace("pfdr::", "")[:40]


def main(path, skip=200):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r["Queue_Id"]].append(r)
    for q, rs in sorted(byq.items()):
        gaps = collections.defaultdict(list)
        busy = collections.defaultdict(list)
        for a, b in zip(rs[skip:], rs[skip + 1:]):
            gaps[(short(a["Kernel_Name"]), short(b["Kernel_Name"]))].append(
                (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
        for r in rs[skip:]:
            busy[short(r["Kernel_Name"])].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        print("queue %s: %d kernels" % (q, len(rs)))
        for k, v in sorted(busy.items(), key=lambda kv: -sum(kv[1])):
            print("  %-42s %5d x  median %8.1f us" % (k, len(v), statistics.median(v)))
        for (a, b), v in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
            print("  gap %-28s -> %-28s %5d x  median %6.1f  mean %6.1f us"
                  % (a[:28], b[:28], len(v), statistics.median(v), statistics.mean(v)))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 200)
