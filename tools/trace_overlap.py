"""Do two kernel families overlap in time?  Reads a rocprofv3 kernel-trace
CSV and reports, for kernels matching A (e.g. the evolution sums) the share
of their busy time spent while a kernel matching B (e.g. the sweeps) ran,
with their HW queues.  python tools/trace_overlap.py trace.csv A B"""
import csv
import sys


def intervals(rows, pat):
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"])
                  for r in rows if pat in r["Kernel_Name"])


def main(path, a, b):
    rows = list(csv.DictReader(open(path)))
    A, B = intervals(rows, a), intervals(rows, b)
    tot = sum(e - s for s, e, _ in A)
    ov = 0
    j = 0
    for s, e, _ in A:
        for s2, e2, _ in B:
            lo, hi = max(s, s2), min(e, e2)
            if hi > lo:
                ov += hi - lo
    qa = sorted({q for _, _, q in A})
    qb = sorted({q for _, _, q in B})
    print("%s: %d launches, %.3f ms busy, queues %s" % (a, len(A), tot / 1e6, qa))
    print("%s: %d launches, queues %s" % (b, len(B), qb))
    print("overlap: %.3f ms = %.1f %% of %s's busy time" % (ov / 1e6, 100.0 * ov / max(tot, 1), a))


if __name__ == "__main__":
    main(*sys.argv[1:4])
