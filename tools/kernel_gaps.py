"""Gaps between consecutive launches of one kernel in a rocprofv3 kernel
trace (csv): where a step's time goes beyond its kernels.

    python tools/kernel_gaps.py KERNEL_TRACE.csv NAME_SUBSTR [QUERY_GAP_US]
    python tools/kernel_gaps.py KERNEL_TRACE.csv NAME_SUBSTR --window COUNT SKIP_LAST

The second form takes COUNT launches ending SKIP_LAST launches before the
last (bench.py's timed steps: K x launches per step, followed by one checked
step) and prints their busy time (the union of their intervals) per launch --
the rocprof figure to hold beside bench.py's span per launch when launches on
two queues overlap (each kernel's own duration then counts the other's share).

Launches of NAME_SUBSTR are split into queries wherever the gap exceeds
QUERY_GAP_US (default 2000); per query: launches, kernel sum, first start to
last end (span), span / kernel sum, the union of the launches' intervals (the
time at least one ran: launches on two queues overlap, so the span / union is
what a query's launches cost beyond their busy time), and the median / max
gap between two launches with the other kernels that ran inside the gaps."""
import csv
import json
import statistics
import sys
from collections import Counter


def union_us(q):
    """us during which at least one of the (start ns, end ns, name) launches ran"""
    q = sorted(q)
    union, lo, hi = 0, q[0][0], q[0][1]
    for s, e, _ in q[1:]:
        if s > hi:
            union, lo, hi = union + hi - lo, s, e
        else:
            hi = max(hi, e)
    return (union + hi - lo) / 1e3


def main():
    path, sub = sys.argv[1], sys.argv[2]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))]
    rows.sort()
    hits = [r for r in rows if sub in r[2]]
    if len(sys.argv) > 3 and sys.argv[3] == "--window":
        count, skip = int(sys.argv[4]), int(sys.argv[5])
        w = hits[len(hits) - skip - count:len(hits) - skip]
        busy = union_us(w)
        print(json.dumps({"trace": path, "kernel": sub, "launches": len(w), "busy_union_ms": busy / 1e3,
                          "busy_ms_per_launch": busy / 1e3 / len(w),
                          "kernel_ms_mean": sum(e - s for s, e, _ in w) / 1e6 / len(w),
                          "span_ms": (max(e for _, e, _ in w) - w[0][0]) / 1e6}))
        return
    qgap = float(sys.argv[3]) if len(sys.argv) > 3 else 2000.0
    queries, cur = [], []
    for r in hits:
        if cur and (r[0] - max(e for _, e, _ in cur)) / 1e3 > qgap:
            queries.append(cur)
            cur = []
        cur.append(r)
    if cur:
        queries.append(cur)
    for qi, q in enumerate(queries):
        ksum = sum(e - s for s, e, _ in q) / 1e3
        span = (max(e for _, e, _ in q) - q[0][0]) / 1e3
        union = union_us(q)
        gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(q, q[1:])]
        between = Counter()
        for a, b in zip(q, q[1:]):
            for s, e, n in rows:
                if s >= a[1] and e <= b[0]:
                    between[n[:40]] += 1
        print("query %d: %d launches, kernels %.3f ms, span %.3f ms (%.4f x), busy (union) %.3f ms (span %.4f x), "
              "gap median %.1f us max %.1f us; between: %s" % (
                  qi, len(q), ksum / 1e3, span / 1e3, span / ksum if ksum else 0, union / 1e3,
                  span / union if union else 0,
                               statistics.median(gaps) if gaps else 0, max(gaps) if gaps else 0,
                               dict(between.most_common(4))))


if __name__ == "__main__":
    main()
