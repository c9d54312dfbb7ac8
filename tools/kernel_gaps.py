"""Gaps between consecutive launches of one kernel in a rocprofv3 kernel
trace (csv): where a step's time goes beyond its kernels.

    python tools/kernel_gaps.py KERNEL_TRACE.csv NAME_SUBSTR [QUERY_GAP_US]

Launches of NAME_SUBSTR are split into queries wherever the gap exceeds
QUERY_GAP_US (default 2000); per query: launches, kernel sum, first start to
last end (span), span / kernel sum, and the median / max gap between two
launches with the other kernels that ran inside the gaps."""
import csv
import statistics
import sys
from collections import Counter


def main():
    path, sub = sys.argv[1], sys.argv[2]
    qgap = float(sys.argv[3]) if len(sys.argv) > 3 else 2000.0
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))]
    rows.sort()
    hits = [r for r in rows if sub in r[2]]
    queries, cur = [], []
    for r in hits:
        if cur and (r[0] - cur[-1][1]) / 1e3 > qgap:
            queries.append(cur)
            cur = []
        cur.append(r)
    if cur:
        queries.append(cur)
    for qi, q in enumerate(queries):
        ksum = sum(e - s for s, e, _ in q) / 1e3
        span = (q[-1][1] - q[0][0]) / 1e3
        gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(q, q[1:])]
        between = Counter()
        for a, b in zip(q, q[1:]):
            for s, e, n in rows:
                if s >= a[1] and e <= b[0]:
                    between[n[:40]] += 1
        print("query %d: %d launches, kernels %.3f ms, span %.3f ms (%.4f x), gap median %.1f us max %.1f us; "
              "between: %s" % (qi, len(q), ksum / 1e3, span / 1e3, span / ksum if ksum else 0,
                               statistics.median(gaps) if gaps else 0, max(gaps) if gaps else 0,
                               dict(between.most_common(4))))


if __name__ == "__main__":
    main()
