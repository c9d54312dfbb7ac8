"""Cuts a rocprofv3 csv trace (kernel + HIP API) to the WINDOW printed by
tools/readme_window.py and summarises it: API calls by total time, kernels
by count/time, and the per-thread timeline gaps."""
import collections
import csv
import sys

win_file, kern_csv = sys.argv[1], sys.argv[2]
api_csv = sys.argv[3] if len(sys.argv) > 3 else None
w = [l for l in open(win_file) if l.startswith("WINDOW")][-1].split()
t0, t1 = int(w[1]), int(w[2])
print("window %.3f ms" % ((t1 - t0) / 1e6))
ks = [r for r in csv.DictReader(open(kern_csv)) if t0 <= int(r["Start_Timestamp"]) <= t1]
agg = collections.defaultdict(lambda: [0, 0])
for r in ks:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    a = agg[r["Kernel_Name"][:60]]
    a[0] += 1
    a[1] += d
busy = sum(v[1] for v in agg.values())
print("kernels %d, busy %.3f ms" % (len(ks), busy / 1e6))
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print("  %5d %8.3f ms  %s" % (v[0], v[1] / 1e6, k))
if ks:
    first = min(int(r["Start_Timestamp"]) for r in ks)
    last = max(int(r["End_Timestamp"]) for r in ks)
    print("first kernel +%.3f ms, last kernel end +%.3f ms" % ((first - t0) / 1e6, (last - t0) / 1e6))
if api_csv:
    rows = [r for r in csv.DictReader(open(api_csv)) if t0 <= int(r["Start_Timestamp"]) <= t1]
    agg = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        a = agg[r["Function"]]
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print("HIP API calls %d" % len(rows))
    for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
        print("  %6d %9.3f ms  %s" % (v[0], v[1] / 1e6, k))
