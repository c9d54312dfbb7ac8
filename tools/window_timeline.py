"""Every kernel and HIP API call inside the WINDOW printed by
tools/readme_window.py (one query), in start order, relative to the window
start, with the thread of each API call: where a query's time goes between
`execute` being called, its first kernel, its last kernel and its return.
    python tools/window_timeline.py window.txt kernel_trace.csv hip_api_trace.csv"""
import csv
import sys

win_file, kern_csv, api_csv = sys.argv[1:4]
w = [l for l in open(win_file) if l.startswith("WINDOW")][-1].split()
t0, t1 = int(w[1]), int(w[2])
ev = []
for r in csv.DictReader(open(kern_csv)):
    s = int(r["Start_Timestamp"])
    if t0 - 50_000 <= s <= t1:
        ev.append((s, int(r["End_Timestamp"]), "K", r["Kernel_Name"][:60]))
for r in csv.DictReader(open(api_csv)):
    s = int(r["Start_Timestamp"])
    if t0 <= s <= t1:
        ev.append((s, int(r["End_Timestamp"]), "T%s" % r.get("Thread_Id", "?"), r["Function"]))
print("window %.3f ms" % ((t1 - t0) / 1e6))
for s, e, kind, name in sorted(ev):
    print("%10.1f us  +%9.1f us  %-10s %s" % ((s - t0) / 1e3, (e - s) / 1e3, kind, name))
ks = [x for x in ev if x[2] == "K"]
if ks:
    print("first kernel start +%.1f us, last kernel end +%.1f us, window end +%.1f us"
          % ((min(x[0] for x in ks) - t0) / 1e3, (max(x[1] for x in ks) - t0) / 1e3, (t1 - t0) / 1e3))
