"""Timeline of a rocprofv3 csv trace (kernel + HIP API): every kernel and
every HIP call longer than MIN_US, in start order, over the last SPAN_MS of
the trace (the timed steps of a bench run), relative to the span start.
    python tools/trace_timeline.py kernel_trace.csv hip_api_trace.csv [SPAN_MS] [MIN_US]"""
import csv
import sys

kern_csv, api_csv = sys.argv[1], sys.argv[2]
span = float(sys.argv[3]) if len(sys.argv) > 3 else 1000.0
min_us = float(sys.argv[4]) if len(sys.argv) > 4 else 500.0
ev = []
for r in csv.DictReader(open(kern_csv)):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:50]))
for r in csv.DictReader(open(api_csv)):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A%s" % r.get("Thread_Id", ""), r["Function"]))
end = max(e[1] for e in ev)
t0 = end - int(span * 1e6)
for s, e, kind, name in sorted(ev):
    if s < t0 or (kind != "K" and (e - s) < min_us * 1e3):
        continue
    print("%10.3f %9.3f  %-8s %s" % ((s - t0) / 1e6, (e - s) / 1e6, kind, name))
