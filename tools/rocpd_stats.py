#!/usr/bin/env python3
"""Kernel statistics (name, calls, total/avg duration in us, percent) out of a
rocprofv3 --kernel-trace --stats SQLite database (ROCm 7.2's default output
format) into CSV, the shape of rocprofv3's kernel_stats.csv.
usage: rocpd_stats.py RESULTS.db OUT.csv"""
import csv
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
con = sqlite3.connect(db)
rows = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for r in rows:
        w.writerow(r)
print(out, len(rows), "kernels")
