#!/usr/bin/env python3
"""One-off: give the PMC summaries imported before tools/pmc_import.py stamped
`measured_at_unix` the committer time of their `measured_at_commit` (git log
order = measurement order), so bench.py can order them by when they were
measured rather than by file name.  Files already stamped are left alone."""
import glob
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_*.json"))):
    d = json.load(open(f))
    if d.get("measured_at_unix") or not d.get("measured_at_commit"):
        continue
    c = d["measured_at_commit"].replace("-dirty", "")
    t = subprocess.run(["git", "show", "-s", "--format=%ct", c], capture_output=True, text=True, cwd=ROOT)
    if t.returncode:
        print("skip", f, "(commit %s not found)" % c)
        continue
    d["measured_at_unix"] = float(t.stdout.strip())
    d["measured_at_unix_source"] = "committer time of measured_at_commit (backfilled)"
    json.dump(d, open(f, "w"), indent=1)
    print(os.path.basename(f), c, int(d["measured_at_unix"]))
