#!/usr/bin/env python3
"""Copy a PMC summary from gpurun_out/ into profiles/, stamping the commit it
was measured at (the box has no .git: the snapshot sent was this checkout's
HEAD plus its working-tree changes, recorded as "-dirty").
usage: pmc_import.py SRC.json profiles/DST.json"""
import json
import subprocess
import sys

src, dst = sys.argv[1], sys.argv[2]
d = json.load(open(src))
head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True).stdout.strip()
dirty = subprocess.run(["git", "status", "--porcelain", "--", "fuse-query_amd/csrc"], capture_output=True,
                       text=True).stdout.strip()
d["measured_at_commit"] = head + ("-dirty" if dirty else "")
json.dump(d, open(dst, "w"), indent=1)
print(dst, d["measured_at_commit"], d.get("kernel_sources_sha256", "")[:12])
