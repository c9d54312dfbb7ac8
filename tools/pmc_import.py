#!/usr/bin/env python3
"""Copy a PMC summary from gpurun_out/ into profiles/, stamping the commit it
was measured at, the time of the import (measurement order) and the fingerprint of the query's own kernel sources (what
bench.py checks).  The box has no .git: the snapshot it ran was this
checkout's HEAD plus its working-tree changes ("-dirty"); the summary's
all-sources fingerprint must equal this tree's, or the import is refused.
usage: pmc_import.py SRC.json profiles/DST.json QUERY"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from srchash import kernel_sources_sha256  # noqa: E402

import time  # noqa: E402

src, dst, query = sys.argv[1], sys.argv[2], sys.argv[3]
d = json.load(open(src))
if d.get("kernel_sources_sha256") != kernel_sources_sha256():
    raise SystemExit("refused: %s was measured on other kernel sources than this tree's" % src)
head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True).stdout.strip()
dirty = subprocess.run(["git", "status", "--porcelain", "--", "fuse-query_amd/csrc"], capture_output=True,
                       text=True).stdout.strip()
d["measured_at_commit"] = head + ("-dirty" if dirty else "")
# measurement order for bench.py's roofline.traffic (newest measured wins, not
# the name that sorts last): the import follows the gpurun call that measured it
d["measured_at_unix"] = time.time()
d["query"] = query
d["query_sources_sha256"] = kernel_sources_sha256(query)
json.dump(d, open(dst, "w"), indent=1)
print(dst, d["measured_at_commit"], d["query_sources_sha256"][:12])
