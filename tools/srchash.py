"""Fingerprint of the product's kernel sources: a PMC traffic summary is
valid only for the sources it was measured on (tools/pmc_summary.py records
the fingerprint of every kernel source, tools/pmc_import.py adds the one of the
query's own sources, bench.py compares that one)."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# the sources each bench query's kernels are built from (csrc/ relative);
# fq_knobs.cpp holds every launch-shape default
_SCAN = ["fq_aggregate.hip", "fq_scan.h", "fq_device.h", "fq_knobs.cpp"]
_JIT = ["fq_jit.hip", "fq_scan.h", "fq_device.h", "fq_knobs.cpp"]
QUERY_SOURCES = {
    "c2": _SCAN, "c3": _SCAN, "max": _SCAN, "avg": _SCAN,
    "c4": _SCAN + _JIT, "max1": _SCAN + _JIT, "c4s": _SCAN + _JIT,
    "p1": _JIT + ["fq_filter.hip"],
    "g1": _JIT + ["fq_groupby.hip"], "g2": _JIT + ["fq_groupby.hip"],
}


def kernel_sources_sha256(query=None, root=ROOT):
    """sha256 over the query's kernel sources (every csrc/*.hip and *.h when
    query is None)."""
    csrc = os.path.join(root, "fuse-query_amd", "csrc")
    if query is None:
        files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h")))
    else:
        files = sorted(os.path.join(csrc, f) for f in set(QUERY_SOURCES[query]))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()
