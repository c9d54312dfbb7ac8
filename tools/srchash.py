"""Fingerprint of the product's kernel sources (fuse-query_amd/csrc/*.hip,
*.h): a PMC traffic summary is valid only for the sources it was measured on
(tools/pmc_summary.py records it, bench.py compares it)."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_sources_sha256(root=ROOT):
    h = hashlib.sha256()
    csrc = os.path.join(root, "fuse-query_amd", "csrc")
    for f in sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h"))):
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()
