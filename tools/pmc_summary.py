#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs into profiles/<name>.json.

HBM traffic per launch follows /opt/skills/guides/MI355X_MICROARCH.md (HBM):
FETCH_SIZE is in KB and on gfx950 reads exactly half the bytes of a wide
(16 B/lane) coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE (KB) is exact for 16-B streaming stores.  Counters come from
separate --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one pass).

usage: pmc_summary.py OUT.json ROWS_PER_LAUNCH counter_collection.csv [...]
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from srchash import kernel_sources_sha256  # noqa: E402


def main():
    out, rows_per_launch, files = sys.argv[1], float(sys.argv[2]), sys.argv[3:]
    acc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName")
                ctr = r.get("Counter_Name") or r.get("Counter-Name")
                val = r.get("Counter_Value") or r.get("Counter-Value")
                if not name or not ctr or val is None:
                    continue
                acc[name][ctr].append(float(val))
    kernels = []
    for name, ctrs in sorted(acc.items()):
        k = {"name": name}
        for c, vals in ctrs.items():
            k[c + "_avg"] = sum(vals) / len(vals)
            k[c + "_dispatches"] = len(vals)
        fetch = k.get("FETCH_SIZE_avg")
        write = k.get("WRITE_SIZE_avg", 0.0)
        if fetch is not None:
            k["read_bytes_per_launch"] = 2.0 * fetch * 1024.0
            k["hbm_bytes_per_launch"] = k["read_bytes_per_launch"] + write * 1024.0
            k["rows_per_launch"] = rows_per_launch
            k["algorithmic_bytes_per_launch"] = 8.0 * rows_per_launch
            k["traffic_over_algorithmic"] = k["hbm_bytes_per_launch"] / (8.0 * rows_per_launch)
        kernels.append(k)
    json.dump({"source": files, "correction": "read = 2 x FETCH_SIZE KB (gfx950), write = WRITE_SIZE KB",
               "kernel_sources_sha256": kernel_sources_sha256(), "kernels": kernels}, open(out, "w"), indent=1)
    for k in kernels:
        print(k["name"][:90], {c: round(v, 3) for c, v in k.items() if isinstance(v, float)})


if __name__ == "__main__":
    main()
