#!/usr/bin/env python3
"""GROUP BY key shapes over resident numbers_mt(N) through the engine: the g2
key (number % 100000: consecutive keys, so a wave's rows share a range bin)
against keys whose consecutive rows land in different bins
((number * 7919) % 100000, (number / 3) % 100000, number % 99991).  Each query
runs --reps times after one warm run; the median wall ms and the result's group
count are printed as one JSON line per shape.
usage: group_key_shapes.py [--rows 1e10] [--reps 3]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))

from fq_amd import ops  # noqa: E402
from fq_amd.engine import Engine  # noqa: E402

SHAPES = ["number % 100000", "(number * 7919) % 100000", "(number / 3) % 100000", "number % 99991"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e10)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    ops.require_gpu()
    n = int(a.rows)
    e = Engine()
    e.materialize_numbers(n)
    try:
        for k in SHAPES:
            sql = "SELECT %s, count(number), sum(number), max(number) FROM system.numbers_mt(%d) GROUP BY %s" % (k, n, k)
            r = e.execute(sql)  # warm: kernel compile, workspace pages
            ms = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                r = e.execute(sql)
                ms.append((time.perf_counter() - t0) * 1e3)
            ms.sort()
            total = sum(row[1] for row in r.rows)
            print(json.dumps({"key": k, "rows": n, "groups": len(r.rows), "count_total": total,
                              "ms_median": ms[len(ms) // 2], "ms": ms}), flush=True)
            assert total == n, "counts must add up to the rows"
    finally:
        e.release_numbers()
        e.close()


if __name__ == "__main__":
    main()
