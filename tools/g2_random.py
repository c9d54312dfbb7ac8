#!/usr/bin/env python3
"""g2's GROUP BY shape on a RANDOM column: the general-column cost of the
radix-partitioned GROUP BY (fq_group_aggregate_partitioned), where the engine's
numbers_mt blocks take the 4-byte-row path (FQ_GROUP_NARROW_ROWS) because their
values are consecutive.  A splitmix64 column (fq_fill_splitmix64) has no such
range, so its partition rows are 8 bytes: 24 B of HBM per row (read 8, blocks
written 8, blocks read 8) against the 8 B the query's achieved figure counts.

Mirrors what GroupByPartialTransform does for `SELECT x % 100000, count(x),
sum(x), max(x) ... GROUP BY x % 100000` over one 1.25e9-row partition: the same
P (2^7 bins, ~1,024 groups per bin), three equal chunks of 4.17e8 rows, one
table.  Checks a 2e7-row run against numpy first, then times --reps passes over
the 10 GB partition with HIP events (median).  One JSON line on stdout.
usage: g2_random.py [--reps 5] [--rows 1.25e9] [--narrow-iota] [--tune KNOB=V]"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fq_amd import abi, ops  # noqa: E402
from fq_amd._lib import check, lib  # noqa: E402
from fq_amd.expr import chain  # noqa: E402

D = 100_000
LOG2P = 7
U = abi.DT_UINT64
AGGS = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, U)]


def run(col, table, chunk, narrow, stream):
    key = chain(U, [("%", D)])[0]
    vals = (abi.fq_expr * abi.MAX_GROUP_AGGS)()
    lp = LOG2P | (abi.GROUP_NARROW_ROWS if narrow else 0)
    for off in range(0, col.len, chunk):
        c = abi.fq_col(C.c_void_p(col.ptr + 8 * off), min(chunk, col.len - off), U, 0)
        check(lib.fq_group_aggregate_partitioned(C.byref(table.desc), C.byref(c), None, C.byref(key), vals, lp,
                                                 table.ws.ptr, table.ws.nbytes, C.c_void_p(stream.cuda_stream)))


def new_table(chunk):
    t = ops.GroupTable(2 * D * 2, AGGS)
    t.ws = ops.Workspace(lib.fq_group_partition_workspace_bytes(chunk, LOG2P))
    return t


def check_small(narrow):
    n = 20_000_000
    col = ops.numbers_column(7_000_000_000, n) if narrow else ops.splitmix_column(0x5EED, 0, n)
    t = new_table(n)
    s = torch.cuda.current_stream()
    run(col, t, n, narrow, s)
    keys, st = t.extract()
    x = col.to_numpy()
    k = x % D
    order = np.argsort(k, kind="stable")
    ks, xs = k[order], x[order]
    uk, first = np.unique(ks, return_index=True)
    cnt = np.diff(np.append(first, len(ks)))
    sm = np.add.reduceat(xs, first)  # uint64 wraps like the device sums
    mx = np.maximum.reduceat(xs, first)
    o = np.argsort(keys)
    assert np.array_equal(keys[o], uk), "keys"
    assert np.array_equal(st[0][o], cnt) and np.array_equal(st[1][o], sm) and np.array_equal(st[2][o], mx), "states"
    return len(uk)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rows", type=float, default=1.25e9)
    ap.add_argument("--narrow-iota", action="store_true", help="a numbers_mt partition (4-byte rows) instead")
    ap.add_argument("--tune", action="append", default=[], metavar="KNOB=VALUE", help="fq_tune_set (A/B sweeps)")
    a = ap.parse_args()
    ops.require_gpu()
    for kv in a.tune:
        k, v = kv.split("=", 1)
        ops.tune_set(k.upper(), int(v))
    groups = check_small(a.narrow_iota)
    n = int(a.rows)
    chunk = ((n + 2) // 3 + 63) // 64 * 64
    col = ops.numbers_column(1_250_000_000, n) if a.narrow_iota else ops.splitmix_column(0x5EED, 0, n)
    t = new_table(chunk)
    s = torch.cuda.current_stream()
    run(col, t, chunk, a.narrow_iota, s)  # warm (kernel compile, workspace pages)
    ms = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        run(col, t, chunk, a.narrow_iota, s)
        e1.record(s)
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    ms.sort()
    med = ms[len(ms) // 2]
    print(json.dumps({
        "tool": "tools/g2_random.py", "column": "numbers_mt iota (4-byte partition rows)" if a.narrow_iota else
        "splitmix64(seed 0x5EED) random u64 (8-byte partition rows)",
        "query_shape": "GROUP BY x %% %d: count, sum, max; P = 2^%d bins, 3 chunks of %d rows" % (D, LOG2P, chunk),
        "rows": n, "groups_checked_small": groups, "tune": a.tune, "ms_per_partition": {"median": med, "min": ms[0], "max": ms[-1]},
        "algorithmic_gbps": 8 * n / (med * 1e-3) / 1e9, "frac_of_8tbs": 8 * n / (med * 1e-3) / 1e9 / 8000.0,
    }), flush=True)


if __name__ == "__main__":
    main()
