#!/usr/bin/env python3
"""Sweep the C3 scan's launch/loop configuration on one MI355X (interleaved
rounds in ONE process, median of R; cdna_hip_programming.md 5.4 rule 24).

usage: python tools/tune_scan.py [--gb 10] [--rounds 7] [--write] > gpurun_out/tune.json
Variant = U*100 + NT*10 + MAP (fuse-query_amd/csrc/fq_tune.hip).
"""
import argparse
import ctypes as C
import itertools
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fq_amd import ops  # noqa: E402
from fq_amd._lib import check  # noqa: E402

# the sweep kernels live in their own library (make -C fuse-query_amd tune)
_TUNE = os.path.join(ROOT, "fuse-query_amd", "lib", "libfq_tune.so")
if not os.path.exists(_TUNE):
    subprocess.run(["make", "-C", os.path.join(ROOT, "fuse-query_amd"), "tune"], check=True)
lib = C.CDLL(_TUNE)
lib.fq_tune_scan_u64.restype = C.c_int32
lib.fq_tune_scan_u64.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
lib.fq_tune_write_u64.restype = C.c_int32
lib.fq_tune_write_u64.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]


def write_sweep(args):
    """--write: fill (KIND 0, 8 B/row written) and add-one (KIND 1, 8 read + 8 written)."""
    n = int(args.gb * 1e9 / 8)
    src = ops.numbers_column(0, n)
    dst = torch.empty(n * 8, dtype=torch.uint8, device="cuda")
    stream = ops._stream()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    configs = []
    for kind, u, nt, m, g in itertools.product((0, 1), [int(x) for x in args.us.split(",")], (0, 1), (0, 2),
                                               [int(x) for x in args.grids.split(",")]):
        if m == 0 and u != 1:
            continue
        configs.append((kind * 1000 + u * 100 + nt * 10 + m, cus * g, 256))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {c: [] for c in configs}
    k = 1 << 20
    for c in configs:
        dst.zero_()
        check(lib.fq_tune_write_u64(C.c_void_p(src.ptr), C.c_void_p(dst.data_ptr()), n, c[0], c[1], c[2], stream))
        got = dst[: 8 * k].cpu().numpy().view(np.uint64)
        exp = np.arange(k, dtype=np.uint64) + (np.uint64(1) if c[0] >= 1000 else np.uint64(0))
        assert np.array_equal(got, exp), c
        tail = dst[8 * (n - 2): 8 * n].cpu().numpy().view(np.uint64)
        assert int(tail[0]) == n - 2 + (1 if c[0] >= 1000 else 0), c
    for r in range(args.rounds):
        for c in (configs if r % 2 == 0 else configs[::-1]):
            ev0.record()
            check(lib.fq_tune_write_u64(C.c_void_p(src.ptr), C.c_void_p(dst.data_ptr()), n, c[0], c[1], c[2],
                                        stream))
            ev1.record()
            ev1.synchronize()
            times[c].append(ev0.elapsed_time(ev1))
    res = []
    for c, ts in times.items():
        med = statistics.median(ts)
        nbytes = n * 8 * (2 if c[0] >= 1000 else 1)
        res.append({"variant": c[0], "kind": "add" if c[0] >= 1000 else "fill", "U": (c[0] // 100) % 10,
                    "NT": (c[0] // 10) % 10, "MAP": c[0] % 10, "grid": c[1], "block": c[2], "ms_median": med,
                    "tbps": nbytes / (med * 1e-3) / 1e12})
    res.sort(key=lambda x: (x["kind"], x["ms_median"]))
    for x in res:
        print("%-4s U=%d NT=%d MAP=%d grid=%5d  %.3f ms  %.3f TB/s" % (
            x["kind"], x["U"], x["NT"], x["MAP"], x["grid"], x["ms_median"], x["tbps"]), file=sys.stderr)
    print(json.dumps({"gb": args.gb, "rows": n, "results": res}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=10.0)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--us", default="2,4,8,16")
    ap.add_argument("--grids", default="2,4,8,16")
    ap.add_argument("--blocks", default="256,512")
    ap.add_argument("--maps", default="0,1,2,3", help="0 vector grid-stride, 1 chunked, 2 tile-contiguous, 3 XCD-partitioned")
    ap.add_argument("--write", action="store_true", help="sweep the write-side kernels instead")
    args = ap.parse_args()
    if args.write:
        return write_sweep(args)
    n = int(args.gb * 1e9 / 8)
    col = ops.numbers_column(0, n)
    parts = torch.empty(4096 * 2 * 48, dtype=torch.uint8, device="cuda")
    stream = ops._stream()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    configs = []
    maps = [int(x) for x in args.maps.split(",")]
    for u, nt, m, g, b in itertools.product([int(x) for x in args.us.split(",")], (0, 1), maps,
                                            [int(x) for x in args.grids.split(",")],
                                            [int(x) for x in args.blocks.split(",")]):
        if m == 3 and nt == 0:
            continue  # the XCD-partitioned map is built non-temporal only
        grid = cus * g * 256 // b
        configs.append((u * 100 + nt * 10 + m, grid, b))
    times = {c: [] for c in configs}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    exp_sum = (n * (n - 1) // 2) % 2**64
    # correctness of each variant once
    for c in configs:
        check(lib.fq_tune_scan_u64(C.c_void_p(col.ptr), n, c[0], c[1], c[2], C.c_void_p(parts.data_ptr()), stream))
        p = np.frombuffer(parts[: c[1] * 48].cpu().numpy().tobytes(), dtype=np.uint64).reshape(-1, 6)
        s = int(p[:, 0].sum(dtype=np.uint64))
        assert s == exp_sum and int(p[:, 1].max()) == n - 1 and int(p[:, 2].min()) == 0 \
            and int(p[:, 3].sum()) == n, c
    for r in range(args.rounds):
        order = configs if r % 2 == 0 else configs[::-1]
        for c in order:
            ev0.record()
            check(lib.fq_tune_scan_u64(C.c_void_p(col.ptr), n, c[0], c[1], c[2], C.c_void_p(parts.data_ptr()),
                                       stream))
            ev1.record()
            ev1.synchronize()
            times[c].append(ev0.elapsed_time(ev1))
    res = []
    for c, ts in times.items():
        med = statistics.median(ts)
        res.append({"variant": c[0], "U": c[0] // 100, "NT": (c[0] // 10) % 10, "MAP": c[0] % 10,
                    "grid": c[1], "block": c[2], "ms_median": med, "ms_min": min(ts),
                    "tbps": n * 8 / (med * 1e-3) / 1e12})
    res.sort(key=lambda x: x["ms_median"])
    for x in res[:25]:
        print("U=%2d NT=%d MAP=%d grid=%5d block=%3d  %.3f ms  %.3f TB/s" % (
            x["U"], x["NT"], x["MAP"], x["grid"], x["block"], x["ms_median"], x["tbps"]), file=sys.stderr)
    print(json.dumps({"gb": args.gb, "rows": n, "results": res}))


if __name__ == "__main__":
    main()
