"""fq_aggregate on one 10 GB numbers_mt partition for each aggregate mask,
interleaved (HIP events, median of 10 per round)."""
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd"))
import torch  # noqa: E402

from fq_amd import abi, ops  # noqa: E402
from fq_amd._lib import check, lib  # noqa: E402

n = 1_250_000_000
a = ops.numbers_column(0, n)
aws = ops.Workspace(lib.fq_aggregate_workspace_bytes(n))
dst = torch.empty(48, dtype=torch.uint8, device="cuda")
st = ops._stream()
S, X, N, K = abi.AGG_SUM, abi.AGG_MAX, abi.AGG_MIN, abi.AGG_COUNT
masks = {"ALL": S | X | N | K, "MAX|CNT": X | K, "SUM|CNT": S | K, "SUM": S, "CNT": K, "MAX|MIN|CNT": X | N | K}
c = a.col()


def agg(mask):
    check(lib.fq_aggregate(C.byref(c), 10000, None, None, mask, C.c_void_p(dst.data_ptr()), aws.ptr, aws.nbytes, st))


res = {k: [] for k in masks}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rnd in range(3):
    for name, m in masks.items():
        agg(m)
        ts = []
        for _ in range(10):
            e0.record()
            agg(m)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        res[name].append(statistics.median(ts))
for name, v in res.items():
    print("%-12s %s ms  -> %.0f GB/s" % (name, " ".join("%.3f" % x for x in v), 8 * n / (min(v) * 1e-3) / 1e9))
