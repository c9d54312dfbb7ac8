"""Filtered-sum (block-mode) scan on one 10 GB partition, HIP events (FQ_BLOCK_U sweep)."""
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd"))
import torch  # noqa: E402

from fq_amd import abi, ops  # noqa: E402
from fq_amd._lib import check, lib  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402
knobs.apply_env()
from fq_amd.expr import chain, predicate  # noqa: E402

n = 1_250_000_000
a = ops.numbers_column(0, n)
aws = ops.Workspace(lib.fq_aggregate_workspace_bytes(n))
dst = torch.empty(48, dtype=torch.uint8, device="cuda")
st = ops._stream()
c = a.col()
v, _ = chain(abi.DT_UINT64, [("+", 1)])
p = predicate(abi.DT_UINT64, [("%", 8)], "<", 3)


def agg():
    check(lib.fq_aggregate(C.byref(c), 10000, C.byref(p), C.byref(v), abi.AGG_SUM, C.c_void_p(dst.data_ptr()),
                           aws.ptr, aws.nbytes, st))


agg()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(15):
    e0.record()
    agg()
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1))
ms = statistics.median(ts)
print("FQ_BLOCK_U=%s: %.3f ms, %.0f GB/s" % (os.environ.get("FQ_TUNE_BLOCK_U", "8"), ms, 8 * n / ms / 1e6), flush=True)
