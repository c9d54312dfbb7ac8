"""fq_filter_project (3/8 kept, 2 outputs) on a 10 GB column, HIP events."""
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
b = ops.splitmix_column(7, 0, n)
out, out2 = ops.empty_column(n, abi.DT_UINT64), ops.empty_column(n, abi.DT_UINT64)
pws = ops.Workspace(lib.fq_filter_project_workspace_bytes(n))
kept = C.c_int64(0)
st = ops._stream()
frac = float(os.environ.get("KEEP", "0.375"))
p38 = predicate(abi.DT_UINT64, [], "<", min(int(frac * 2**64), 2**64 - 1))
nout = int(os.environ.get("NOUT", "2"))
vals = (abi.fq_expr * 2)(chain(abi.DT_UINT64, [("+", 1)])[0], chain(abi.DT_UINT64, [("/", 2)])[0])
outs = (C.c_void_p * 2)(out.ptr, out2.ptr)
bc = b.col()


def project():
    check(lib.fq_filter_project(C.byref(bc), C.byref(p38), vals, nout, outs, C.byref(kept), pws.ptr, pws.nbytes, st))
    if ops.tune_get("SELECT_DEBUG"):  # the library keeps the counters; the tool prints them
        h = ops.tune_select_counters()
        t = max(h[0], 1)
        print("[select-debug] tiles %d polls/tile %.2f windows/tile %.2f | per tile (cycles): ticket %.0f "
              "load+pred %.0f lookback %.0f store %.0f | wg life %.1f us" %
              (h[0], h[1] / t, h[7] / t, h[3] / t, h[4] / t, h[2] / t, h[5] / t, h[12] / 100.0), flush=True)


project()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(10):
    e0.record()
    project()
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1))
ms = statistics.median(ts)
nb = 8 * n + nout * 8 * kept.value
print("keep=%s WG/CU=%s nout=%d: %.3f ms, %.0f GB/s algorithmic, kept %d" % (os.environ.get("KEEP", "0.375"), os.environ.get("FQ_TUNE_SELECT_WG_PER_CU", "8"), nout, ms,
                                                                     nb / ms / 1e6, kept.value), flush=True)
