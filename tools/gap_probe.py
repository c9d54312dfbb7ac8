"""Back-to-back fq_aggregate launches on one stream: total time of 8 scans of
one 10 GB partition each, with the 48-byte state written to device memory vs
to mapped pinned host memory (what the engine does), and per-launch HIP-event
pairs vs none.  Shows what the boundary between two scans costs."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd"))
import torch  # noqa: E402

from fq_amd import ops  # noqa: E402
from fq_amd._lib import check, lib  # noqa: E402

n = 1_250_000_000
cols = [ops.numbers_column(i * n, n) for i in range(8)]
ws = ops.Workspace(lib.fq_aggregate_workspace_bytes(n))
dev_out = torch.empty(48 * 8, dtype=torch.uint8, device="cuda")
host_out = torch.empty(48 * 8, dtype=torch.uint8).pin_memory()
hip = C.CDLL("libamdhip64.so.7")
dptr = C.c_void_p()
assert hip.hipHostGetDevicePointer(C.byref(dptr), C.c_void_p(host_out.data_ptr()), 0) == 0
s = torch.cuda.current_stream()


# events: 0 none, 1 torch (hipEventDefault), 2 hipEventDisableSystemFence,
# 3 hipEventReleaseToDevice -- what a timing pair costs between two scans
FLAGS = {2: 0x20000000, 3: 0x40000000}
_pool = {k: [] for k in FLAGS}


def hip_event(kind, i):
    pool = _pool[kind]
    while len(pool) <= i:
        e = C.c_void_p()
        assert hip.hipEventCreateWithFlags(C.byref(e), C.c_uint(FLAGS[kind])) == 0
        pool.append(e)
    return pool[i]


def rec(kind, i):
    e = hip_event(kind, i)
    assert hip.hipEventRecord(e, C.c_void_p(s.cuda_stream)) == 0
    return e


def run(to_host, events):
    evs = []
    for i, c in enumerate(cols):
        if events == 1:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
        elif events > 1:
            e0 = rec(events, 2 * i)
        out = (dptr.value + 48 * i) if to_host else (dev_out.data_ptr() + 48 * i)
        cc = c.col()
        check(lib.fq_aggregate(C.byref(cc), 10000, None, None, 0xF, C.c_void_p(out), ws.ptr, ws.nbytes,
                               C.c_void_p(s.cuda_stream)))
        if events == 1:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(s)
            evs.append((e0, e1))
        elif events > 1:
            evs.append((e0, rec(events, 2 * i + 1)))


for to_host in (0, 1):
    for events in (0, 1, 2, 3):
        for _ in range(2):
            run(to_host, events)
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(10):
            a.record(s)
            run(to_host, events)
            b.record(s)
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        print("state->%s events=%d: 8 scans %.3f ms (median of 10), %.1f us per boundary beyond 8 x 1.384"
              % ("host" if to_host else "device", events, ts[5], (ts[5] - 8 * 1.384) / 8 * 1e3), flush=True)
