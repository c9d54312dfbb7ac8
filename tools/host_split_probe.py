"""Host/device split of one query: time in fq_engine_execute (C++ pipeline:
planning, kernels, AggregateFinal, result assembly) vs building the Python
Result from the fq_result handle, and the engine's own scan-event time.
    python tools/host_split_probe.py g2|g1|c3 [reps]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd"))
import torch  # noqa: E402

from fq_amd._lib import check, lib  # noqa: E402
from fq_amd.engine import Engine, Result  # noqa: E402

SQLS = {
    "c3": "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(10000000000)",
    "g1": "SELECT number%1000, count(number), sum(number), max(number) FROM system.numbers_mt(10000000000) "
          "GROUP BY number%1000",
    "g2": "SELECT number%100000, count(number), sum(number), max(number) FROM system.numbers_mt(10000000000) "
          "GROUP BY number%100000",
}
q = sys.argv[1] if len(sys.argv) > 1 else "g2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
e = Engine(device=0, profile=True)
e.materialize_numbers(10**10)
torch.cuda.synchronize()
sql = SQLS[q].encode()
for i in range(reps + 2):
    e.reset_stats()
    out = C.c_void_p()
    t0 = time.perf_counter()
    check(lib.fq_engine_execute(e.h, sql, C.byref(out)))
    t1 = time.perf_counter()
    r = Result(out)
    t2 = time.perf_counter()
    st = e.stats()
    if i >= 2:
        print("%s: execute %.2f ms (scan events %.2f ms, plan %.3f ms, first launch %.3f ms), Result %.2f ms, %d rows"
              % (q, (t1 - t0) * 1e3, st["scan_ms"], st["plan_ms"], st["first_launch_ms"], (t2 - t1) * 1e3,
                 len(r.rows)), flush=True)
e.close()
