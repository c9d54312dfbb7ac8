"""Where a distributed GROUP BY step spends its time, on one rank: the plain
query (fq_engine_execute), the partial (local GROUP BY + flat rows,
fq_engine_execute_partial) and the final over `world` copies of those rows
(fq_engine_execute_final: device merge of the exchanged rows, extract, sort,
result).  python tools/group_exchange_probe.py [world] [rows]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd"))
import torch  # noqa: E402

from fq_amd import dist as fqd  # noqa: E402,F401  (prototypes)
from fq_amd._lib import check, lib  # noqa: E402
from fq_amd.engine import Engine, Result  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10**10
sql = ("SELECT number%%100000, count(number), sum(number), max(number) FROM system.numbers_mt(%d) "
       "GROUP BY number%%100000" % N).encode()
e = Engine(device=0, profile=True)
e.materialize_numbers(N)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    out = C.c_void_p()
    check(lib.fq_engine_execute(e.h, sql, C.byref(out)))
    t1 = time.perf_counter()
    lib.fq_result_free(out)
    cap = 64 << 20
    buf = C.create_string_buffer(cap)
    n = C.c_size_t(0)
    check(lib.fq_engine_execute_partial(e.h, sql, 0, 1, buf, cap, C.byref(n)))
    t2 = time.perf_counter()
    stride = n.value
    rows = (C.c_char * (stride * world))()
    for r in range(world):
        C.memmove(C.addressof(rows) + r * stride, buf, stride)
    t3 = time.perf_counter()
    out = C.c_void_p()
    check(lib.fq_engine_execute_final(e.h, sql, rows, stride, world, C.byref(out)))
    t4 = time.perf_counter()
    res = Result(out)
    t5 = time.perf_counter()
    print("execute %.1f ms | partial %.1f ms (%.1f MB of rows) | final over %d ranks %.1f ms | Result %.1f ms, %d rows"
          % ((t1 - t0) * 1e3, (t2 - t1) * 1e3, stride / 1e6, world, (t4 - t3) * 1e3, (t5 - t4) * 1e3, len(res.rows)),
          flush=True)
e.close()
