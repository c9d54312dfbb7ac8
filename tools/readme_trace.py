"""Latency of the README LIMIT query over resident numbers_mt(1e10) with 1
and 8 device queues (run under rocprofv3 --kernel-trace for the timeline)."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd"))
import torch  # noqa: E402,F401

from fq_amd.engine import OPT_STREAMS, Engine  # noqa: E402

sql = ("select (number+1) as c1, number/2 as c2 from system.numbers_mt(10000000000) "
       "where (c1+c2+1) < 100 limit 3")
e = Engine(device=0)
e.materialize_numbers(10**10)
torch.cuda.synchronize()
for streams in (1, 8, 1, 8):
    e.set_option(OPT_STREAMS, streams)
    ts = []
    for i in range(6):
        t = time.perf_counter()
        r = e.execute(sql)
        ts.append((time.perf_counter() - t) * 1e3)
    print("streams=%d median %.3f ms  all %s" % (streams, statistics.median(ts[1:]), " ".join("%.2f" % x for x in ts)),
          r.rows, flush=True)
e.close()
