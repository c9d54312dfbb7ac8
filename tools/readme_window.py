"""Runs the README LIMIT query (resident numbers_mt(1e10)) a few times and
prints the CLOCK_MONOTONIC window of the last run, so a rocprofv3
kernel/HIP-API trace of this script can be cut to that one query."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd"))
import torch  # noqa: E402

from fq_amd.engine import Engine  # noqa: E402

SQLS = {
    "readme": "select (number+1) as c1, number/2 as c2 from system.numbers_mt(10000000000) where (c1+c2+1) < 100 limit 3",
    "filter_limit": "select number, number*3 from system.numbers_mt(10000000000) where number % 1000 = 999 limit 100",
    "c3": "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(10000000000)",
    "g2": "SELECT number%100000, count(number), sum(number), max(number) FROM system.numbers_mt(10000000000) "
          "GROUP BY number%100000",
}
sql = SQLS[sys.argv[1] if len(sys.argv) > 1 else "readme"]
e = Engine(device=0, profile=int(sys.argv[2]) if len(sys.argv) > 2 else 0)  # FQ_OPT_PROFILE (bench: 2)
e.materialize_numbers(10**10)
torch.cuda.synchronize()
for _ in range(5):
    e.execute(sql)
t0 = time.monotonic_ns()
r = e.execute(sql)
t1 = time.monotonic_ns()
print("WINDOW %d %d %.3f ms" % (t0, t1, (t1 - t0) / 1e6), r.rows[:3], flush=True)
e.close()
