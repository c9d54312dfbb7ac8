"""Whole-query step time with and without the engine's per-scan timing
events, alternated in one process (python tools/step_overhead.py)."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd"))
import torch  # noqa: E402

from fq_amd.engine import OPT_PROFILE, Engine  # noqa: E402

sql = "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(10000000000)"
e = Engine(device=0, profile=True)
e.materialize_numbers(10**10)
torch.cuda.synchronize()
res = {0: [], 1: []}
for rnd in range(6):
    for prof in (1, 0) if rnd % 2 == 0 else (0, 1):
        e.set_option(OPT_PROFILE, prof)
        for _ in range(2):
            e.execute(sql)
        t = time.perf_counter()
        for _ in range(10):
            e.execute(sql)
        res[prof].append((time.perf_counter() - t) / 10 * 1e3)
for prof in (1, 0):
    print("profile=%d ms/step median %.3f  all %s" % (prof, statistics.median(res[prof]),
                                                     " ".join("%.3f" % x for x in res[prof])), flush=True)
