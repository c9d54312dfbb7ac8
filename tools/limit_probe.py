"""Latency of LIMIT queries over numbers_mt(1e10) through the engine (row
pipelines stream morsels; a satisfied LIMIT stops the scan).
python tools/limit_probe.py [KNOB=V ...]  (launch-shape knobs through fq_tune_set)"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd"))
import torch  # noqa: E402,F401

from fq_amd import ops  # noqa: E402
from fq_amd.engine import Engine  # noqa: E402

for kv in sys.argv[1:]:
    k, v = kv.split("=", 1)
    ops.tune_set(k.upper(), int(v))

QS = {
    "readme": "select (number+1) as c1, number/2 as c2 from system.numbers_mt(10000000000) "
              "where (c1+c2+1) < 100 limit 3",
    "limit5": "SELECT number FROM system.numbers_mt(10000000000) LIMIT 5",
    "filter_limit": "SELECT number, number*3 FROM system.numbers_mt(10000000000) WHERE number % 1000 = 999 LIMIT 100",
}
out = {}
for resident in (False, True):
    e = Engine(device=0)
    if resident:
        e.materialize_numbers(10**10)
        torch.cuda.synchronize()
    for name, sql in QS.items():
        e.execute(sql)
        ts = []
        for _ in range(10):
            t = time.perf_counter()
            r = e.execute(sql)
            ts.append((time.perf_counter() - t) * 1e3)
        out["%s%s" % (name, "_resident" if resident else "")] = {"ms_median": statistics.median(ts), "rows": len(r.rows)}
        print(name, "resident" if resident else "generated", "%.3f ms" % statistics.median(ts), r.rows[:3], flush=True)
    e.close()
print(json.dumps({"tune": sys.argv[1:], **out}))
