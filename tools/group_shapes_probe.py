"""GROUP BY key shapes through SQL over resident numbers_mt(1e10): dense
(`% d`), hashed scattered keys, and run-length keys (`/ d`: consecutive rows
share a key, so a wave's 64 lanes hit one slot).  Per query: wall time and
the engine's scan-event time per 10 GB partition launch.
    python tools/group_shapes_probe.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd"))
import torch  # noqa: E402

from fq_amd.engine import Engine  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402
knobs.apply_env()

N = 10**10
KEYS = ["number%1000", "number%4093", "(number*7)%1000", "number/1000000", "number/10000000", "number/100000000",
        "(number/1000)%1000", "number%8", "(number/100)%1000", "(number/20)%1000", "(number/4)%1000", "(number/3)%1000"]
if os.environ.get("KEYS"):  # e.g. KEYS="number%1000;(number/1000)%1000"
    KEYS = os.environ["KEYS"].split(";")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
e = Engine(device=0, profile=True)
e.materialize_numbers(N)
torch.cuda.synchronize()
for k in KEYS:
    sql = "SELECT %s, count(number), sum(number), max(number) FROM system.numbers_mt(%d) GROUP BY %s" % (k, N, k)
    r = e.execute(sql)  # warm (JIT compile)
    best = None
    for _ in range(reps):
        e.reset_stats()
        t0 = time.perf_counter()
        r = e.execute(sql)
        dt = time.perf_counter() - t0
        st = e.stats()
        per = st["scan_ms"] / max(st["scan_launches"], 1)
        if best is None or dt < best[0]:
            best = (dt, per)
    print("%-22s groups %8d  query %8.2f ms  scan %7.3f ms per 10 GB launch" % (k, len(r.rows), best[0] * 1e3, best[1]),
          flush=True)
e.close()
