"""GROUP BY throughput vs number of groups and aggregates over one numbers_mt
partition (python tools/groupby_sweep.py [rows] [mods] [naggs] [launches] [log2_parts]); one line per shape.
log2_parts > 0 runs the radix-partitioned path (fq_group_aggregate_partitioned);
"auto" picks ceil(log2(groups / 1024)) in [1, 8] for groups above 3,072 (as the engine does).
With launches L > 1 the column is aggregated L times into one table (as the
engine does for the partitions of one query); the time is per launch."""
import sys, os, ctypes as C, statistics
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd"))
import torch
from fq_amd import abi, ops
from fq_amd._lib import check, lib
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402
knobs.apply_env()
from fq_amd.expr import chain
U = abi.DT_UINT64
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_250_000_000
# RANDOM=1: a splitmix64 column (keys in random order) instead of numbers_mt's iota
a = ops.splitmix_column(0x5EED, 0, n) if os.environ.get("RANDOM") == "1" else ops.numbers_column(0, n)
st = ops._stream()
def timed(fn, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(); torch.cuda.synchronize(); ts = []
    for _ in range(reps):
        e0.record(); fn(); e1.record(); e1.synchronize(); ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)
MODS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [8, 64, 1000, 4096, 100000]
NAGGS = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 3]
L = int(sys.argv[4]) if len(sys.argv) > 4 else 1
PARTS = sys.argv[5] if len(sys.argv) > 5 else "0"


def log2_parts(groups):
    if PARTS != "auto":
        return int(PARTS)
    if groups <= 3072:
        return 0
    p = 1
    while p < 8 and (groups >> p) > 1024:
        p += 1
    return p
for mod in MODS:
    for naggs in NAGGS:
        key, _ = chain(U, [("%", mod)])
        aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, U)][:naggs]
        gt = ops.GroupTable(max(64, 4 * min(mod, n)), aggs)
        lp = log2_parts(min(mod, n))
        if L == 1:
            def f():
                check(lib.fq_group_table_init(C.byref(gt.desc), st)); gt.aggregate(a, key=key, log2_parts=lp)
            ms = timed(f)
            print("mod=%6d aggs=%d parts=2^%d  %.3f ms  %.1f G rows/s" % (mod, naggs, lp, ms, n / ms / 1e6), flush=True)
            continue
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(L + 1)]
        per = []
        for rep in range(3):
            check(lib.fq_group_table_init(C.byref(gt.desc), st))
            ev[0].record()
            for i in range(L):
                gt.aggregate(a, key=key, log2_parts=lp)
                ev[i + 1].record()
            ev[L].synchronize()
            per.append([ev[i].elapsed_time(ev[i + 1]) for i in range(L)])
        first = statistics.median(p[0] for p in per)
        rest = statistics.median(statistics.mean(p[1:]) for p in per)
        print("mod=%6d aggs=%d parts=2^%d launches=%d  first %.3f ms, then %.3f ms/launch (%.1f G rows/s)"
              % (mod, naggs, lp, L, first, rest, n / rest / 1e6), flush=True)
