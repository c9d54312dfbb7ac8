"""One rank of a multi-GPU C3 step, rehearsed on one GPU.

Rank R of G owns numbers_mt partitions [8R/G, 8(R+1)/G) -- at --rows 1e10 and
G = 8 one 1.25e9-row partition: the strong-scaling 8-GPU case.  Each timed
step is ONE library call, fq_engine_execute_exchange_row: the partial over
R's shard (its fused scan), the exchange through the real RCCL all-reduce of
a [G x row] buffer over the library's world-1 communicator, and
AggregateFinal over G rows -- the peers' rows copied from R's by a native
callback (tests/native/fq_loopback_peers.c), as if they arrived at once.
What the rehearsal cannot show: the wait for slower peers and the xGMI hops
of a real world-G ring (tens of microseconds for 104-byte rows).

Reports the step against the scan span (the engine's FQ_OPT_PROFILE 2 span of
its scans): step_over_scan is what the per-rank fixed costs add.

python tools/rank_rehearsal.py [--rank 7] [--world 8] [--rows 1e10] [--steps 30]
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=7)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rows", type=float, default=1e10)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle-s", type=float, default=3.0)
    args = ap.parse_args()
    bench._load_runtime()
    torch, abi, fqd = bench.torch, bench.abi, bench.fqd
    from fq_amd._lib import check, lib
    from fq_amd.engine import PROFILE_SPAN, Engine
    n = int(args.rows)
    sql = bench.QUERIES["c3"].format(N=n)
    mine = bench.shard(bench.generate_parts(n), args.rank, args.world)
    rows = sum(bench.stream_rows(b, e) for _, b, e in mine)
    # the final over G copies of rank R's states: its sum G times (wrapping
    # u64, as the reference's Sum state adds) over its count G times
    s = sum((b + e) * (e - b + 1) // 2 for _, b, e in mine)
    cnt = sum(e - b + 1 for _, b, e in mine)
    g = args.world
    expect = [(g * s % 2**64) // (g * cnt), max(e for _, _, e in mine), min(b for _, b, _ in mine)]

    eng = Engine(device=0, profile=PROFILE_SPAN)
    eng.materialize_numbers(n, args.rank, args.world)
    torch.cuda.synchronize()
    comm = fqd.RcclComm.single(0)

    class Loopback(C.Structure):
        _fields_ = [("comm", C.c_void_p), ("rank", C.c_int32), ("world", C.c_int32)]

    lb = C.CDLL(os.path.join(ROOT, "fuse-query_amd", "lib", "libfq_loopback.so"))
    fn = fqd.ALLREDUCE_FN(("fq_loopback_allreduce", lb))  # a native function pointer: no Python per step
    user = Loopback(comm.h.value, args.rank, args.world)
    sql_b = sql.encode()
    row = (abi.fq_value * 8)()
    ncols = C.c_int32(0)
    call = lib.fq_engine_execute_exchange_row

    def step():
        st = call(eng.h, sql_b, args.rank, args.world, fn, C.byref(user), row, 8, C.byref(ncols))
        if st:
            check(st)

    t_end = time.perf_counter() + args.settle_s
    while time.perf_counter() < t_end:
        step()
    for _ in range(args.warmup):
        step()
    got = [v.bits for v in row[:ncols.value]]
    if got != expect:
        raise SystemExit("PARITY FAILURE: got %r expected %r" % (got, expect))
    eng.reset_stats()
    per = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = time.perf_counter()
        step()
        per.append(time.perf_counter() - a)
    dt = (time.perf_counter() - t0) / args.steps
    got = [v.bits for v in row[:ncols.value]]
    assert got == expect
    st = eng.stats()
    scan_ms = st["scan_ms"] / args.steps
    launches = max(st["scan_launches"], 1)
    out = {
        "what": "rank %d of %d of the C3 step, rehearsed on one GPU (tools/rank_rehearsal.py)" % (args.rank, args.world),
        "workload": sql, "rows_on_rank": rows, "partitions_on_rank": len(mine),
        "step_ms": dt * 1e3, "step_ms_median": statistics.median(per) * 1e3,
        "scan_span_ms": scan_ms, "step_over_scan": dt * 1e3 / scan_ms if scan_ms else None,
        "scan_frac": (st["scan_bytes"] / launches) / ((st["scan_ms"] / launches) * 1e-3) / 1e9 / bench.HBM_PEAK_GBPS,
        "partial_ms": st["partial_ms"] / args.steps, "exchange_ms": st["exchange_ms"] / args.steps,
        "final_ms": st["final_ms"] / args.steps, "exchange_rounds": st["exchange_rounds"] / args.steps,
        "exchange_bytes": st["exchange_bytes"] / args.steps,
        "result": got, "expected_rank_aggregates": expect, "steps": args.steps,
        "transport": "RCCL all-reduce of the [%d x row] buffer over the world-1 communicator; peers' rows copied "
                     "from this rank's (tests/native/fq_loopback_peers.c)" % args.world,
    }
    print(json.dumps(out), flush=True)
    comm.close()
    eng.close()


if __name__ == "__main__":
    main()
