"""BASELINE configs[4] (C5) end to end on the HIP path:

    SELECT sum(number)/count(number), max(number), min(number)
    FROM system.numbers_mt(80000000000)

8 partitions of 1e10 rows (numbers_table.rs:29-55), each read as the
reference's 10,000-row blocks (numbers_stream.rs:27-62) -- here generated on
the GPU in FQ_OPT_CHUNK_ROWS pieces, never materialised whole (80 GB per
partition) -- AggregatePartial per partition, then ONE fan-in
(processor_merge.rs:45-63) into AggregateFinal.  Run two ways on the box's one
GPU:

  * one process: the engine's 8 pipes, the merge channel, AggregateFinal;
  * 8 ranks (the C5 sharding, one partition per rank) sharing the GPU over
    gloo: each rank's partial states go through the native exchange
    (fq_engine_execute_exchange, the protocol fq_engine_execute_rccl runs over
    RCCL) and every rank's AggregateFinal must give the same row.

Closed forms: the wrapped sum 8713275208247570432, so
sum/count = 108915940, max = 79999999999, min = 0."""
import json
import os
import socket
import sys
import time

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 80_000_000_000
C5 = "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(%d)" % N
SUM = "SELECT sum(number) FROM system.numbers_mt(%d)" % N
WRAPPED = N * (N - 1) // 2 % 2**64
EXPECT_C5 = [(WRAPPED // N, N - 1, 0)]
EXPECT_SUM = [(WRAPPED,)]
CHUNK_ROWS = 400_000_000  # 3.2 GB pieces (FQ_OPT_CHUNK_ROWS default): 8 ranks fit in HBM together


def _evidence(name, obj):
    d = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, name), "w") as fh:
            json.dump(obj, fh, indent=1)


def test_closed_forms():
    assert WRAPPED == 8713275208247570432
    assert EXPECT_C5 == [(108915940, 79999999999, 0)]


def test_c5_single_process_generated_partitions():
    sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))
    from fq_amd import ops
    from fq_amd.engine import OPT_CHUNK_ROWS, PROFILE_SPAN, Engine
    ops.require_gpu()
    with Engine(device=0, profile=PROFILE_SPAN) as e:
        e.set_option(OPT_CHUNK_ROWS, CHUNK_ROWS)
        t0 = time.perf_counter()
        r = e.execute(C5)
        t1 = time.perf_counter()
        s = e.execute(SUM)
        t2 = time.perf_counter()
        st = e.stats()
    assert r.rows == EXPECT_C5
    assert s.rows == EXPECT_SUM
    _evidence("c5_single_process.json", {
        "sql": C5, "result": r.rows[0], "sum_result": s.rows[0][0], "c5_s": t1 - t0, "sum_s": t2 - t1,
        "rows_per_s": N / (t1 - t0), "chunk_rows": CHUNK_ROWS, "scan_launches": st["scan_launches"],
        "scan_rows": st["scan_rows"], "scan_span_ms": st["scan_ms"],
        "note": "one process, 8 pipes, every partition generated in 3.2 GB pieces (fill + fused scan per piece); "
                "scan_span_ms spans both queries' fills and scans (FQ_OPT_PROFILE 2)"})
    # 200 pieces of 4e8 rows per query, each one fused scan
    assert st["scan_launches"] == 2 * N // CHUNK_ROWS and st["scan_rows"] == 2 * N


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    for p in (os.path.join(ROOT, "fuse-query_amd"),):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from fq_amd import dist as fqd
    from fq_amd.engine import OPT_CHUNK_ROWS, Engine

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with Engine(device=0) as e:
            e.set_option(OPT_CHUNK_ROWS, CHUNK_ROWS)
            dist.barrier()
            t0 = time.perf_counter()
            r = fqd.execute(e, C5).rows
            t1 = time.perf_counter()
            s = fqd.execute(e, SUM).rows
            st = e.stats()
            e.trim_memory()  # hand the pieces back before the other ranks' next query
        q.put((rank, r, s, t1 - t0, {k: st[k] for k in ("partial_ms", "exchange_ms", "final_ms", "exchange_rounds",
                                                         "exchange_bytes", "scan_launches", "scan_rows")}))
    finally:
        dist.destroy_process_group()


def test_c5_eight_gloo_ranks_share_the_gpu():
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        results = sorted(q.get(timeout=280) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0
    _evidence("c5_world8_gloo.json", {
        "sql": C5, "world": world, "transport": "gloo (fq_engine_execute_exchange), 8 ranks on one GPU",
        "chunk_rows": CHUNK_ROWS,
        "ranks": [{"rank": r, "result": res[0], "sum_result": s[0][0], "c5_s": dt, "stats": st}
                  for r, res, s, dt, st in results]})
    for rank, res, s, dt, st in results:
        assert res == EXPECT_C5, rank
        assert s == EXPECT_SUM, rank
        # this rank's one partition: 1e10 rows in 25 generated pieces per query
        assert st["scan_rows"] == 2 * N // world and st["scan_launches"] == 2 * 25
        # one all-reduce per query, sized to the states (C3: 96 B + 8 B length per rank)
        assert st["exchange_rounds"] == 2
