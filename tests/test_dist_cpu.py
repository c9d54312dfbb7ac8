"""CPU, world_size 2 (and 3) over gloo: the multi-GPU path minus the GPU.
Each rank owns its numbers_mt shard [8r/G, 8(r+1)/G) (fq_amd.numbers.shard),
ships its merged partial states through fq_amd.dist.allgather_states (the
native fq_exchange_states protocol bench.py runs over RCCL), and every rank's
AggregateFinal merge must equal the single-process oracle result.  The
per-rank partial states come from the oracle: without a GPU the scan cannot
run, and there is no CPU fallback to run it with."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SQL = ("SELECT sum(number)/count(number), max(number), min(number), count(number) "
       "FROM system.numbers_mt(%d)")


def worker(rank, world, port, n, out_q):
    for p in (os.path.join(ROOT, "fuse-query_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    import fq_ref as R
    from fq_amd import dist as fqd
    from fq_amd.engine import Engine
    from fq_amd.numbers import generate_parts, shard
    from test_engine_cpu import encode_states

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        num = R.E_field("number")
        exprs = [R.E_bin("/", R.E_fn("sum", num), R.E_fn("count", num)), R.E_fn("max", num),
                 R.E_fn("min", num), R.E_fn("count", num)]
        mine = [(b, e) for _, b, e in shard(generate_parts(n), rank, world)]
        local = encode_states(R.aggregate_partial_states(n, exprs, mine))
        with Engine(device=-1) as eng:
            # round 1 sized to the states (what fq_engine_execute_exchange does)
            cap = eng.partial_state_bytes(SQL % n)
            everyone = fqd.allgather_states(local, cap=cap)
            rows = eng.execute_final(SQL % n, everyone).rows
        out_q.put((rank, rows, [len(s) for s in everyone] + [len(local), cap]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1000000), (2, 7), (3, 123457)])
def test_sharded_exchange_and_final_merge(world, n):
    import fq_ref as R
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    num = R.E_field("number")
    exp = [tuple(v.value for v in R.aggregate_query(n, [
        R.E_bin("/", R.E_fn("sum", num), R.E_fn("count", num)), R.E_fn("max", num), R.E_fn("min", num),
        R.E_fn("count", num)]))]
    for rank, rows, lens in results:
        assert rows == exp, (rank, rows, exp)
        # every rank's states are exactly the planned size: one round, stride = that size
        *strides, local_len, cap = lens
        assert local_len == cap and strides == [(cap + 7) // 8 * 8] * world, (rank, lens)


GB_SQL = "SELECT number%%97, count(number), sum(number), min(number+3) FROM system.numbers_mt(%d) GROUP BY number%%97"


def gb_worker(rank, world, port, n, out_q):
    for p in (os.path.join(ROOT, "fuse-query_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    import fq_ref as R
    from fq_amd import dist as fqd
    from fq_amd.engine import Engine
    from fq_amd.numbers import generate_parts, shard
    from test_engine_cpu import encode_states

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        num = R.E_field("number")
        key = R.E_bin("%", num, R.E_const(97))
        exprs = [R.E_fn("count", num), R.E_fn("sum", num), R.E_fn("min", R.E_bin("+", num, R.E_const(3)))]
        mine = [(b, e) for _, b, e in shard(generate_parts(n), rank, world)]
        local = encode_states(R.group_by_partial_states(n, key, exprs, mine))
        everyone = fqd.allgather_states(local)  # > 4096 bytes: length agreed first
        with Engine(device=-1) as eng:
            rows = eng.execute_final(GB_SQL % n, everyone).rows
        out_q.put((rank, rows, len(local)))
    finally:
        dist.destroy_process_group()


def test_group_by_exchange_and_final_merge():
    import fq_ref as R
    world, n = 2, 400000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=gb_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    num = R.E_field("number")
    exp = R.group_by_query(n, R.E_bin("%", num, R.E_const(97)),
                           [R.E_fn("count", num), R.E_fn("sum", num), R.E_fn("min", R.E_bin("+", num, R.E_const(3)))])
    for rank, rows, nbytes in results:
        assert nbytes > 4096
        assert rows == exp, rank


def ragged_worker(rank, world, port, lens, out_q, cap=None):
    for p in (os.path.join(ROOT, "fuse-query_amd"),):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from fq_amd import dist as fqd

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = bytes((rank * 31 + i) % 251 + 1 for i in range(lens[rank]))
        rows = fqd.allgather_states(mine, cap=cap)
        out_q.put((rank, rows))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("lens,cap", [((5000, 40), None), ((0, 0, 7), None), ((4096, 4097, 1), None), ((10, 20), None),
                                      ((10, 20), 0), ((96, 96, 97), 96), ((96, 96, 96), 96), ((3, 0), 5)])
def test_exchange_protocol_ragged_lengths(lens, cap):
    """fq_exchange_states(_sized): every rank takes the same number of
    all-reduces even when only SOME ranks' states exceed the first round's
    cap (a per-rank decision would leave the others waiting in a collective);
    cap None = FQ_EXCHANGE_CAP_BYTES, 0 = lengths only in round 1."""
    world = len(lens)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=ragged_worker, args=(r, world, port, lens, q, cap)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c8 = ((4096 if cap is None else cap) + 7) // 8 * 8
    stride = c8 if max(lens) <= c8 else (max(lens) + 7) // 8 * 8
    for rank, rows in results:
        assert len(rows) == world
        for r, row in enumerate(rows):
            exp = bytes((r * 31 + i) % 251 + 1 for i in range(lens[r]))
            assert len(row) == stride and row[:lens[r]] == exp and not any(row[lens[r]:]), (rank, r)


def test_group_by_final_merges_flat_rows_on_the_host():
    # execute_final on a host-only engine over three ranks' GROUP BY rows in
    # the flat wire format ("FQG1", pipeline.cpp encode_group_rows): Int64
    # keys (negative and positive), keys shared between ranks, more groups
    # than the final's radix-sort threshold; the merge folds equal keys
    # (count/sum add, max keeps the largest) and orders by key
    import random
    import struct

    sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))
    from fq_amd import abi
    from fq_amd.engine import Engine

    def fqg1(rows):
        nl = 3
        out = b"FQG1" + struct.pack("<IQii", nl, len(rows), abi.DT_INT64, 0)
        out += struct.pack("<3i", abi.DT_UINT64, abi.DT_UINT64, abi.DT_UINT64) + b"\0" * 4
        out += struct.pack("<%dq" % len(rows), *[r[0] for r in rows])
        for a in range(nl):
            out += struct.pack("<%dQ" % len(rows), *[r[1 + a] for r in rows])
        return out

    rng = random.Random(5)
    ranks, exp = [], {}
    for _ in range(3):
        keys = rng.sample(range(-30000, 30000), 9000)
        rows = [(k, rng.randint(1, 9), rng.randint(0, 2**63), rng.randint(0, 2**64 - 1)) for k in keys]
        ranks.append(fqg1(rows))
        for k, c, s, m in rows:
            e = exp.get(k)
            exp[k] = (c, s, m) if e is None else (e[0] + c, (e[1] + s) % 2**64, max(e[2], m))
    sql = "SELECT number%97, count(number), sum(number), max(number) FROM system.numbers_mt(1000) GROUP BY number%97"
    with Engine(device=-1) as eng:
        rows = eng.execute_final(sql, ranks).rows
    assert rows == [(k,) + exp[k] for k in sorted(exp)]


# ---- the C5 shape: 8 ranks, numbers_mt(8e10), one partition per rank --------

def closed_form_states(parts):
    """Per-rank partial states of SQL's four functions over `parts`, in closed
    form (a rank's NumbersStream rows are contiguous from each partition's
    begin, numbers.stream_rows); Null states when the rank owns nothing (no
    merge_state ever reached them, function_aggregator.rs:24-36)."""
    import fq_ref as R
    if not parts:
        return [[R.Value("Null", None)] * 2, [R.Value("Null", None)], [R.Value("Null", None)],
                [R.Value("Null", None)]]
    from fq_amd.numbers import stream_rows
    s = c = 0
    mx, mn = 0, None
    for _, b, e in parts:
        rows = stream_rows(b, e)
        s += rows * (2 * b + rows - 1) // 2
        c += rows
        mx = max(mx, b + rows - 1)
        mn = b if mn is None else min(mn, b)
    u = lambda x: R.Value("UInt64", x % 2**64)  # noqa: E731
    return [[u(s), u(c)], [u(mx)], [u(mn)], [u(c)]]


def c5_worker(rank, world, port, n, out_q):
    for p in (os.path.join(ROOT, "fuse-query_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from fq_amd import dist as fqd
    from fq_amd.engine import Engine
    from fq_amd.numbers import generate_parts, shard
    from test_engine_cpu import encode_states

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = shard(generate_parts(n), rank, world)
        with Engine(device=-1) as eng:
            local = encode_states(closed_form_states(mine))
            cap = eng.partial_state_bytes(SQL % n)
            assert len(local) == cap  # a rank owning nothing ships Null states of the same size
            everyone = fqd.allgather_states(local, cap=cap)
            rows = eng.execute_final(SQL % n, everyone).rows
        out_q.put((rank, [name for name, _, _ in mine], rows))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [80_000_000_000, 7])
def test_world8_c5_shards_exchange_and_final(n):
    """BASELINE configs[4] at world 8 over gloo: numbers_table.rs:29-55 names
    8 partitions and rank r owns exactly partition r; at N=7 there is one
    partition "7-0-6" and only rank 7 owns it (shard [8r/G, 8(r+1)/G)), the
    other 7 ranks ship Null states.  Every rank's AggregateFinal over the
    exchanged states equals the closed form (processor_merge.rs:45-63 merges
    the partial streams in any order; the state merge is order-free)."""
    from fq_amd.numbers import generate_parts
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=c5_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    names = [nm for nm, _, _ in generate_parts(n)]
    if n == 7:
        assert names == ["7-0-6"]
        assert [owned for _, owned, _ in results] == [[]] * 7 + [["7-0-6"]]
    else:
        assert [owned for _, owned, _ in results] == [[names[r]] for r in range(8)]
        assert names[7] == "80000000000-70000000000-79999999999"
    s = n * (n - 1) // 2 % 2**64
    exp = [(s // n, n - 1, 0, n)]
    for rank, _, rows in results:
        assert rows == exp, (rank, rows, exp)


def test_group_rows_with_a_wrapping_row_count_are_rejected():
    # a row count whose byte size wraps 64 bits must not pass the length check
    # (pipeline.cpp decode_group_rows; the buffer crosses fq_engine_execute_final)
    import struct

    sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))
    from fq_amd import abi
    from fq_amd._lib import FQError
    from fq_amd.engine import Engine

    nl = 3
    rows = (1 << 61) + 1  # 8 * (1 + nl) * rows = 2^66 + 32: wraps to 32
    bad = b"FQG1" + struct.pack("<IQii", nl, rows, abi.DT_UINT64, 0)
    bad += struct.pack("<3i", abi.DT_UINT64, abi.DT_UINT64, abi.DT_UINT64) + b"\0" * 4 + b"\0" * 64
    sql = "SELECT number%97, count(number), sum(number), max(number) FROM system.numbers_mt(1000) GROUP BY number%97"
    with Engine(device=-1) as eng:
        with pytest.raises(FQError, match="truncated"):
            eng.execute_final(sql, [bad])


def error_worker(rank, world, port, sql, out_q):
    sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from fq_amd import FQError
    from fq_amd import dist as fqd
    from fq_amd.engine import Engine

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with Engine(device=-1) as eng:
            cap = eng.partial_state_bytes(sql)
            try:
                fqd.execute(eng, sql)
                out_q.put((rank, None, cap, eng.stats()))
            except FQError as e:
                out_q.put((rank, (e.status, str(e)), cap, eng.stats()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sql,rounds", [
    ("SELECT sum(number) FROM system.numbers_mt(1000000)", 2),  # 32 B of states: the 103 B record takes round 2
    (SQL % 1_000_000, 1),  # 120 B of states: the record fits round 1
])
def test_exchange_carries_error_records_past_the_sized_first_round(sql, rounds):
    """fq_engine_execute_exchange over gloo with host-only engines: every
    rank's partial fails (no device: the hot path has no CPU fallback), so every
    rank ships an error record ("FQE1", status, message: 103 B here) instead of
    its states.  Round 1 is sized to the SQL's states; a record longer than that
    takes the second round, and every rank reports the same error -- none waits
    in the collective.  The engine's exchange counters see the rounds."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=error_worker, args=(r, world, port, sql, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from fq_amd import abi
    errs = {err for _, err, _, _ in results}
    assert len(errs) == 1
    status, msg = errs.pop()
    assert status == abi.FQ_E_HIP and "no device" in msg
    for _, _, cap, st in results:
        assert st["exchanges"] == 1 and st["exchange_rounds"] == rounds
        round1 = world * (8 + (cap + 7) // 8 * 8)
        assert st["exchange_bytes"] == round1 + (world * 104 if rounds == 2 else 0)


def dead_peer_worker(rank, world, port, mode, deadline_s, out_q):
    """rank 0 exchanges; rank 1 never reaches the exchange ("absent": it
    idles past the deadline) or dies before it ("dead")."""
    import time
    for p in (os.path.join(ROOT, "fuse-query_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from fq_amd import FQError
    from fq_amd import dist as fqd
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dist.barrier()
    if rank == 1:
        if mode == "absent":
            time.sleep(deadline_s * 4)
        os._exit(0)
    t0 = time.monotonic()
    try:
        fqd.allgather_states(b"FQS1" + bytes(60), cap=64, timeout_s=deadline_s)
        out_q.put(("returned", time.monotonic() - t0, ""))
        code = 0
    except FQError as e:
        out_q.put(("failed", time.monotonic() - t0, "%d %s" % (e.status, e)))
        code = 3  # what a bench rank does: exit non-zero, the launcher tears the job down
    out_q.close()
    out_q.join_thread()
    os._exit(code)  # no group teardown with a peer gone


@pytest.mark.parametrize("mode", ["absent", "dead"])
def test_exchange_with_a_peer_that_never_arrives_fails_within_the_deadline(mode):
    """The exchange protocol's deadline: rank 0 runs the
    native fq_exchange_states protocol through the fq_allreduce_fn callback
    with a 3 s deadline while rank 1 never reaches the collective, or is gone.
    Rank 0 must not wait without end: the call fails with FQ_E_RCCL naming the
    rank within the deadline (+ slack), and the process exits non-zero.  The
    RCCL transport bounds the same wait natively (fq_comm.cpp comm_wait:
    ncclCommGetAsyncError polled against FQ_COMM_TIMEOUT_MS, then
    ncclCommAbort)."""
    from fq_amd import abi
    deadline = 3.0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=dead_peer_worker, args=(r, 2, port, mode, deadline, q)) for r in range(2)]
    for p in procs:
        p.start()
    what, elapsed, msg = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert what == "failed", (what, msg)
    assert msg.startswith("%d rank 0 of 2: the state all-reduce" % abi.FQ_E_RCCL), msg
    assert elapsed < deadline + 10, elapsed
    if mode == "absent":
        assert "did not complete within 3 s" in msg and elapsed >= deadline * 0.9, (msg, elapsed)
    assert procs[0].exitcode == 3
