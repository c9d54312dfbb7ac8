"""Device memory held by the engine between queries (stream-ordered block
cache + the default pool's release threshold) is reclaimed before any
allocation fails: a materialisation sized above the HBM the driver reports
free -- but below free + what the engine holds -- succeeds right after a
streamed row-pipeline query, and fq_engine_trim_memory hands the held memory
back on demand."""
import pytest

pytestmark = pytest.mark.gpu

GB = 1 << 30


def _free():
    import torch
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info()[0]


@pytest.fixture(scope="module")
def Engine():
    from fq_amd import ops
    ops.require_gpu()
    from fq_amd.engine import Engine as E
    return E


def _stream(e):
    # full scans through growing morsels (160,000 rows doubling to 327,680,000
    # per partition): blocks of many size classes freed on the pipes' queues
    r = e.execute("SELECT number FROM system.numbers_mt(4000000000) WHERE number % 1000000007 = 3")
    assert sorted(v for (v,) in r.rows) == [3, 1000000010, 2000000017, 3000000024]
    r = e.execute("SELECT number + 1 FROM system.numbers_mt(2000000000) WHERE number % 999999937 = 0 LIMIT 2")
    assert len(r.rows) == 2


def test_materialize_after_streamed_query_reclaims_held_memory(Engine):
    import torch
    torch.cuda.empty_cache()
    e = Engine()
    try:
        before = _free()
        _stream(e)
        after = _free()
        held = before - after
        assert held >= 0
        if held < GB // 2:
            pytest.skip("engine holds %d MB after the query: nothing to reclaim" % (held >> 20))
        # rows whose columns need more than the free HBM but fit once the held memory is back
        want = after + held // 2
        total = (want // 8) // 80000 * 80000
        e.materialize_numbers(total)
        r = e.execute("SELECT count(number), max(number) FROM system.numbers_mt(%d)" % total)
        assert r.rows == [(total, total - 1)]
        e.release_numbers()
    finally:
        e.close()


def test_trim_memory_returns_held_memory(Engine):
    import torch
    torch.cuda.empty_cache()
    e = Engine()
    try:
        before = _free()
        _stream(e)
        held = before - _free()
        e.trim_memory()
        released = _free() - (before - held)
        # everything the queries kept is back, up to allocator granularity
        assert released >= held - 64 * (1 << 20), (held, released)
        _stream(e)  # and the engine still runs afterwards
    finally:
        e.close()


def test_kept_group_by_workspaces_leave_the_small_block_cache_room(Engine):
    """A partitioned GROUP BY keeps one ~3.4 GB workspace per queue for the next
    query (DeviceBuffer::alloc_workspace).  Those are counted apart from the
    small-block cache's 6 GB cap: with two queues the kept workspaces alone pass
    6 GB, and the small blocks of the next row pipeline must still be cached."""
    import torch
    torch.cuda.empty_cache()
    e = Engine(streams=2)
    try:
        e.trim_memory()
        n = 8_000_000_000  # 1e9-row partitions, generated in 4e8-row chunks
        r = e.execute("SELECT number%%100000, count(number) FROM system.numbers_mt(%d) GROUP BY number%%100000" % n)
        assert len(r.rows) == 100000 and r.rows[0] == (0, n // 100000) and r.rows[-1] == (99999, n // 100000)
        ws = e.stats()["cached_workspace_bytes"]
        assert ws > 6 * GB, ws  # one per queue, beyond the small-block cap together
        _stream(e)
        st = e.stats()
        assert st["cached_block_bytes"] > 0, st
        assert st["cached_workspace_bytes"] == ws
        e.trim_memory()
        st = e.stats()
        assert st["cached_block_bytes"] == 0 and st["cached_workspace_bytes"] == 0
    finally:
        e.close()


def test_large_block_cache_leaves_room_for_torch(Engine):
    """The engine keeps a row pipeline's large projected blocks (2.5 GB each)
    for the next query, but sized to the device -- at most 3/10 of its HBM --
    and never past the point where less than max(8 GB, 1/16) of it would stay
    free: after a 1e10-row p1 query (32 blocks of 2 x 2.5 GB) a torch
    allocation of most of the free HBM still succeeds."""
    import torch
    torch.cuda.empty_cache()
    e = Engine()
    try:
        total = torch.cuda.mem_get_info()[1]
        with e.execute_blocks("SELECT number+1, number/2 FROM system.numbers_mt(10000000000) WHERE (number%8)<3") as st:
            kept = sum(b.rows for b in st)
        assert kept == 3_750_000_000
        cached = e.stats()["cached_block_bytes"]
        assert cached <= total * 3 // 10 + (64 << 20), (cached, total)
        free = _free()
        assert free >= max(8 * GB, total // 16) - 4 * GB, (free, total)
        x = torch.empty(free - 2 * GB, dtype=torch.uint8, device="cuda")  # no OOM
        del x
        torch.cuda.empty_cache()
    finally:
        e.close()
