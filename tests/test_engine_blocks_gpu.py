"""The engine's row pipelines as a stream of device DataBlocks
(fq_engine_execute_blocks): FilterTransform -> ProjectionTransform over
numbers_mt runs fq_filter_project_blocks inside the engine, and the blocks come
back in HBM in the reference's per-block geometry.

Parity: for every partition pipe, the concatenation of its device blocks'
sub-blocks equals oracle/fq_ref.py projection_blocks -- the reference's own
loop: each 10,000-row numbers block (numbers_stream.rs:27-83, including the
short last block of the row-dropping quirk) filtered by
FilterTransform::expression_executor (transform_filter.rs:38-55), then every
projected expression (transform_projection.rs:45-56, stream_expression.rs:38-50)
-- bit-exact, block by block, empty blocks included.  Resident and generated
partitions, one or several device blocks per partition (FQ_OPT_CHUNK_ROWS), and
at numbers_mt(1e10) the kept count and each column's wrapping sum against
closed forms."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

U64 = 2**64


@pytest.fixture(scope="module")
def eng():
    from fq_amd import ops
    ops.require_gpu()
    from fq_amd.engine import Engine
    e = Engine(profile=True)
    yield e
    e.close()


def _pull(eng, sql):
    """{pipe: [block][column] -> np.ndarray} from the engine's block stream,
    plus the number of device blocks and their layouts."""
    from fq_amd import ops
    per_pipe, layouts = {}, []
    with eng.execute_blocks(sql) as s:
        for b in s:
            layouts.append((b.pipe, b.block_rows, b.n_blocks, b.rows))
            cols = ops.device_block_to_numpy(b)
            if b.block_rows > 0:
                assert sum(len(x) for x in cols[0]) == b.rows
                blocks = [[c[k] for c in cols] for k in range(b.n_blocks)]
            else:
                blocks = [[c for c in cols]]
            per_pipe.setdefault(b.pipe, []).extend(blocks)
    return per_pipe, layouts


def _check_against_oracle(per_pipe, expect, float_cols=()):
    assert sorted(per_pipe) == list(range(len(expect)))
    for pipe, exp_blocks in enumerate(expect):
        got = per_pipe[pipe]
        assert len(got) == len(exp_blocks), (pipe, len(got), len(exp_blocks))
        for k, (g, e) in enumerate(zip(got, exp_blocks)):
            for j, (gc, ec) in enumerate(zip(g, e)):
                if j in float_cols:
                    assert np.array_equal(gc.view(np.uint64), np.array(ec, dtype=np.float64).view(np.uint64)), (pipe, k)
                else:
                    assert gc.tolist() == [int(x) % U64 for x in ec], (pipe, k, j)


import fq_ref as R  # noqa: E402

NUM = R.E_field("number")
C = R.E_const
P1_EXPRS = [R.E_bin("+", NUM, C(1)), R.E_bin("/", NUM, C(2))]
P1_WHERE = R.E_bin("<", R.E_bin("%", NUM, C(8)), C(3))


@pytest.mark.parametrize("n", [400_037, 80_000, 7, 123_456])
def test_block_stream_matches_the_reference_blocks(eng, n):
    # n = 400,037: partitions of 50,004 / 50,009 rows (the quirk: the last
    # block is remain + 1 rows); 80,000: whole blocks; 7: one partition "7-0-6"
    # of 7 rows (one pipe); 123,456: partitions of 15,432 rows, of which the
    # quirk yields 5,433 (one short block)
    sql = "SELECT number+1, number/2 FROM system.numbers_mt(%d) WHERE (number%%8)<3" % n
    s0 = eng.stats()["project_launches"]
    per_pipe, layouts = _pull(eng, sql)
    _check_against_oracle(per_pipe, R.projection_blocks(n, P1_EXPRS, P1_WHERE))
    # the block-stream kernel ran inside the engine for the partitions >= its tile
    assert eng.stats()["project_launches"] > s0 or n < 8192
    assert all(br == 10000 for _, br, _, _ in layouts if br)


def test_block_stream_resident_and_in_pieces(eng):
    from fq_amd.engine import OPT_CHUNK_ROWS
    n = 800_000 * 3 + 80_017  # 8 partitions of 310,002 rows (+ remainder)
    sql = "SELECT number+1, number/2 FROM system.numbers_mt(%d) WHERE (number%%8)<3" % n
    expect = R.projection_blocks(n, P1_EXPRS, P1_WHERE)
    eng.materialize_numbers(n)
    try:
        per_pipe, layouts = _pull(eng, sql)  # resident partitions: zero-copy slices
        _check_against_oracle(per_pipe, expect)
        assert len(layouts) == 8
        eng.set_option(OPT_CHUNK_ROWS, 100_000)  # pieces of <= 10 blocks: 4 device blocks per partition
        per_pipe, layouts = _pull(eng, sql)
        _check_against_oracle(per_pipe, expect)
        assert len(layouts) == 32 and {nb for _, _, nb, _ in layouts} <= {8, 7}
    finally:
        eng.set_option(OPT_CHUNK_ROWS, 400_000_000)
        eng.release_numbers()
    per_pipe, _ = _pull(eng, sql)  # generated partitions
    _check_against_oracle(per_pipe, expect)


def test_block_stream_expression_shapes(eng):
    # the README's aliased WHERE (an expression tree, FilterPushDown), a float
    # output, an AND predicate, and no predicate at all (plain columns)
    n = 200_003
    sql = ("select (number+1) as c1, number/2 as c2, number*1.5 from system.numbers_mt(%d) "
           "where (c1+c2+1) < 150000" % n)
    exprs = [R.E_alias("c1", R.E_bin("+", NUM, C(1))), R.E_alias("c2", R.E_bin("/", NUM, C(2))),
             R.E_bin("*", NUM, C(1.5))]
    where = R.E_bin("<", R.E_bin("+", R.E_bin("+", R.E_bin("+", NUM, C(1)), R.E_bin("/", NUM, C(2))), C(1)), C(150000))
    per_pipe, _ = _pull(eng, sql)
    _check_against_oracle(per_pipe, R.projection_blocks(n, exprs, where), float_cols=(2,))
    sql = "SELECT number%%1000 FROM system.numbers_mt(%d) WHERE (number%%8)<3 and number>70000" % n
    where = R.E_bin("and", R.E_bin("<", R.E_bin("%", NUM, C(8)), C(3)), R.E_bin(">", NUM, C(70000)))
    per_pipe, _ = _pull(eng, sql)
    _check_against_oracle(per_pipe, R.projection_blocks(n, [R.E_bin("%", NUM, C(1000))], where))
    sql = "SELECT number+1 FROM system.numbers_mt(%d)" % n  # no filter: plain columns
    per_pipe, layouts = _pull(eng, sql)
    assert all(br == 0 for _, br, _, _ in layouts)
    # plain columns: each pipe's rows in order equal its partition's blocks
    # back to back (25,000-row partitions yield 15,001 rows: the quirk)
    expect = R.projection_blocks(n, [R.E_bin("+", NUM, C(1))])
    assert sorted(per_pipe) == list(range(len(expect)))
    for pipe, exp_blocks in enumerate(expect):
        got = np.concatenate([blk[0] for blk in per_pipe[pipe]])
        assert got.tolist() == [v for blk in exp_blocks for v in blk[0]], pipe


def test_block_stream_limit_and_errors(eng):
    from fq_amd import FQError, abi
    # LIMIT compacts the kept rows into plain columns (stream_limit.rs:28-48)
    rows = []
    with eng.execute_blocks("SELECT number+1 FROM system.numbers_mt(1000000) WHERE (number%8)<3 LIMIT 5") as s:
        from fq_amd import ops
        for b in s:
            assert b.block_rows == 0
            rows.extend(ops.device_block_to_numpy(b)[0].tolist())
    assert len(rows) == 5 and all((r - 1) % 8 < 3 for r in rows)
    with pytest.raises(FQError) as ei:
        eng.execute_blocks("SELECT sum(number) FROM system.numbers_mt(100)")
    assert ei.value.status == abi.FQ_E_UNSUPPORTED
    # the reference's error order through the block path: divide by zero in WHERE
    with pytest.raises(FQError, match="Divide by zero"):
        with eng.execute_blocks("SELECT number+1 FROM system.numbers_mt(100000) WHERE (1000 % number) = 1000") as s:
            for _ in s:
                pass


def test_host_rows_through_the_block_path_match_the_oracle(eng):
    # fq_engine_execute over the same pipeline: the blocks are compacted
    # (fq_blocks_compact) into host rows, partition by partition
    n = 300_007
    r = eng.execute("SELECT number+1, number/2 FROM system.numbers_mt(%d) WHERE (number%%8)<3" % n)
    exp = R.projection_query(n, P1_EXPRS, P1_WHERE)
    assert sorted(r.rows) == sorted(exp)


def test_block_stream_c5_shape_closed_forms(eng):
    """numbers_mt(1e10) resident: 8 partitions x 4 device blocks of 3.125e8
    rows; kept rows and each column's wrapping sum over the valid rows equal
    the closed forms (number%8 < 3 keeps 3 of every 8)."""
    import torch

    from fq_amd import ops
    n = 10_000_000_000
    eng.materialize_numbers(n)
    try:
        kept = s1 = s2 = 0
        nblk = 0
        with eng.execute_blocks("SELECT number+1, number/2 FROM system.numbers_mt(%d) WHERE (number%%8)<3" % n) as s:
            for b in s:
                nblk += 1
                assert b.block_rows == 10000
                counts = ops.device_view(b.d_counts, 8 * b.n_blocks).view(torch.int64)
                valid = (torch.arange(b.columns[0].len, device="cuda") % 10000) < \
                    counts.repeat_interleave(10000)[:b.columns[0].len]
                for j in range(2):
                    col = ops.device_view(b.columns[j].data, 8 * b.columns[j].len).view(torch.int64)
                    t = int(torch.where(valid, col, torch.zeros_like(col)).sum().item()) % U64
                    if j == 0:
                        s1 += t
                    else:
                        s2 += t
                kept += b.rows
                del valid, counts
        assert nblk == 32
        exp_kept = 3 * n // 8
        exp_s1 = exp_s2 = 0
        for c in range(3):
            k = n // 8
            sj = (k - 1) * k // 2
            exp_s1 += 8 * sj + k * (c + 1)
            exp_s2 += 4 * sj + k * (c // 2)
        assert kept == exp_kept
        assert s1 % U64 == exp_s1 % U64 and s2 % U64 == exp_s2 % U64
    finally:
        eng.release_numbers()


def test_block_stream_dropped_early_stops_the_pipes(eng):
    """A host that stops pulling after the first block frees the stream: the
    merge channel closes, the pipes stop after the block they are producing,
    and the engine answers the next query normally (nothing left running)."""
    import time
    n = 4_000_000_000
    sql = "SELECT number+1, number/2 FROM system.numbers_mt(%d) WHERE (number%%8)<3" % n
    t0 = time.perf_counter()
    s = eng.execute_blocks(sql)
    b = s.next()
    assert b is not None and b.rows > 0
    s.close()
    assert time.perf_counter() - t0 < 30
    r = eng.execute("SELECT count(number), max(number) FROM system.numbers_mt(%d)" % 800_000)
    assert r.rows == [(800_000, 799_999)]
    per_pipe, _ = _pull(eng, "SELECT number+1, number/2 FROM system.numbers_mt(80000) WHERE (number%8)<3")
    _check_against_oracle(per_pipe, R.projection_blocks(80_000, P1_EXPRS, P1_WHERE))


def test_engine_destroyed_with_a_stream_open():
    """fq_engine_destroy while a block stream is open (its pipes mid-partition,
    blocked on the full merge channel): the engine closes and joins the stream
    first -- no hang, no use of freed queues -- the orphaned stream's next call
    fails with a message and fq_block_stream_free still releases it; the Python
    Engine.close() closes its open BlockStreams itself."""
    import ctypes as C

    from fq_amd import abi
    from fq_amd._lib import lib
    from fq_amd.engine import Engine, fq_device_block
    sql = b"SELECT number+1 FROM system.numbers_mt(4000000000) WHERE (number%8)<3"
    e = Engine()
    h = C.c_void_p()
    assert lib.fq_engine_execute_blocks(e.h, sql, 0, 1, C.byref(h)) == 0
    b, has = fq_device_block(), C.c_int32(0)
    assert lib.fq_block_stream_next(h, C.byref(b), C.byref(has)) == 0 and has.value == 1
    lib.fq_engine_destroy(e.h)  # the raw handle: the Python registry does not know this stream
    e.h = None
    assert lib.fq_block_stream_next(h, C.byref(b), C.byref(has)) == abi.FQ_E_INVALID
    assert b"engine was destroyed" in lib.fq_last_error()
    lib.fq_block_stream_free(h)
    # the wrapper: close() closes the stream before the engine
    e2 = Engine()
    st = e2.execute_blocks(sql.decode())
    assert st.next() is not None
    e2.close()
    assert st.h is None


def test_block_stream_launch_after_launch_and_after_an_error(eng):
    """The engine's projection launches (engine/functions.cpp project_blocks):
    the worker's resident workspace and result words, a one-thread hand-off
    kernel after each projection kernel, one span per query -- several launches
    per pipe yield the reference's blocks, twice, then the divide-by-zero error
    of a kept row, then the right blocks again (the workspace re-zeroed, the
    words of the failed launch not carried over)."""
    from fq_amd import FQError
    from fq_amd.engine import OPT_CHUNK_ROWS
    n = 800_000 * 3 + 80_017
    sql = "SELECT number+1, number/2 FROM system.numbers_mt(%d) WHERE (number%%8)<3" % n
    expect = R.projection_blocks(n, P1_EXPRS, P1_WHERE)
    try:
        eng.set_option(OPT_CHUNK_ROWS, 100_000)
        for _ in range(2):
            per_pipe, layouts = _pull(eng, sql)
            _check_against_oracle(per_pipe, expect)
            assert len(layouts) == 32
        with pytest.raises(FQError, match="Divide by zero"):
            _pull(eng, "SELECT 7/(number-300000) FROM system.numbers_mt(%d) WHERE number > 200000" % n)
        per_pipe, _ = _pull(eng, sql)
        _check_against_oracle(per_pipe, expect)
    finally:
        eng.set_option(OPT_CHUNK_ROWS, 400_000_000)


def test_block_stream_span_is_the_union_over_the_row_queues():
    """Row pipelines without a LIMIT run pipe p on row queue p % 2
    (engine/core.h Runtime::kRowQueues) and LaunchSpan times a query's
    projections as ONE span: the earliest first-launch start to the latest
    end over both queues (engine/functions.cpp LaunchSpan::arrive) -- never
    the sum of the two queues' spans, which would exceed the query's wall
    time while their launches overlap.  Results stay the reference's blocks."""
    import time
    from fq_amd.engine import PROFILE_SPAN, Engine
    n = 800_000_000  # 8 partitions of 1e8 rows: one launch each, four per row queue
    sql = "SELECT number+1, number/2 FROM system.numbers_mt(%d) WHERE (number%%8)<3" % n
    with Engine(profile=PROFILE_SPAN) as e:
        e.materialize_numbers(n)
        def rows():
            with e.execute_blocks(sql) as st:
                return sum(b.rows for b in st)

        kept = rows()  # warm: compile, map the outputs
        assert kept == 3 * n // 8
        e.reset_stats()
        t0 = time.perf_counter()
        for _ in range(3):
            assert rows() == kept
        wall_ms = (time.perf_counter() - t0) * 1e3
        st = e.stats()
        assert st["project_launches"] == 3 * 8
        assert 0 < st["project_ms"] <= wall_ms, (st["project_ms"], wall_ms)
        per_pipe, _ = _pull(e, "SELECT number+1, number/2 FROM system.numbers_mt(400037) WHERE (number%8)<3")
        _check_against_oracle(per_pipe, R.projection_blocks(400_037, P1_EXPRS, P1_WHERE))
