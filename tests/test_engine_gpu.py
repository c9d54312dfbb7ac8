"""End-to-end parity of the C++ pipeline (SQL -> Source -> Filter ->
AggregatePartial x 8 -> Merge -> AggregateFinal, Projection, Limit) on the
GPU against the reference's own test expectations, the README results and
the C oracle.  Integer results are bit-exact."""
import pytest

from fq_amd import abi
from fq_amd.expr import chain, predicate

import oracle_c

pytestmark = pytest.mark.gpu

Engine = None
E = None


def setup_module():
    global Engine, E
    from fq_amd import ops
    ops.require_gpu()
    from fq_amd.engine import Engine as _E
    Engine = _E
    E = Engine()


def teardown_module():
    if E is not None:
        E.close()


def q(sql):
    return E.execute(sql)


def oracle(total, aggs, pred=None):
    """[(kind, dtype, value)] from the oracle's Source->Partial->Final."""
    return [v for _, _, v in oracle_c.numbers_query(total, aggs, pred)]


# ---- the reference's own pipeline tests ----------------------------------

def test_transform_aggregate_sum_plus_2_is_122():
    # src/transforms/transform_aggregate_test.rs:5-59 (sum(number)+2 over numbers_mt(16))
    r = q("SELECT sum(number)+2 FROM system.numbers_mt(16)")
    assert r.rows == [(122,)]
    assert r.names == ["Sum(number) + 2"]
    assert r.types == [abi.DT_UINT64]


def test_transform_filter_number_eq_1():
    # src/transforms/transform_filter_test.rs:5-44
    r = q("SELECT number FROM system.numbers_mt(8) WHERE number = 1")
    assert r.rows == [(1,)]


def test_source_reads_all_rows():
    # transform_source_test.rs: numbers_mt(16) -> 16 rows
    r = q("SELECT number FROM system.numbers_mt(16)")
    assert sorted(v for (v,) in r.rows) == list(range(16))


def test_readme_projection_filter_limit():
    # README.md:120-127 with the aliased expressions spelled out
    r = q("select (number+1) as c1, number/2 as c2 from system.numbers_mt(10000000) "
          "where ((number+1)+(number/2)+1) < 100 limit 3")
    assert r.names == ["c1", "c2"]
    assert r.rows == [(1, 0), (2, 0), (3, 1)]


def test_readme_query_verbatim_with_aliases():
    # README.md:116-127: the WHERE uses the projection's aliases; the
    # FilterPushDownOptimizer (optimizer_filter_push_down.rs) rewrites them
    r = q("select (number+1) as c1, number/2 as c2 from system.numbers_mt(10000000) where (c1+c2+1) < 100 limit 3")
    assert r.names == ["c1", "c2"]
    assert r.rows == [(1, 0), (2, 0), (3, 1)]


def test_explain_matches_reference_format():
    txt = E.explain("select (number+1) as c1, number/2 as c2 from system.numbers_mt(10000000) "
                    "where ((number+1)+(number/2)+1) < 100 limit 3")
    plan, pipe = txt.split("\n", 4)[:4], txt
    assert txt.startswith("└─ Limit: 3\n  └─ Projection: (number + 1) as c1, (number / 2) as c2\n"
                          "    └─ Filter: ((((number + 1) + (number / 2)) + 1) < 100)\n"
                          "      └─ ReadDataSource: scan parts [8](Read from system.numbers_mt table)")
    assert ("\n  └─ LimitTransform × 1 processor\n    └─ Merge (LimitTransform × 8 processors) to "
            "(MergeProcessor × 1)\n      └─ LimitTransform × 8 processors\n        └─ ProjectionTransform"
            " × 8 processors\n          └─ FilterTransform × 8 processors\n            └─ SourceTransform"
            " × 8 processors") in pipe


def test_explain_aggregate_pipeline_shape():
    # pipeline_builder_test.rs:25-31
    txt = E.explain("SELECT sum(number) FROM system.numbers_mt(80000)")
    assert ("└─ AggregateFinalTransform × 1 processor\n    └─ Merge (AggregatePartialTransform × 8 "
            "processors) to (MergeProcessor × 1)\n      └─ AggregatePartialTransform × 8 processors\n"
            "        └─ SourceTransform × 8 processors") in txt


# ---- BASELINE configs at oracle-sized N ----------------------------------

AGGS_C3 = [(abi.AGG_SUM, None), (abi.AGG_COUNT, None), (abi.AGG_MAX, None), (abi.AGG_MIN, None)]


def test_execute_row_equals_the_result_api():
    """fq_engine_execute_row: one call for a one-row statement -- the same
    values and types as fq_engine_execute + fq_result_value; a statement with
    another number of rows fails with FQ_E_INVALID and the row count."""
    from fq_amd.engine import FQError
    from fq_amd.expr import from_bits
    for sql in ("SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(1000003)",
                "SELECT max(number), count(number) FROM system.numbers_mt(100000) WHERE number % 7 = 3",
                "SELECT sum(number * 1.5), min(number - 5) FROM system.numbers_mt(777)"):
        r = q(sql)
        row = E.execute_row(sql)
        assert len(r.rows) == 1 and len(row) == len(r.types)
        for v, want, t in zip(row, r.rows[0], r.types):
            assert v.is_some and v.dtype == t
            assert from_bits(v.bits, t) == want
    assert len(E.execute_row("SELECT count(number), sum(number), max(number) FROM system.numbers_mt(10)", cap=2)) == 2
    with pytest.raises(FQError) as ei:
        E.execute_row("SELECT number FROM system.numbers_mt(5)")
    assert ei.value.status == abi.FQ_E_INVALID and "returned 5 rows" in str(ei.value)


@pytest.mark.parametrize("n", [1, 7, 8, 9, 16, 10000, 79999, 80000, 100001, 1000000, 12345679])
def test_c3_matches_oracle(n):
    r = q("SELECT sum(number)/count(number), max(number), min(number), count(number), sum(number) "
          "FROM system.numbers_mt(%d)" % n)
    s, c, mx, mn = oracle(n, AGGS_C3)
    assert r.rows == [(s // c, mx, mn, c, s)]


def test_numbers_mt_row_quirk_counts():
    # SURVEY finding 8: numbers_mt(100001) yields 20,009 rows, (1000000) 920,008
    assert q("SELECT count(number) FROM system.numbers_mt(100001)").rows == [(20009,)]
    assert q("SELECT count(number) FROM system.numbers_mt(1000000)").rows == [(920008,)]


@pytest.mark.parametrize("n", [80000, 1000000, 7777777])
def test_c4_matches_oracle(n):
    r = q("SELECT max(number+1), count(number+1) FROM system.numbers_mt(%d) WHERE (number%%8)<3" % n)
    value, _ = chain(abi.DT_UINT64, [("+", 1)])
    pred = predicate(abi.DT_UINT64, [("%", 8)], "<", 3)
    exp = oracle(n, [(abi.AGG_MAX, value), (abi.AGG_COUNT, value)], pred)
    assert r.rows == [tuple(exp)]


def test_c1_sum_1e8():
    assert q("SELECT sum(number) FROM system.numbers_mt(100000000)").rows == [(4999999950000000,)]


def test_c2_c3_c4_full_size_closed_forms():
    # BASELINE.md section 3 expected results at N = 1e10 (80 GB resident)
    n = 10_000_000_000
    E.materialize_numbers(n)
    try:
        assert q("SELECT sum(number) FROM system.numbers_mt(%d)" % n).rows == [(13106511847580896768,)]
        assert q("SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(%d)"
                 % n).rows == [(1310651184, 9999999999, 0)]
        assert q("SELECT max(number+1), count(number) FROM system.numbers_mt(%d) WHERE (number%%8)<3"
                 % n).rows == [(9999999995, 3750000000)]
    finally:
        E.release_numbers()


def _range_closed_forms(b, e):
    """C3 + C4 results over the rows [b, e) of numbers_mt (no dropped rows)."""
    s = ((b + e - 1) * (e - b) // 2) % 2**64
    top = e - 1
    while top % 8 >= 3:
        top -= 1
    kept = sum(max(0, (e - r + 7) // 8 - (b - r + 7) // 8) for r in range(3))
    return s, e - b, e - 1, b, top + 1, kept


@pytest.mark.parametrize("world,rank", [(2, 1), (4, 3), (8, 7)])
def test_weak_scaling_shard_beyond_2_pow_32_rows(world, rank):
    # bench.py at N GPUs: numbers_mt(1e10 * N), rank r owns partitions
    # [8r/N, 8(r+1)/N) -- 2.5e9 / 5e9 / 1e10-row partitions (> 2^31 and 2^32
    # rows per launch, values up to 8e10), which the 1-GPU run never reaches
    n = 10_000_000_000 * world
    per = n // 8
    b, e = per * 8 * rank // world, per * 8 * (rank + 1) // world
    E.materialize_numbers(n, rank, world)
    try:
        sql3 = "SELECT sum(number), count(number), max(number), min(number) FROM system.numbers_mt(%d)" % n
        sql4 = "SELECT max(number+1), count(number) FROM system.numbers_mt(%d) WHERE (number%%8)<3" % n
        s, c, mx, mn, m4, k4 = _range_closed_forms(b, e)
        assert E.execute_final(sql3, [E.execute_partial(sql3, rank, world)]).rows == [(s, c, mx, mn)]
        assert E.execute_final(sql4, [E.execute_partial(sql4, rank, world)]).rows == [(m4, k4)]
        st = E.stats()
        assert st["scan_rows"] > 0
    finally:
        E.release_numbers()


# ---- expression shapes beyond the fused chain ------------------------------

def test_non_chain_argument_uses_materialised_path():
    # (number+1)*(number+2) is a tree, not a chain: eval kernels + identity scan
    n = 50000
    r = q("SELECT sum((number+1)*(number+2)), max((number+1)*(number+2)) FROM system.numbers_mt(%d)" % n)
    exp_sum = sum((i + 1) * (i + 2) for i in range(n)) % 2**64
    assert r.rows == [(exp_sum, n * (n + 1))]


def test_filtered_non_chain_argument():
    n = 40000
    r = q("SELECT sum((number+1)*(number+2)), count(number) FROM system.numbers_mt(%d) "
          "WHERE (number%%7) > 2" % n)
    keep = [i for i in range(n) if i % 7 > 2]
    assert r.rows == [(sum((i + 1) * (i + 2) for i in keep) % 2**64, len(keep))]


def test_f64_expression_within_tolerance():
    n = 800_000  # a multiple of 80,000: numbers_mt drops no rows
    r = q("SELECT sum(number/2.0), max(number*1.5) FROM system.numbers_mt(%d)" % n)
    exp = sum(i / 2.0 for i in range(n))
    (s, mx), = r.rows
    # tolerance: relative 1e-12 (summation order differs from arrow's simd lanes)
    assert abs(s - exp) <= 1e-12 * exp
    assert mx == (n - 1) * 1.5


def test_sum_over_count_is_integer_division():
    # SURVEY finding 5 / function_aggregator_test.rs:118-140: UInt64 '/' truncates
    assert q("SELECT sum(number)/count(number) FROM system.numbers_mt(10)").rows == [(4,)]


# ---- error behaviour (texts as the reference formats them) ----------------

def err(sql, eng=None):
    from fq_amd import FQError
    with pytest.raises(FQError) as ei:
        (eng or E).execute(sql)
    return str(ei.value)


def test_error_modulo_disabled_is_reference_behaviour():
    with Engine(modulo=False) as e2:
        assert err("SELECT max(number+1) FROM system.numbers_mt(100) WHERE (number%8)<3", e2) == \
            "Internal Error: Unsupported Function: %"


def test_error_filtered_sum_with_empty_block():
    # number < 5 leaves the second 10,000-row block of partition 0 empty:
    # arrow sum -> None -> state add fails (data_value_arithmetic.rs)
    assert err("SELECT sum(number) FROM system.numbers_mt(1000000) WHERE number < 5") == \
        "Internal Error: DataValue to array cannot be NONE NULL"
    # count/max survive empty blocks
    assert q("SELECT count(number), max(number) FROM system.numbers_mt(1000000) WHERE number < 5").rows \
        == [(5, 4)]


def test_error_final_none_to_array():
    # every partition single-block and empty -> Sum state None -> to_array(1) fails
    assert err("SELECT sum(number) FROM system.numbers_mt(10) WHERE number > 100") == \
        "Internal Error: DataValue to array cannot be NONE NULL"


def test_error_divide_by_zero():
    assert err("SELECT sum(number/0) FROM system.numbers_mt(100)") == "Internal Error: Divide by zero error"


def test_error_unknown_function_and_table():
    assert err("SELECT avg(number) FROM system.numbers_mt(100)") == "Internal Error: Unsupported Function: avg"
    assert err("SELECT number FROM system.numbers(100)") == "Internal Error: Cannot find the table: numbers"
    assert err("SELECT number FROM numbers_mt(100)") == "Internal Error: Cannot find the database: default"
    assert err("SELECT sum(number), number FROM system.numbers_mt(10)") == \
        "Error during plan: Projection references non-aggregate values"


def test_error_aggregate_in_where():
    assert err("SELECT number FROM system.numbers_mt(10) WHERE sum(number) > 1") == \
        "Internal Error: Aggregate function (sum([number]) > 1) is found in WHERE in query"


@pytest.mark.parametrize("pipe", [1, 4, 8])
@pytest.mark.parametrize("sql", [
    "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(8000000)",
    "SELECT max(number+1) FROM system.numbers_mt(8000000) WHERE (number%8)<3",
    # a LIMIT no partition can satisfy: every pipe is read to its end
    "SELECT number+1, number/2 FROM system.numbers_mt(8000000) WHERE number%999999937 = 0 LIMIT 3",
    # a block-stream row pipeline (its projections timed by one LaunchSpan)
    "SELECT number+1, number/2 FROM system.numbers_mt(800000) WHERE (number%8)<3",
])
def test_pipe_that_cannot_set_up_its_context_fails_the_query(sql, pipe):
    """A pipe whose device context cannot be set up (a failed workspace
    allocation, forced by FQ_OPT_FAULT_PIPE) sends its error the way the
    reference's task sends Err (processor_merge.rs:50-54) and releases its place
    in the query's scan group: the query returns the error -- the other pipes'
    deferred states never wait for it -- and the engine runs on.  Row
    pipelines' blocks arrive in the order the pipes finish (the reference's
    merge channel, processor_merge.rs:45-63), so rows compare as a multiset."""
    from fq_amd import FQError
    from fq_amd.engine import OPT_FAULT_PIPE
    with Engine(profile=True) as e2:
        want = sorted(e2.execute(sql).rows)
        e2.set_option(OPT_FAULT_PIPE, pipe)
        with pytest.raises(FQError, match="out of memory"):
            e2.execute(sql)
        e2.set_option(OPT_FAULT_PIPE, 0)
        assert sorted(e2.execute(sql).rows) == want


# ---- distributed split on one device ---------------------------------------

def test_partial_final_split_matches_single_pipeline():
    sql = "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(1000000)"
    world = 4
    states = [E.execute_partial(sql, r, world) for r in range(world)]
    assert E.execute_final(sql, states).rows == q(sql).rows


def test_partial_states_none_error_survives_exchange():
    # 8 single-block partitions, one per rank: rank 0 holds Some(10), the others
    # None; only the cross-rank AggregateFinal merge meets Some + None
    sql = "SELECT sum(number) FROM system.numbers_mt(80) WHERE number < 5"
    states = [E.execute_partial(sql, r, 8) for r in range(8)]
    from fq_amd import FQError
    with pytest.raises(FQError) as ei:
        E.execute_final(sql, states)
    assert str(ei.value) == "Internal Error: DataValue to array cannot be NONE NULL"


def test_engine_stats_count_fused_scans():
    with Engine(profile=True) as e2:
        e2.execute("SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(800000)")
        s = e2.stats()
        assert s["scan_launches"] == 8  # one fused scan per partition for all 4 aggregators
        assert s["scan_rows"] == 800000 and s["scan_bytes"] == 6400000
        assert s["scan_ms"] > 0


def test_mysql_writer_types_and_boolean_error():
    # mysql_stream.rs:30-62: Boolean has no MySQL column arm -> Internal error
    r = q("SELECT number = 1 FROM system.numbers_mt(8)")
    assert r.mysql_error == "Internal Error: Unsupported column type:Boolean"
    r = q("select (number+1) as c1, number/2 as c2 from system.numbers_mt(10000000) where number+1=4 limit 10")
    assert r.mysql_types == [3, 3] and r.text_rows == [("4", "1")]


def test_f64_division_within_one_ulp():
    # north_star: f64 division within 1 ULP of the reference CPU path.  The
    # device divides in IEEE binary64 exactly as the CPU does, so the
    # distance is 0 ULP; max/min of a quotient involve no summation order.
    import numpy as np
    n = 10_000_000
    r = q("SELECT max(number/3.0), min((number+1)/7.0), max(number/0.1) FROM system.numbers_mt(%d)" % n)
    x = np.arange(0, n, dtype=np.uint64).astype(np.float64)  # 1.25M-row partitions: no dropped rows
    exp = [np.max(x / 3.0), np.min((x + 1) / 7.0), np.max(x / 0.1)]
    for got, e in zip(r.rows[0], exp):
        ulp = abs(np.float64(got).view(np.int64) - np.float64(e).view(np.int64))
        assert ulp <= 1, (got, e, ulp)
        assert ulp == 0



@pytest.mark.parametrize("where", [
    ("number > 100 AND number % 7 = 3", "and"),
    ("number < 1000 OR number % 97 = 0", "or"),
    ("(number % 8 < 3 AND number > 10) OR number = 5", "nested"),
])
def test_logic_in_where_matches_oracle(where):
    # LogicFunction (function_logic.rs) over device bitmaps; the aggregate
    # consumes the combined bitmap as its predicate
    import fq_ref as R
    n = 1_000_000
    sql_where, kind = where
    r = q("SELECT count(number), sum(number), max(number), min(number) FROM system.numbers_mt(%d) WHERE %s"
          % (n, sql_where))
    N = R.E_field("number")
    c = R.E_const
    if kind == "and":
        w = R.E_bin("and", R.E_bin(">", N, c(100)), R.E_bin("=", R.E_bin("%", N, c(7)), c(3)))
    elif kind == "or":
        w = R.E_bin("or", R.E_bin("<", N, c(1000)), R.E_bin("=", R.E_bin("%", N, c(97)), c(0)))
    else:
        w = R.E_bin("or", R.E_bin("and", R.E_bin("<", R.E_bin("%", N, c(8)), c(3)), R.E_bin(">", N, c(10))),
                    R.E_bin("=", N, c(5)))
    exp = R.aggregate_query(n, [R.E_fn("count", N), R.E_fn("sum", N), R.E_fn("max", N), R.E_fn("min", N)], where=w)
    assert r.rows == [tuple(v.value for v in exp)]


def test_logic_projection_and_errors():
    r = q("SELECT number FROM system.numbers_mt(100) WHERE number > 3 AND number < 7")
    assert sorted(r.rows) == [(4,), (5,), (6,)]
    assert err("SELECT count(number) FROM system.numbers_mt(100) WHERE number > 3 AND number") == \
        "Internal Error: Cannot downcast_array from datatype:UInt64 item to:BooleanArray"
    assert err("SELECT count(number) FROM system.numbers_mt(100) WHERE number > 3 AND 1") == \
        "Internal Error: Cannot do data_array and, left:Boolean, right:UInt64"


# ---- row pipelines stream morsels; a satisfied LIMIT stops early -----------

def _stream_rows(total):
    """Rows numbers_mt(total) yields, partition by partition (fq_ref restates
    numbers_table.rs / numbers_stream.rs, quirk included)."""
    import fq_ref as R
    out = []
    for b, e in R.generate_parts(total):
        for bb, be in R.numbers_blocks(b, e):
            out.extend(range(bb, be + 1))
    return out


@pytest.mark.parametrize("total", [8, 100001, 1_280_000, 25_600_001])
def test_projection_morsels_cover_every_row_in_order(total):
    # one partition = several morsels (160,000 rows, then doubling): the rows of
    # each partition arrive complete and in order
    import fq_ref as R
    r = E.execute("SELECT number, number+1 FROM system.numbers_mt(%d) WHERE number %% 97 = 5" % total)
    got = [a for a, _ in r.rows]
    assert all(b == a + 1 for a, b in r.rows)
    exp = [x for x in _stream_rows(total) if x % 97 == 5]
    assert sorted(got) == exp
    # within a partition the order is the stream's
    for b, e in R.generate_parts(total):
        part = [x for x in got if b <= x <= e]
        assert part == sorted(part)


def test_limit_over_ten_billion_rows_stops_early():
    # README.md:116-127 at numbers_mt(1e10), nothing resident: the pipes stop
    # after their first morsels (the reference's LimitStream stops pulling),
    # instead of materialising 8 x 10 GB partitions
    import time
    e = Engine()
    try:
        t = time.perf_counter()
        r = e.execute("select (number+1) as c1, number/2 as c2 from system.numbers_mt(10000000000) "
                      "where (c1+c2+1) < 100 limit 3")
        dt = time.perf_counter() - t
        assert r.rows == [(1, 0), (2, 0), (3, 1)]
        r = e.execute("SELECT number FROM system.numbers_mt(10000000000) LIMIT 5")
        assert len(r.rows) == 5
        assert all(v % 1250000000 < 160000 for (v,) in r.rows)  # first morsel of some partition
        assert dt < 5.0, dt
    finally:
        e.close()


@pytest.mark.parametrize("n", [0, 1, 9999, 10000, 100001, 80_000_000])
def test_count_only_reads_no_column(n):
    # count(number) alone: the reference's Count adds block.num_rows()
    # (function_aggregator.rs:60-66); the device path counts rows without a scan
    import fq_ref as R
    from fq_amd import ops
    if n:
        r = q("SELECT count(number) FROM system.numbers_mt(%d)" % n)
        exp = R.aggregate_query(n, [R.E_fn("count", R.E_field("number"))]) if n <= 100001 else None
        rows = sum(be - bb + 1 for b, e in R.generate_parts(n) for bb, be in R.numbers_blocks(b, e))
        assert r.rows == [(rows,)]
        if exp is not None:
            assert r.rows == [tuple(v.value for v in exp)]
    col = ops.numbers_column(0, n)
    st = ops.aggregate(col, 10000, None, None, abi.AGG_COUNT)
    assert st.count == n and st.blocks == (n + 9999) // 10000


@pytest.mark.parametrize("sql", [
    "SELECT sum(number)/count(number), max(number), min(number), count(number), sum(number) FROM system.numbers_mt(%d)",
    "SELECT max(number+1), count(number), min(number*3) FROM system.numbers_mt(%d) WHERE (number%%8)<3",
    "SELECT sum(number) FROM system.numbers_mt(%d) WHERE number %% 100000 < 3",   # empty blocks -> the reference's error
    "SELECT sum(number+1) FROM system.numbers_mt(%d) WHERE number %% 7 = 2",
    "SELECT number%%10, count(number), max(number) FROM system.numbers_mt(%d) GROUP BY number%%10",
])
def test_generated_partitions_stream_in_chunks(sql):
    # numbers_mt partitions that are not resident are read in FQ_OPT_CHUNK_ROWS
    # device blocks (whole 10,000-row blocks): the same results and errors as
    # one block per partition
    from fq_amd import FQError
    from fq_amd.engine import OPT_CHUNK_ROWS
    n = 1_000_003
    e = Engine()
    try:
        e.set_option(OPT_CHUNK_ROWS, 30000)
        try:
            got = e.execute(sql % n).rows
        except FQError as ex:
            got = ("error", str(ex))
    finally:
        e.close()
    try:
        exp = q(sql % n).rows
    except FQError as ex:
        exp = ("error", str(ex))
    assert got == exp
    with pytest.raises(FQError):
        E.set_option(OPT_CHUNK_ROWS, 12345)


def test_non_resident_numbers_mt_beyond_hbm():
    # numbers_mt(4e11): 3.2 TB generated in 3.2 GB chunks -- the reference
    # streams it through 10,000-row blocks; one device block per partition
    # would need 400 GB of HBM
    e = Engine()
    try:
        r = e.execute("SELECT count(number), max(number), min(number) FROM system.numbers_mt(400000000000)")
        assert r.rows == [(400000000000, 399999999999, 0)]
    finally:
        e.close()


def test_row_pipeline_over_resident_partitions_matches_generated():
    # morsels of a materialised partition are slices of its resident column;
    # the same query over generated partitions must return the same rows
    n = 40_000_000
    sql = ("SELECT number, number*3 + number%%7 FROM system.numbers_mt(%d) WHERE number %% 999983 < 2" % n)
    gen = sorted(q(sql).rows)
    e = Engine()
    try:
        e.materialize_numbers(n)
        res = sorted(e.execute(sql).rows)
        lim = e.execute("SELECT number FROM system.numbers_mt(%d) WHERE number %% 999983 = 1 LIMIT 3" % n).rows
    finally:
        e.close()
    assert res == gen
    assert [r[0] for r in gen] == [x for x in range(n) if x % 999983 < 2]
    assert all(b == a * 3 + a % 7 for a, b in gen)
    assert len(lim) == 3 and all(v % 999983 == 1 for (v,) in lim)


def test_device_block_cache_reuse_across_queries_and_engines():
    # engine/core.cpp BlockCache: buffers freed on a queue are reused by later
    # allocations on that queue (morsel outputs, fused-scan states, workspaces).
    # Interleave row pipelines of different morsel sizes with aggregates, three
    # rounds, then close the engine (its queues' cached blocks are freed) and
    # run again on a fresh one: every result stays exact.
    cases = []
    for total in (100001, 1_280_000, 5_000_000):
        exp = [x for x in _stream_rows(total) if x % 31 == 7]
        cases.append(("SELECT number, number*3 FROM system.numbers_mt(%d) WHERE number %% 31 = 7" % total,
                      sorted((x, 3 * x) for x in exp)))
        rows = _stream_rows(total)
        cases.append(("SELECT sum(number), count(number), max(number) FROM system.numbers_mt(%d)" % total,
                      [(sum(rows) % 2**64, len(rows), max(rows))]))
    cases.append(("SELECT number FROM system.numbers_mt(1000000) LIMIT 5", None))

    def run(eng):
        for sql, exp in cases:
            r = eng.execute(sql)
            if exp is None:
                assert len(r.rows) == 5
                assert all(0 <= v < 1000000 for (v,) in r.rows)
            else:
                assert sorted(r.rows) == exp, sql

    e = Engine()
    try:
        for _ in range(3):
            run(e)
    finally:
        e.close()
    e2 = Engine()
    try:
        run(e2)
    finally:
        e2.close()
