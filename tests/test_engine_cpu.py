"""CPU: the engine's host-side layers without a GPU (device = -1): SQL
planning, EXPLAIN text, plan-time error texts, and the AggregateFinal merge of
exchanged partial states.  Anything that would touch a column must fail
loudly -- there is no CPU fallback for the hot path."""
import struct

import pytest

import fq_ref as R
from fq_amd import FQError, abi
from fq_amd.engine import Engine
from fq_amd.expr import to_bits
from fq_amd.numbers import generate_parts, shard

README_SQL = ("select (number+1) as c1, number/2 as c2 from system.numbers_mt(10000000) "
              "where ((number+1)+(number/2)+1) < 100 limit 3")


@pytest.fixture(scope="module")
def eng():
    e = Engine(device=-1)
    yield e
    e.close()


def encode_states(per_func):
    """The engine's partial-state wire format (pipeline.cpp encode_states)."""
    out = b"FQS1" + struct.pack("<I", len(per_func))
    for vals in per_func:
        out += struct.pack("<II", len(vals), 0)
        for v in vals:
            kind = 0 if v.type == "Null" else (1 if v.value is None else 2)
            dt = abi.DT_BY_NAME[v.type] if kind else 0
            out += struct.pack("<iiQ", kind, dt, to_bits(v.value, dt) if kind == 2 else 0)
    return out


def test_explain_plan_and_pipeline_text(eng):
    # README.md:98-113 (plan + pipeline display)
    txt = eng.explain(README_SQL)
    assert txt == (
        "└─ Limit: 3\n  └─ Projection: (number + 1) as c1, (number / 2) as c2\n"
        "    └─ Filter: ((((number + 1) + (number / 2)) + 1) < 100)\n"
        "      └─ ReadDataSource: scan parts [8](Read from system.numbers_mt table)\n"
        "\n  └─ LimitTransform × 1 processor\n    └─ Merge (LimitTransform × 8 processors) to (MergeProcessor × 1)"
        "\n      └─ LimitTransform × 8 processors\n        └─ ProjectionTransform × 8 processors"
        "\n          └─ FilterTransform × 8 processors\n            └─ SourceTransform × 8 processors")


README_ALIAS_SQL = ("select (number+1) as c1, number/2 as c2 from system.numbers_mt(10000000) "
                    "where (c1+c2+1) < 100 limit 3")  # README.md:96, verbatim


def test_filter_push_down_optimizer(eng):
    # optimizers/optimizer_filter_push_down_test.rs:19-32: aliases in WHERE are
    # replaced by the projected expressions
    txt = eng.explain("select (number+1) as c1, number as c2 from system.numbers_mt where (c1+c2+1)=1")
    assert txt.startswith("└─ Projection: (number + 1) as c1, number as c2"
                          "\n  └─ Filter: ((((number + 1) + number) + 1) = 1)"
                          "\n    └─ ReadDataSource: scan parts [8](Read from system.numbers_mt table)\n")


def test_readme_explain_with_aliases(eng):
    # README.md:96-113: the optimised plan of the aliased statement is the one
    # the README prints
    assert eng.explain(README_ALIAS_SQL) == eng.explain(README_SQL)
    assert eng.explain("explain " + README_ALIAS_SQL) == eng.explain(README_SQL)


def test_filter_push_down_leaves_other_fields(eng):
    # a Field that names no projection output stays; an aggregate plan's map
    # is built below the Aggregate (optimizer.rs:48-50) and is empty here
    assert "Filter: (number > 1)" in eng.explain(
        "select number+1 as c1 from system.numbers_mt(100) where number > 1")
    assert "Filter: (c1 > 1)" in eng.explain("select sum(number) as c1 from system.numbers_mt(100) where c1 > 1")


def test_explain_worker_threads_chunking():
    # pipeline_builder.rs:75-84: workers < partitions -> chunks of parts/workers per source
    with Engine(device=-1, worker_threads=2) as e:
        txt = e.explain("SELECT sum(number) FROM system.numbers_mt(1000)")
    assert "AggregatePartialTransform × 2 processors" in txt and "SourceTransform × 2 processors" in txt


def test_small_n_single_partition(eng):
    assert "scan parts [1]" in eng.explain("SELECT sum(number) FROM system.numbers_mt(7)")


@pytest.mark.parametrize("sql,msg", [
    ("SELECT max(number) FROM system.numbers_mt(10) WHERE number %% 8 < 3", None),
    ("SELECT avg(number) FROM system.numbers_mt(10)", "Internal Error: Unsupported Function: avg"),
    ("SELECT number FROM system.nope(10)", "Internal Error: Cannot find the table: nope"),
    ("SELECT number FROM nope.numbers_mt(10)", "Internal Error: Cannot find the database: nope"),
    ("SELECT number FROM numbers_mt(10)", "Internal Error: Cannot find the database: default"),
    ("SELECT sum(number), number FROM system.numbers_mt(10)",
     "Error during plan: Projection references non-aggregate values"),
    ("SELECT sum(number) FROM system.numbers_mt(10) HAVING sum(number) > 1",
     "Internal Error: HAVING is not implemented yet"),
    ("SELECT number FROM system.numbers_mt(10) LIMIT 1.5",
     "Error during plan: Unexpected expression for LIMIT clause"),
    ("SELECT sum(number) + 'a' FROM system.numbers_mt(10)", "Internal Error: Unsupported (UInt64) + (Utf8)"),
    ("SELECT nope FROM system.numbers_mt(10)",
     'Internal Error: Invalid argument error: Unable to get field named "nope". Valid fields: ["number"]'),
])
def test_plan_time_errors(eng, sql, msg):
    sql = sql.replace("%%", "%")
    if msg is None:
        eng.explain(sql)  # '%' is accepted (extension on by default)
        return
    with pytest.raises(FQError) as ei:
        eng.explain(sql)
    assert str(ei.value) == msg


def test_modulo_off_matches_reference_error():
    with Engine(device=-1, modulo=False) as e:
        with pytest.raises(FQError) as ei:
            e.explain("SELECT max(number+1) FROM system.numbers_mt(100) WHERE (number%8)<3")
    assert str(ei.value) == "Internal Error: Unsupported Function: %"


def test_host_only_engine_has_no_cpu_fallback(eng):
    with pytest.raises(FQError) as ei:
        eng.execute("SELECT sum(number) FROM system.numbers_mt(10)")
    assert ei.value.status == abi.FQ_E_HIP


def test_result_column_names_follow_function_debug(eng):
    n = R.E_field("number")
    exprs = [R.E_bin("/", R.E_fn("sum", n), R.E_fn("count", n)), R.E_fn("max", n), R.E_fn("min", n)]
    states = [encode_states(R.aggregate_partial_states(80, exprs, [(b, e) for _, b, e in generate_parts(80)]))]
    r = eng.execute_final("SELECT sum(number)/count(number), max(number), min(number) "
                          "FROM system.numbers_mt(80)", states)
    assert r.names == ["Sum(number) / Count(number)", "Max(number)", "Min(number)"]
    assert r.rows == [(39, 79, 0)]
    # the reference's MySQL writer: UInt64 -> MYSQL_TYPE_LONG (mysql_stream.rs:32-45),
    # values through arrow array_value_to_string
    assert r.mysql_types == [3, 3, 3] and r.mysql_error is None
    assert r.text_rows == [("39", "79", "0")]


def test_result_mysql_float_type_and_text(eng):
    n = R.E_field("number")
    exprs = [R.E_fn("sum", R.E_bin("/", n, R.E_const(2.0))), R.E_fn("max", R.E_bin("*", n, R.E_const(1.5)))]
    states = [encode_states(R.aggregate_partial_states(80, exprs, [(b, e) for _, b, e in generate_parts(80)]))]
    r = eng.execute_final("SELECT sum(number/2.0), max(number*1.5) FROM system.numbers_mt(80)", states)
    assert r.mysql_types == [4, 4]  # Float64 -> MYSQL_TYPE_FLOAT
    assert r.text_rows == [("1580", "118.5")]  # Rust f64 Display


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("n", [7, 80000, 1000000, 123457])
def test_final_merge_of_sharded_partials_matches_oracle(eng, world, n):
    num = R.E_field("number")
    exprs = [R.E_bin("/", R.E_fn("sum", num), R.E_fn("count", num)), R.E_fn("max", num), R.E_fn("min", num),
             R.E_bin("+", R.E_fn("sum", R.E_bin("*", num, R.E_const(3))), R.E_const(1))]
    sql = ("SELECT sum(number)/count(number), max(number), min(number), sum(number*3)+1 "
           "FROM system.numbers_mt(%d)" % n)
    parts = generate_parts(n)
    states = [encode_states(R.aggregate_partial_states(n, exprs, [(b, e) for _, b, e in shard(parts, r, world)]))
              for r in range(world)]
    got = eng.execute_final(sql, states).rows
    exp = [tuple(v.value for v in R.aggregate_query(n, exprs))]
    assert got == exp


def test_final_merge_none_error(eng):
    # one rank Some(10), the others None: only the cross-rank merge fails
    num = R.E_field("number")
    where = R.E_bin("<", num, R.E_const(5))
    parts = generate_parts(80)
    states = [encode_states(R.aggregate_partial_states(80, [R.E_fn("sum", num)], [(b, e) for _, b, e in
                                                                                    shard(parts, r, 8)], where))
              for r in range(8)]
    with pytest.raises(FQError) as ei:
        eng.execute_final("SELECT sum(number) FROM system.numbers_mt(80) WHERE number < 5", states)
    assert str(ei.value) == "Internal Error: DataValue to array cannot be NONE NULL"


# ---- GROUP BY: planning and the cross-rank merge (host-only engine) ----
GB_SQL = ("SELECT number%%10, count(number), sum(number)/count(number), max(number+1) "
          "FROM system.numbers_mt(%d) WHERE (number%%8)<3 GROUP BY number%%10")


def _gb_exprs():
    n = R.E_field("number")
    key = R.E_bin("%", n, R.E_const(10))
    exprs = [R.E_fn("count", n), R.E_bin("/", R.E_fn("sum", n), R.E_fn("count", n)),
             R.E_fn("max", R.E_bin("+", n, R.E_const(1)))]
    where = R.E_bin("<", R.E_bin("%", n, R.E_const(8)), R.E_const(3))
    return key, exprs, where


def test_group_by_explain_keeps_reference_display(eng):
    txt = eng.explain("SELECT number%10, sum(number) FROM system.numbers_mt(80000) GROUP BY number%10")
    # plan_display.rs:37-50: aggregate list, then the group list with no separator
    assert txt.splitlines()[0] == "└─ Aggregate: sum([number])(number % 10)"
    assert "AggregatePartialTransform × 8 processors" in txt and "AggregateFinalTransform × 1 processor" in txt


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("total", [80000, 123457])
def test_group_by_final_merge_of_sharded_partials(eng, world, total):
    key, exprs, where = _gb_exprs()
    parts = [(b, e) for _, b, e in generate_parts(total)]
    states = []
    for r in range(world):
        mine = parts[len(parts) * r // world: len(parts) * (r + 1) // world]
        states.append(encode_states(R.group_by_partial_states(total, key, exprs, mine, where)))
    res = eng.execute_final(GB_SQL % total, states)
    assert res.rows == R.group_by_query(total, key, exprs, where)
    assert res.names == ["number % 10", "Count(number)", "Sum(number) / Count(number)", "Max(number + 1)"]


def test_group_by_plan_errors(eng):
    with pytest.raises(FQError) as ei:
        eng.explain("SELECT number, number+1, sum(number) FROM system.numbers_mt(10) GROUP BY number%3")
    assert str(ei.value) == "Error during plan: Projection references non-aggregate values"


def test_explain_logic_predicate(eng):
    txt = eng.explain("SELECT sum(number) FROM system.numbers_mt(80000) WHERE number > 1 AND number < 5")
    assert "Filter: ((number > 1) AND (number < 5))" in txt


@pytest.mark.parametrize("exprs,nvals", [
    ("sum(number)/count(number), max(number), min(number)", [2, 1, 1]),  # C3
    ("sum(number)", [1]),  # C2
    ("max(number+1), count(number)", [1, 1]),
    ("(sum(number)+1)*max(number)", [3]),  # the constant has a state value too (function_constant.rs)
])
def test_partial_state_bytes_is_the_states_size_on_every_rank(eng, exprs, nvals):
    """fq_engine_partial_state_bytes: the serialised partial states' size is a
    function of the SQL alone (one 16-byte record per accumulate_result value,
    function.rs:28-131), so the exchange sizes its one all-reduce without first
    exchanging lengths; the oracle's states (Null on a rank that owns nothing,
    Some elsewhere) all encode to it."""
    sql = "SELECT %s FROM system.numbers_mt(%%d)" % exprs
    exp = 8 + sum(8 + 16 * k for k in nvals)
    for n in (7, 1000000):
        assert eng.partial_state_bytes(sql % n) == exp
    if exprs.startswith("sum(number)/"):
        num = R.E_field("number")
        fs = [R.E_bin("/", R.E_fn("sum", num), R.E_fn("count", num)), R.E_fn("max", num), R.E_fn("min", num)]
        for parts in ([], [(b, e) for _, b, e in generate_parts(1000000)][:3]):
            assert len(encode_states(R.aggregate_partial_states(1000000, fs, parts))) == exp


def test_partial_state_bytes_group_by_and_errors(eng):
    # GROUP BY states grow with the groups: 0 = lengths go first
    assert eng.partial_state_bytes("SELECT number%10, count(number) FROM system.numbers_mt(100) GROUP BY number%10") == 0
    with pytest.raises(FQError, match="aggregate queries only"):
        eng.partial_state_bytes("SELECT number FROM system.numbers_mt(100)")
