"""Expression trees in the fused device path (FQ_OP_PUSH / FQ_OPERAND_STACK,
hipRTC kernels): kernel-level parity against the C oracle's tree evaluation
(fq_aggregate value/predicate, fq_filter_project), and SQL-level parity of
the engine (aggregates, WHERE, projection, GROUP BY key) against the numpy
restatement of the reference's Function trees (oracle/fq_ref.py).  Integer
results bit-exact."""
import numpy as np
import pytest

from fq_amd import abi
from fq_amd.expr import COL, PUSH, STACK, chain, predicate

import oracle_c
from replay import as_tuple, replay

pytestmark = pytest.mark.gpu

ops = None
E = None
U64, I64, F64 = abi.DT_UINT64, abi.DT_INT64, abi.DT_FLOAT64
AGGS = [abi.AGG_SUM, abi.AGG_MAX, abi.AGG_MIN, abi.AGG_COUNT]
ALL = abi.AGG_SUM | abi.AGG_MAX | abi.AGG_MIN | abi.AGG_COUNT

TREES = [
    (U64, [("+", 1), PUSH, ("/", 2), ("+", STACK, True)]),
    (U64, [("+", 1), PUSH, ("+", 2), ("*", STACK, True), ("%", 1000003)]),
    (U64, [("/", 3), PUSH, ("%", 7), ("*", 2), ("-", STACK, True)]),
    (U64, [("+", 1), PUSH, ("/", 2.0), ("+", STACK, True)]),
    (U64, [("+", 1), PUSH, ("+", 2), PUSH, ("%", 5), ("-", STACK, True), ("*", STACK, True)]),
    (U64, [("-", (5, "Int64")), PUSH, ("*", 3), ("+", STACK, True)]),
    (I64, [("*", (3, "Int64")), PUSH, ("%", (7, "Int64")), ("+", (1, "Int64")), ("/", STACK, True)]),
    (F64, [("*", 2.0), PUSH, ("+", COL), ("/", STACK, True)]),
]


def setup_module():
    global ops, E
    from fq_amd import ops as _ops
    _ops.require_gpu()
    _ops.jit_config(abi.JIT_AUTO, 1 << 22)
    ops = _ops
    from fq_amd.engine import Engine
    E = Engine()


def teardown_module():
    if E is not None:
        E.close()


def _column(dt, n, seed):
    rng = np.random.default_rng(seed)
    if dt == U64:
        return rng.integers(0, 2**40, size=n, dtype=np.uint64)
    if dt == I64:
        return rng.integers(-2**40, 2**40, size=n, dtype=np.int64)
    return rng.standard_normal(n) * 1000.0


def _check(host, dt, block_rows, pred=None, value=None):
    col = ops.from_numpy(host, dt)
    aggs = [(op, value) for op in AGGS]
    try:
        exp = [as_tuple(s) for s in oracle_c.column_partial(host, dt, block_rows, aggs, pred)]
        exp_err = None
    except oracle_c.OracleError as e:
        exp, exp_err = None, e
    st = ops.aggregate(col, block_rows, pred, value, ALL)
    if exp_err is not None:
        with pytest.raises(oracle_c.OracleError) as ei:
            for op in AGGS:
                replay(op, st)
        assert str(ei.value) == str(exp_err)
        return
    got = [replay(op, st) for op in AGGS]
    if dt == F64 or (value is not None and value.out_dtype == F64):
        for g, x in zip(got, exp):  # sums: reduction order differs (rel 1e-12)
            gv, xv = np.frombuffer(np.uint64(g[2]).tobytes(), np.float64)[0], np.frombuffer(np.uint64(x[2]).tobytes(), np.float64)[0]
            assert g[:2] == x[:2] and (gv == xv or abs(gv - xv) <= 1e-12 * abs(xv)), (g, x)
    else:
        assert got == exp, (got, exp)


@pytest.mark.parametrize("i", range(len(TREES)))
@pytest.mark.parametrize("n", [1, 1000, 65_537, 300_001])
def test_tree_value_matches_oracle(i, n):
    dt, steps = TREES[i]
    host = _column(dt, n, 100 + i)
    _check(host, dt, 10000, value=chain(dt, steps)[0])


@pytest.mark.parametrize("i", range(len(TREES)))
def test_tree_predicate_matches_oracle(i):
    dt, steps = TREES[i]
    host = _column(dt, 200_003, 200 + i)
    rhs = {U64: 2**39, I64: (0, "Int64"), F64: 0.5}[dt]
    pred = predicate(dt, steps, "<", rhs)
    _check(host, dt, 10000, pred=pred, value=chain(dt, [("+", 1)] if dt != I64 else [("+", (1, "Int64"))])[0])
    # block mode (filtered sum over several reference blocks)
    _check(host, dt, 10000, pred=pred)


def test_tree_numbers_iota_and_division_by_zero_in_right_subtree():
    host = np.arange(100_000, dtype=np.uint64)
    _check(host, U64, 10000, value=chain(U64, [("+", 1), PUSH, ("%", 4), ("/", STACK, True)])[0])  # x%4 == 0 -> error
    _check(host, U64, 10000, value=chain(U64, [("+", 1), PUSH, ("%", 4), ("+", 1), ("/", STACK, True)])[0])


def test_tree_needs_the_jit():
    col = ops.from_numpy(np.arange(1000, dtype=np.uint64))
    ops.jit_config(abi.JIT_OFF)
    try:
        with pytest.raises(ops.FQError) as ei:
            ops.aggregate(col, 10000, None, chain(U64, TREES[0][1])[0], ALL)
        assert ei.value.status == abi.FQ_E_UNSUPPORTED
    finally:
        ops.jit_config(abi.JIT_AUTO, 1 << 22)


def test_tree_filter_project():
    host = np.arange(250_000, dtype=np.uint64)
    col = ops.from_numpy(host)
    pred = predicate(U64, [("+", 1), PUSH, ("/", 2), ("+", STACK, True), ("+", 1)], "<", 100_000)
    outs = ops.filter_project(col, pred, [chain(U64, TREES[1][1])[0], chain(U64, TREES[3][1])[0]])
    k = host[(host + 1) + host // 2 + 1 < 100_000]
    assert np.array_equal(outs[0].to_numpy(), ((k + np.uint64(1)) * (k + np.uint64(2))) % np.uint64(1000003))
    assert np.array_equal(outs[1].to_numpy(), (k + np.uint64(1)).astype(np.float64) + k.astype(np.float64) / 2.0)


# ---- SQL: the engine fuses trees; fq_ref evaluates the reference's Functions

def _ref():
    import fq_ref as R
    N, c = R.E_field("number"), R.E_const
    return R, N, c


def test_sql_tree_aggregates_match_oracle():
    R, N, c = _ref()
    n = 1_000_000
    r = E.execute("SELECT sum((number+1)*(number+2)), max(number*3 + number/7), min((number%1000) - (number%7)), "
                  "count(number) FROM system.numbers_mt({N})".replace("{N}", str(n)))
    B = R.E_bin
    exp = R.aggregate_query(n, [
        R.E_fn("sum", B("*", B("+", N, c(1)), B("+", N, c(2)))),
        R.E_fn("max", B("+", B("*", N, c(3)), B("/", N, c(7)))),
        R.E_fn("min", B("-", B("%", N, c(1000)), B("%", N, c(7)))),
        R.E_fn("count", N)])
    assert r.rows == [tuple(v.value for v in exp)]


def test_sql_tree_where_matches_oracle():
    R, N, c = _ref()
    n = 2_000_000
    B = R.E_bin
    r = E.execute("SELECT count(number), sum(number), max(number) FROM system.numbers_mt({N}) "
                  "WHERE (number % 100) * (number % 7) < 50".replace("{N}", str(n)))
    w = B("<", B("*", B("%", N, c(100)), B("%", N, c(7))), c(50))
    exp = R.aggregate_query(n, [R.E_fn("count", N), R.E_fn("sum", N), R.E_fn("max", N)], where=w)
    assert r.rows == [tuple(v.value for v in exp)]


def test_sql_readme_query_fully_fused():
    # README.md:116-127 at numbers_mt(1e10): the WHERE (after FilterPushDown)
    # and both projections run as one fq_filter_project per morsel
    j0 = ops.jit_stats()["jit_launches"]
    r = E.execute("select (number+1) as c1, number/2 as c2 from system.numbers_mt(10000000000) "
                  "where (c1+c2+1) < 100 limit 3")
    assert r.rows == [(1, 0), (2, 0), (3, 1)]
    assert ops.jit_stats()["jit_launches"] > j0


def test_sql_tree_projection_matches_oracle():
    R, N, c = _ref()
    n = 100_000
    B = R.E_bin
    r = E.execute("SELECT (number+1)*(number%3), number/2 + number%5 FROM system.numbers_mt({N}) "
                  "WHERE (number % 10) + (number % 7) = 3".replace("{N}", str(n)))
    exp = R.projection_query(n, [B("*", B("+", N, c(1)), B("%", N, c(3))), B("+", B("/", N, c(2)), B("%", N, c(5)))],
                             where=B("=", B("+", B("%", N, c(10)), B("%", N, c(7))), c(3)))
    assert sorted(r.rows) == sorted(exp)


def test_sql_tree_group_by_key():
    n = 80_000
    r = E.execute("SELECT (number%10)*(number%3), count(number) FROM system.numbers_mt({N}) "
                  "GROUP BY (number%10)*(number%3)".replace("{N}", str(n)))
    keys = (np.arange(n) % 10) * (np.arange(n) % 3)
    u, cnt = np.unique(keys, return_counts=True)
    assert r.rows == [(int(a), int(b)) for a, b in zip(u, cnt)]


def test_sql_trees_with_jit_off_fall_back_to_per_node_kernels():
    n = 100_000
    sql = ("SELECT sum((number+1)*(number+2)), max(number*3 + number/7) FROM system.numbers_mt({N}) "
           "WHERE (number % 100) * (number % 7) < 50".replace("{N}", str(n)))
    fused = E.execute(sql).rows
    ops.jit_config(abi.JIT_OFF)
    try:
        from fq_amd.engine import Engine
        e = Engine()
        try:
            assert e.execute(sql).rows == fused
        finally:
            e.close()
    finally:
        ops.jit_config(abi.JIT_AUTO, 1 << 22)
