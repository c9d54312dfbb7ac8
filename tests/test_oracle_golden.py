"""CPU: pin the oracles against the reference's own test vectors
(tests/golden/reference_vectors.json, extracted from its *_test.rs tables),
its hand-written function/transform test expectations, the README and the
closed forms; and cross-check the two oracles (numpy restatement vs the C
faithful-structure path) on random small queries."""
import json
import os

import numpy as np
import pytest

import fq_ref as R
import oracle_c
from fq_amd import abi
from fq_amd.expr import chain, predicate

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.json")))


def lit(d):
    if d["array"]:
        vals = d["values"]
        return R.Arr(d["type"], vals) if d["type"] in R.NP else R.Arr(d["type"], list(vals))
    return R.Value(d["type"], d.get("value") if d["kind"] == "some" else None)


def same_array(got, exp):
    if got.type != exp["type"]:
        return False
    vals = got.to_list()
    if exp["type"] == "Float32":
        return np.array_equal(np.float32(vals), np.float32(exp["values"]))
    return vals == exp["values"]


def same_value(got, exp):
    return got == lit(exp)


def run_table(t, fn):
    """Reference harness: Ok -> compare with expect[i]; Err -> error[i] text."""
    results = []
    cases = t["args"] if "args" in t else [None]
    for i, args in enumerate(cases):
        try:
            results.append(("ok", fn(args)))
        except R.RefError as e:
            results.append(("err", str(e)))
    return results


def ids(tables):
    return ["%s:%s" % (t["fn"], t["name"]) for t in tables]


@pytest.mark.parametrize("t", GOLDEN["array_arithmetic"], ids=ids(GOLDEN["array_arithmetic"]))
def test_golden_array_arithmetic(t):
    if "args" in t:
        for i, (l, r) in enumerate(t["args"]):
            try:
                got = R.data_array_arithmetic_op(t["op"], lit(l), lit(r))
                assert same_array(got, t["expect"][i]), (i, got.to_list(), t["expect"][i])
            except R.RefError as e:
                assert str(e) == t["error"][i]
    else:
        arr, sc = lit(t["array"]), lit(t["scalar"])
        if t["fn"] == "test_array_scalar_arithmetic":
            got = R.data_array_arithmetic_op(t["op"], arr, sc)
        else:
            got = R.data_array_arithmetic_op(t["op"], sc, arr)
        assert same_array(got, t["expect"])


@pytest.mark.parametrize("t", GOLDEN["array_comparison"], ids=ids(GOLDEN["array_comparison"]))
def test_golden_array_comparison(t):
    if "args" in t:
        for i, (l, r) in enumerate(t["args"]):
            got = R.data_array_comparison_op(t["op"], lit(l), lit(r))
            assert same_array(got, t["expect"][i]), (i, got.to_list())
    else:
        arr, sc = lit(t["array"]), lit(t["scalar"])
        if t["fn"] == "test_array_scalar_comparison":
            got = R.data_array_comparison_op(t["op"], arr, sc)
        else:
            got = R.data_array_comparison_op(t["op"], sc, arr)
        assert same_array(got, t["expect"])


@pytest.mark.parametrize("t", GOLDEN["array_aggregate"], ids=ids(GOLDEN["array_aggregate"]))
def test_golden_array_aggregate(t):
    for i, a in enumerate(t["args"]):
        try:
            got = R.data_array_aggregate_op(t["op"], lit(a))
            assert same_value(got, t["expect"][i]), (i, got, t["expect"][i])
        except R.RefError as e:
            assert str(e) == t["error"][i]


@pytest.mark.parametrize("t", GOLDEN["value_aggregate"] + GOLDEN["value_arithmetic"],
                         ids=ids(GOLDEN["value_aggregate"] + GOLDEN["value_arithmetic"]))
def test_golden_value_ops(t):
    for i, (l, r) in enumerate(t["args"]):
        try:
            if t["op"] in R.ARITH:
                got = R.data_value_arithmetic_op(t["op"], lit(l), lit(r))
            else:
                got = R.data_value_aggregate_op(t["op"], lit(l), lit(r))
            assert same_value(got, t["expect"][i]), (i, got, t["expect"][i])
        except R.RefError as e:
            assert str(e) == t["error"][i]


@pytest.mark.parametrize("t", GOLDEN["array_logic"], ids=ids(GOLDEN["array_logic"]))
def test_golden_array_logic(t):
    for i, (l, r) in enumerate(t["args"]):
        got = R.data_array_logic_op(t["op"], lit(l), lit(r))
        assert same_array(got, t["expect"][i]), (i, got.to_list())


def test_function_logic_display_and_eval():
    # function_logic_test.rs:28-80
    b = R.Block({"a": R.Arr("Boolean", [True, True, True, False]), "b": R.Arr("Boolean", [True, False, True, True])})
    f = R.to_function(R.E_bin("and", R.E_field("a"), R.E_field("b")))
    assert f.display() == "a and b" and f.eval(b).to_list() == [True, False, True, False]
    f = R.to_function(R.E_bin("or", R.E_field("a"), R.E_field("b")))
    assert f.display() == "a or b" and f.eval(b).to_list() == [True, True, True, True]
    with pytest.raises(R.RefError, match="Unsupported aggregate operation for function and"):
        R.to_function(R.E_bin("and", R.E_field("a"), R.E_field("b"))).accumulate_result()


def test_golden_fixture_covers_all_tables():
    n = {k: len(v) for k, v in GOLDEN.items() if isinstance(v, list)}
    assert n == {"array_arithmetic": 12, "array_comparison": 17, "array_aggregate": 3,
                 "value_aggregate": 3, "value_arithmetic": 1, "array_logic": 2,
                 "function_arithmetic": 5, "function_comparison": 1}


FUNCTION_TABLES = GOLDEN["function_arithmetic"] + GOLDEN["function_comparison"]


def function_block(t):
    """The table's block: columns a, b, c in schema order (the arrays as the
    test builds them, whatever the schema's declared types)."""
    return R.Block({n: lit(c) for n, c in zip("abc", t["columns"])})


@pytest.mark.parametrize("t", FUNCTION_TABLES, ids=ids(FUNCTION_TABLES))
def test_golden_function_tables(t):
    # function_arithmetic_test.rs:28-160 / function_comparison_test.rs:25-85:
    # Function over two fields -> display, nullable, eval = expect
    lhs, op, rhs = t["display"].split(" ")
    assert op == t["op"]
    f = R.to_function(R.E_bin(op, R.E_field(lhs), R.E_field(rhs)))
    assert f.display() == t["display"]
    assert t["nullable"] is False and t["error"] == ""
    got = f.eval(function_block(t))
    assert same_array(got, t["expect"]), (got.to_list(), t["expect"])


# ---- function_aggregator_test.rs:5-192 (partial/merge protocol) -----------

def block_ab():
    return R.Block({"a": R.Arr("Int64", [4, 3, 2, 1]), "b": R.Arr("Int64", [1, 2, 3, 4])})


@pytest.mark.parametrize("name,evals,expr,expect", [
    ("count-passed", 1, R.E_fn("count", R.E_field("a")), R.Value("UInt64", 4)),
    ("max-passed", 2, R.E_fn("max", R.E_field("a")), R.Value("Int64", 4)),
    ("min-passed", 2, R.E_fn("min", R.E_field("a")), R.Value("Int64", 1)),
    ("sum-passed", 1, R.E_fn("sum", R.E_field("a")), R.Value("Int64", 10)),
    ("sum(a)+1-merge-passed", 4, R.E_bin("+", R.E_fn("sum", R.E_field("a")), R.E_const(1, "Int64")),
     R.Value("Int64", 71)),
    ("sum(a)/count(a)-merge-passed", 4,
     R.E_bin("/", R.E_fn("sum", R.E_field("a")), R.E_fn("count", R.E_field("a"))), R.Value("Int64", 2)),
    ("(sum(a+1)+2)-merge-passed", 4,
     R.E_bin("+", R.E_fn("sum", R.E_bin("+", R.E_field("a"), R.E_const(1, "Int8"))), R.E_const(2, "Int8")),
     R.Value("Int64", 100)),
])
def test_function_aggregator_protocol(name, evals, expr, expect):
    # func1 accumulates `evals` times, func2 `evals - 1` times, final merges both
    f1 = R.to_function(expr)
    for _ in range(evals):
        f1.accumulate(block_ab())
    f2 = R.to_function(expr)
    for _ in range(1, evals):
        f2.accumulate(block_ab())
    final = R.to_function(expr)
    final.set_depth(0)
    final.merge_state(f1.accumulate_result())
    final.merge_state(f2.accumulate_result())
    assert final.merge_result() == expect


def test_function_display_strings():
    f = R.to_function(R.E_bin("/", R.E_fn("sum", R.E_field("number")), R.E_fn("count", R.E_field("number"))))
    assert f.display() == "Sum(number) / Count(number)"
    assert R.to_function(R.E_bin("+", R.E_field("a"), R.E_const(1))).display() == "a + 1"


# ---- transform tests + README (numbers_mt) ---------------------------------

def test_transform_aggregate_122():
    # transform_aggregate_test.rs:5-59
    got = R.aggregate_query(16, [R.E_bin("+", R.E_fn("sum", R.E_field("number")), R.E_const(2))])
    assert got == [R.Value("UInt64", 122)]


def test_transform_filter_eq_1():
    # transform_filter_test.rs:5-44
    rows = R.projection_query(8, [R.E_field("number")], where=R.E_bin("=", R.E_field("number"), R.E_const(1)))
    assert rows == [(1,)]


def test_readme_select():
    # README.md:120-127 (c1, c2 spelled out: alias push-down is the optimizer's)
    c1 = R.E_bin("+", R.E_field("number"), R.E_const(1))
    c2 = R.E_bin("/", R.E_field("number"), R.E_const(2))
    where = R.E_bin("<", R.E_bin("+", R.E_bin("+", c1, c2), R.E_const(1)), R.E_const(100))
    rows = R.projection_query(10000000, [R.E_alias("c1", c1), R.E_alias("c2", c2)], where=where, limit=3)
    assert rows[:3] == [(1, 0), (2, 0), (3, 1)]


def test_modulo_is_an_extension():
    e = R.E_bin("%", R.E_field("number"), R.E_const(8))
    with pytest.raises(R.RefError, match="Unsupported Function: %"):
        R.aggregate_query(100, [R.E_fn("max", e)], modulo=False)


# ---- closed forms + the two oracles agree -----------------------------------

def test_c_oracle_closed_forms_and_quirks():
    # BASELINE.md section 3 / SURVEY finding 8
    assert oracle_c.numbers_query(10**8, [(abi.AGG_SUM, None)])[0][2] == 4999999950000000
    assert sum(p[2] for p in oracle_c.partitions(100001)) == 20009
    assert sum(p[2] for p in oracle_c.partitions(1000000)) == 920008
    assert oracle_c.partitions(7) == [(0, 6, 7)]


@pytest.mark.parametrize("n", [1, 5, 8, 16, 9999, 10000, 10001, 80000, 100001, 254321])
def test_c_oracle_matches_numpy_oracle(n):
    # C3 + a C4-shaped query on both oracles
    num = R.E_field("number")
    exprs = [R.E_bin("/", R.E_fn("sum", num), R.E_fn("count", num)), R.E_fn("max", num), R.E_fn("min", num)]
    ref = [v.value for v in R.aggregate_query(n, exprs)]
    s, c, mx, mn = (v for _, _, v in oracle_c.numbers_query(
        n, [(abi.AGG_SUM, None), (abi.AGG_COUNT, None), (abi.AGG_MAX, None), (abi.AGG_MIN, None)]))
    assert ref == [s // c, mx, mn]
    where = R.E_bin("<", R.E_bin("%", num, R.E_const(8)), R.E_const(3))
    arg = R.E_bin("+", num, R.E_const(1))
    ref4 = [v.value for v in R.aggregate_query(n, [R.E_fn("max", arg), R.E_fn("count", arg)], where=where)]
    value, _ = chain(abi.DT_UINT64, [("+", 1)])
    pred = predicate(abi.DT_UINT64, [("%", 8)], "<", 3)
    c4 = [v for _, _, v in oracle_c.numbers_query(n, [(abi.AGG_MAX, value), (abi.AGG_COUNT, value)], pred)]
    assert ref4 == c4


def test_both_oracles_agree_on_empty_block_error():
    num = R.E_field("number")
    where = R.E_bin("<", num, R.E_const(5))
    with pytest.raises(R.RefError) as e1:
        R.aggregate_query(100000, [R.E_fn("sum", num)], where=where)
    pred = predicate(abi.DT_UINT64, [], "<", 5)
    with pytest.raises(oracle_c.OracleError) as e2:
        oracle_c.numbers_query(100000, [(abi.AGG_SUM, None)], pred)
    assert str(e1.value) == str(e2.value) == "Internal Error: DataValue to array cannot be NONE NULL"


def test_splitmix_column_oracle():
    L = oracle_c.lib()
    col = np.array([L.fqo_splitmix64(7, i) for i in range(30000)], dtype=np.uint64)
    st = oracle_c.column_partial(col, abi.DT_UINT64, 10000, [(abi.AGG_SUM, None), (abi.AGG_MAX, None)])
    assert st[0].bits == int(col.sum(dtype=np.uint64)) and st[1].bits == int(col.max())


@pytest.mark.parametrize("total", [100001, 1_000_000, 2_400_000])
def test_c_group_by_matches_numpy_oracle(total):
    # the C GROUP BY (bench.py's GROUP BY CPU baseline) against fq_ref's
    # statement of the GROUP BY semantics, on numbers_mt sizes that drop rows
    # (100001: the NumbersStream quirk) and with a filter
    U = abi.DT_UINT64
    key = chain(U, [("%", 37)])[0]
    pred = predicate(U, [("%", 8)], "<", 3)
    v1 = chain(U, [("+", 1)])[0]
    aggs = [(abi.AGG_COUNT, U, None), (abi.AGG_SUM, U, None), (abi.AGG_MAX, U, v1), (abi.AGG_MIN, U, None)]
    keys, st = oracle_c.numbers_group(total, key, aggs, pred=pred, threads=8, cap_groups=64)
    o = np.argsort(keys)
    got = [(int(k),) + tuple(int(x) for x in s) for k, s in zip(keys[o], st[o])]
    N = R.E_field("number")
    c = R.E_const
    exp = R.group_by_query(total, R.E_bin("%", N, c(37)),
                           [R.E_fn("count", N), R.E_fn("sum", N), R.E_fn("max", R.E_bin("+", N, c(1))),
                            R.E_fn("min", N)],
                           where=R.E_bin("<", R.E_bin("%", N, c(8)), c(3)))
    assert got == [tuple(r) for r in exp]


def test_c_group_by_closed_form_and_errors():
    U = abi.DT_UINT64
    n, m = 8_000_000, 1000
    keys, st = oracle_c.numbers_group(n, chain(U, [("%", m)])[0],
                                      [(abi.AGG_COUNT, U, None), (abi.AGG_SUM, U, None), (abi.AGG_MAX, U, None)],
                                      threads=8, cap_groups=2 * m)
    per = n // m
    o = np.argsort(keys)
    assert [(int(k), int(a), int(b), int(x)) for k, (a, b, x) in zip(keys[o], st[o])] == \
        [(k, per, (k * per + m * per * (per - 1) // 2) % 2**64, k + m * (per - 1)) for k in range(m)]
    with pytest.raises(oracle_c.OracleError):  # more groups than the caller's buffer
        oracle_c.numbers_group(100_000, None, [(abi.AGG_COUNT, U, None)], threads=8, cap_groups=1000)
    with pytest.raises(oracle_c.OracleError) as ei:  # 7 / (number % 2): divide by zero
        oracle_c.numbers_group(10_000, chain(U, [("%", 2), ("/", 7, True)])[0], [(abi.AGG_COUNT, U, None)])
    assert "Divide by zero" in str(ei.value)


def test_c_filter_projection_closed_form():
    # the C Filter -> Projection restatement (bench.py --query p1's CPU
    # baseline): kept rows and wrapping sums of number+1, number/2 over the
    # rows with number%8 < 3, against numpy over fq_ref's NumbersStream blocks
    # on a quirky size (100001 drops rows)
    U = abi.DT_UINT64
    pred = predicate(U, [("%", 8)], "<", 3)
    outs = [chain(U, [("+", 1)])[0], chain(U, [("/", 2)])[0]]
    for total in (100001, 800_000):
        kept, sums = oracle_c.numbers_project(total, outs, pred=pred, threads=8)
        x = np.concatenate([np.asarray(b.cols["number"].values, dtype=np.uint64) for b in R.numbers_stream(total)])
        x = x[(x % np.uint64(8)) < 3]
        assert kept == len(x)
        assert sums == [int((x + np.uint64(1)).sum(dtype=np.uint64)), int((x // np.uint64(2)).sum(dtype=np.uint64))]
