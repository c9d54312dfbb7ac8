"""GPU: the reference's Function tests replayed on the PRODUCT's C++ Function
objects through the C ABI (fq_function_*), blocks as device columns:

  function_aggregator_test.rs:5-189    count/max/min/sum and the three merge
        cases: func1 accumulates the block `evals` times, func2 `evals - 1`
        times, a third function merge_states both -> 4/4/1/10/71/2/100
  function_arithmetic_test.rs / function_comparison_test.rs
        (tests/golden/reference_vectors.json): display + eval bit for bit
plus seeded multi-block accumulates against numpy sums (exact integers)."""
import json
import os

import numpy as np
import pytest

from fq_amd import abi

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.json")))
NP = {"Int8": np.int8, "Int16": np.int16, "Int32": np.int32, "Int64": np.int64, "UInt8": np.uint8,
      "UInt16": np.uint16, "UInt32": np.uint32, "UInt64": np.uint64, "Float32": np.float32,
      "Float64": np.float64}
ops = F = None
ENGINE = None


def setup_module():
    global ops, F, ENGINE
    from fq_amd import functions as _F
    from fq_amd import ops as _ops
    _ops.require_gpu()
    ops, F = _ops, _F
    ENGINE = _F.Engine(device=0)


def teardown_module():
    if ENGINE is not None:
        ENGINE.close()


def block_ab():
    a = ops.from_numpy(np.array([4, 3, 2, 1], dtype=np.int64), abi.DT_INT64)
    b = ops.from_numpy(np.array([1, 2, 3, 4], dtype=np.int64), abi.DT_INT64)
    return F.DataBlock(["a", "b"], [a, b])


def agg_cases():
    from tests.test_functions_cpu import AGG_CASES
    return AGG_CASES


@pytest.mark.parametrize("case", range(7))
def test_function_aggregator_protocol_on_product(case):
    name, evals, build, display, expect = agg_cases()[case]
    blk = block_ab()
    func = build()
    assert str(func) == display
    func1 = func.clone()
    for _ in range(evals):
        func1.accumulate(ENGINE, blk)
    state1 = func1.accumulate_result()
    func2 = func.clone()
    for _ in range(1, evals):
        func2.accumulate(ENGINE, blk)
    state2 = func2.accumulate_result()
    final = func.clone()
    final.set_depth(0)
    final.merge_state(state1)
    final.merge_state(state2)
    assert final.merge_result() == expect, (name, state1, state2)


FUNCTION_TABLES = GOLDEN["function_arithmetic"] + GOLDEN["function_comparison"]


@pytest.mark.parametrize("t", FUNCTION_TABLES, ids=["%s:%s" % (t["fn"], t["name"]) for t in FUNCTION_TABLES])
def test_golden_function_tables_on_product(t):
    # function_arithmetic_test.rs:28-160 / function_comparison_test.rs:25-85
    cols = [ops.from_numpy(np.array(c["values"], dtype=NP[c["type"]]), abi.DT_BY_NAME[c["type"]])
            for c in t["columns"]]
    blk = F.DataBlock(list("abc")[:len(cols)], cols)
    lhs, op, rhs = t["display"].split(" ")
    f = F.ScalarFunctionFactory.get(op, [F.FieldFunction.try_create(lhs), F.FieldFunction.try_create(rhs)])
    assert str(f) == t["display"]
    assert f.nullable(blk) is t["nullable"]
    got = f.eval(ENGINE, blk)
    exp = t["expect"]
    assert abi.DT_NAMES[got.dtype] == exp["type"]
    vals = got.to_numpy()
    if exp["type"] == "Boolean":
        assert [bool(x) for x in vals] == exp["values"]
    else:
        assert np.array_equal(vals, np.array(exp["values"], dtype=NP[exp["type"]]))


def test_constant_eval_is_a_scalar():
    blk = block_ab()
    v = F.ConstantFunction.try_create(F.DataValue("Utf8", "xx")).eval(ENGINE, blk)
    assert v == F.DataValue("Utf8", "xx")


@pytest.mark.parametrize("seed", [0, 1])
def test_multi_block_accumulate_matches_numpy(seed):
    # Sum(a + 1) + 2 and Max(a) / Min(a) over 5 ragged blocks, two partials
    rng = np.random.default_rng(seed)
    blocks = [rng.integers(-2**40, 2**40, size=n, dtype=np.int64) for n in (1, 4097, 65536, 3, 100001)]
    a1 = F.ArithmeticFunction.try_create("+", [F.FieldFunction.try_create("a"),
                                               F.ConstantFunction.try_create(F.DataValue("Int8", 1))])
    f = F.ArithmeticFunction.try_create("+", [F.AggregatorFunction.try_create("sum", [a1]),
                                              F.ConstantFunction.try_create(F.DataValue("Int8", 2))])
    mx = F.AggregatorFunction.try_create("max", [F.FieldFunction.try_create("a")])
    p1, p2, m1, m2 = f.clone(), f.clone(), mx.clone(), mx.clone()
    for i, arr in enumerate(blocks):
        blk = F.DataBlock(["a"], [ops.from_numpy(arr, abi.DT_INT64)])
        (p1 if i % 2 == 0 else p2).accumulate(ENGINE, blk)
        (m1 if i % 2 == 0 else m2).accumulate(ENGINE, blk)
    final, fm = f.clone(), mx.clone()
    final.set_depth(0)
    for s in (p1.accumulate_result(), p2.accumulate_result()):
        final.merge_state(s)
    for s in (m1.accumulate_result(), m2.accumulate_result()):
        fm.merge_state(s)
    allv = np.concatenate(blocks)
    want = int((allv + 1).sum(dtype=np.int64)) + 2
    assert final.merge_result() == F.DataValue("Int64", want)
    assert fm.merge_result() == F.DataValue("Int64", int(allv.max()))


def test_empty_block_sum_state_is_none():
    # arrow sum of an empty array is None; Sum's state after one empty block
    # is Int64(None) (function_aggregator.rs:78-90)
    f = F.AggregatorFunction.try_create("sum", [F.FieldFunction.try_create("a")])
    empty = F.DataBlock(["a"], [ops.from_numpy(np.zeros(0, dtype=np.int64), abi.DT_INT64)])
    f.accumulate(ENGINE, empty)
    assert f.accumulate_result() == [F.DataValue("Int64", None)]


# ---- the Function-handle boundary with the reference's block geometry ----
# A host that keeps the reference's transforms hands AggregatePartial a device
# block that spans a partition's 10,000-row reference blocks (fq_block
# block_rows) and carries FilterTransform's predicate (fq_block filter); the
# per-block state machine of function_aggregator.rs:57-100 is replayed over it.

def _num():
    return F.FieldFunction.try_create("number")


def _agg(name, arg=None):
    return F.AggregatorFunction.try_create(name, [arg or _num()])


def _lt(k):
    return F.ComparisonFunction.try_create("<", [_num(), F.ConstantFunction.try_create(F.DataValue("UInt64", k))])


def _oracle(n, exprs, where):
    import fq_ref as R
    num = R.E_field("number")
    w = R.E_bin("<", num, R.E_const(where)) if where is not None else None
    return R.aggregate_query(n, [R.E_fn(e, num) for e in exprs], where=w, parts=[(0, n - 1)])


def test_handles_filtered_sum_over_empty_reference_block_fails_as_the_reference():
    # numbers 0..99,999 as ONE device block of ten 10,000-row reference blocks;
    # WHERE number < 25000 leaves blocks 3..9 empty: the reference's Sum meets
    # a None block sum after two blocks and fails in to_array; Count/Max/Min
    # skip the empty blocks
    import fq_ref as R
    n = 100_000
    col = ops.numbers_column(0, n)
    blk = F.DataBlock(["number"], [col], block_rows=10000, filter=_lt(25000))
    with pytest.raises(R.RefError) as oracle_err:
        _oracle(n, ["sum"], 25000)
    f = _agg("sum")
    with pytest.raises(F.FQError) as e:
        f.accumulate(ENGINE, blk)
    assert str(e.value) == "Internal Error: DataValue to array cannot be NONE NULL" == str(oracle_err.value)
    # the same error through the fused multi-handle call (one scan, block mode)
    with pytest.raises(F.FQError) as e2:
        F.Function.accumulate_all(ENGINE, [_agg("count"), _agg("sum"), _agg("max")], blk)
    assert str(e2.value) == str(e.value)
    # the functions that do not need per-block sums: the oracle's values
    want = [v.value for v in _oracle(n, ["count", "max", "min"], 25000)]
    fs = [_agg("count"), _agg("max"), _agg("min")]
    F.Function.accumulate_all(ENGINE, fs, blk)
    assert [x.merge_result().value for x in fs] == want == [25000, 24999, 0]
    # as ONE reference block (block_rows 0) the filtered Sum is fine
    one = F.DataBlock(["number"], [col], block_rows=0, filter=_lt(25000))
    f1 = _agg("sum")
    f1.accumulate(ENGINE, one)
    assert f1.merge_result() == F.DataValue("UInt64", 25000 * 24999 // 2)


@pytest.mark.parametrize("k", [7, 25000, 10**6])
def test_functions_accumulate_is_one_scan_and_equals_separate_calls(k):
    # C3's aggregators plus a filter (numbers 0..999,999 in 10,000-row blocks,
    # WHERE number < k): one fq_functions_accumulate = one fused scan, the same
    # states as four fq_function_accumulate calls, and the oracle's merge
    n = 1_000_000
    col = ops.numbers_column(0, n)
    blk = F.DataBlock(["number"], [col], block_rows=10000, filter=_lt(k))

    def plan():  # sum(number)/count(number), max(number), min(number)
        avg = F.ArithmeticFunction.try_create("/", [_agg("sum"), _agg("count")])
        avg.set_depth(0)
        return [avg, _agg("max"), _agg("min")]

    fused, single = plan(), plan()
    errs = []
    s0 = ENGINE.stats()["scan_launches"]
    try:
        F.Function.accumulate_all(ENGINE, fused, blk)
    except F.FQError as e:
        errs.append(str(e))
    s1 = ENGINE.stats()["scan_launches"]
    assert s1 - s0 == 1
    for f in single:
        try:
            f.accumulate(ENGINE, blk)
        except F.FQError as e:
            errs.append(str(e))
            break
    if k < n - 10000:  # a block is left empty: Sum fails, both ways alike
        assert errs == ["Internal Error: DataValue to array cannot be NONE NULL"] * 2
        return
    assert not errs
    assert [f.accumulate_result() for f in fused] == [f.accumulate_result() for f in single]
    got = [f.merge_result().value for f in fused]
    import fq_ref as R
    num = R.E_field("number")
    want = R.aggregate_query(n, [R.E_bin("/", R.E_fn("sum", num), R.E_fn("count", num)), R.E_fn("max", num),
                                 R.E_fn("min", num)], where=R.E_bin("<", num, R.E_const(k)), parts=[(0, n - 1)])
    assert got == [v.value for v in want]


def test_eval_over_a_filtered_block_is_its_kept_rows():
    x = np.random.default_rng(3).integers(0, 2**40, 50_000, dtype=np.uint64)
    blk = F.DataBlock(["number"], [ops.from_numpy(x, abi.DT_UINT64)], block_rows=10000, filter=_lt(2**39))
    f = F.ArithmeticFunction.try_create("+", [_num(), F.ConstantFunction.try_create(F.DataValue("UInt64", 1))])
    got = f.eval(ENGINE, blk).to_numpy()
    assert np.array_equal(got, x[x < 2**39] + np.uint64(1))


def test_block_rows_is_validated():
    blk = F.DataBlock(["number"], [ops.numbers_column(0, 10)], block_rows=-1)
    with pytest.raises(F.FQError, match="negative block_rows"):
        _agg("sum").accumulate(ENGINE, blk)
