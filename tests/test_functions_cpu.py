"""CPU: the reference's scalar-state tables and Function protocol run on the
PRODUCT library's host code through the C ABI (fq_data_value_*_op,
fq_function_*), not on the oracle:

  data_value_aggregate_test.rs / data_value_arithmetic_test.rs   ScalarTest tables
                          (tests/golden/reference_vectors.json), values and error texts
  function_aggregator_test.rs:171-189   the merge half of the partial/merge protocol,
                          fed the partial states the test's accumulates produce
  function_factory.rs:14-40             factory names and its error text
Device calls (eval/accumulate) on a host-only engine must fail: no CPU path.
The accumulate half runs on the GPU (tests/test_functions_gpu.py)."""
import json
import os

import pytest

from fq_amd import abi
from fq_amd.engine import Engine
from fq_amd.functions import (AggregatorFunction, ArithmeticFunction, ConstantFunction, DataBlock, DataValue,
                              FieldFunction, FQError, ScalarFunctionFactory, data_value_aggregate_op,
                              data_value_arithmetic_op)

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.json")))
V = DataValue


def lit(d):
    return V(d["type"], d.get("value") if d["kind"] == "some" else None)


def ids(tables):
    return ["%s:%s" % (t["fn"], t["name"]) for t in tables]


VALUE_TABLES = GOLDEN["value_aggregate"] + GOLDEN["value_arithmetic"]


@pytest.mark.parametrize("t", VALUE_TABLES, ids=ids(VALUE_TABLES))
def test_golden_value_ops_on_product(t):
    # the reference harness: Ok -> expect[i], Err -> error[i]
    # (data_value_aggregate_test.rs:146-160, data_value_arithmetic_test.rs:50-66)
    errors = 0
    for i, (l, r) in enumerate(t["args"]):
        try:
            if t["op"] in abi.OP_BY_SYM:
                got = data_value_arithmetic_op(t["op"], lit(l), lit(r))
            else:
                got = data_value_aggregate_op(t["op"], lit(l), lit(r))
            assert got == lit(t["expect"][i]), (i, got, t["expect"][i])
        except FQError as e:
            assert str(e) == t["error"][i], (i, str(e))
            errors += 1
    assert errors == len(t["error"])  # every error row of the table was reached


def test_value_ops_untyped_null_and_none():
    # data_value_arithmetic.rs:10-27: Null is the identity of the merge adds
    assert data_value_arithmetic_op("+", V.NULL, V("UInt64", 4)) == V("UInt64", 4)
    assert data_value_arithmetic_op("+", V("UInt64", 4), V.NULL) == V("UInt64", 4)
    assert data_value_aggregate_op("max", V.NULL, V("Int64", -3)) == V("Int64", -3)
    assert data_value_arithmetic_op("/", V("Int64", 98), V("UInt64", 7)) == V("Int64", 14)


def block_schema():
    # a schema-only block (return_type / nullable read names and types)
    from fq_amd.ops import DeviceColumn
    return DataBlock(["a", "b"], [DeviceColumn(None, 0, abi.DT_INT64), DeviceColumn(None, 0, abi.DT_INT64)])


# function_aggregator_test.rs: (name, evals, builder, display, expect)
def sum_a():
    return AggregatorFunction.try_create("sum", [FieldFunction.try_create("a")])


AGG_CASES = [
    ("count-passed", 1, lambda: AggregatorFunction.try_create("count", [FieldFunction.try_create("a")]),
     "Count(a)", V("UInt64", 4)),
    ("max-passed", 2, lambda: AggregatorFunction.try_create("max", [FieldFunction.try_create("a")]),
     "Max(a)", V("Int64", 4)),
    ("min-passed", 2, lambda: AggregatorFunction.try_create("min", [FieldFunction.try_create("a")]),
     "Min(a)", V("Int64", 1)),
    ("sum-passed", 1, sum_a, "Sum(a)", V("Int64", 10)),
    ("sum(a)+1-merge-passed", 4,
     lambda: ArithmeticFunction.try_create("+", [sum_a(), ConstantFunction.try_create(V("Int64", 1))]),
     "Sum(a) + 1", V("Int64", 71)),
    ("sum(a)/count(a)-merge-passed", 4,
     lambda: ArithmeticFunction.try_create(
         "/", [sum_a(), AggregatorFunction.try_create("count", [FieldFunction.try_create("a")])]),
     "Sum(a) / Count(a)", V("Int64", 2)),
    ("(sum(a+1)+2)-merge-passed", 4,
     lambda: ArithmeticFunction.try_create("+", [
         AggregatorFunction.try_create("sum", [ArithmeticFunction.try_create(
             "+", [FieldFunction.try_create("a"), ConstantFunction.try_create(V("Int8", 1))])]),
         ConstantFunction.try_create(V("Int8", 2))]),
     "Sum(a + 1) + 2", V("Int64", 100)),
]


def host_partial(name, evals):
    """The partial state vector func.accumulate x evals leaves over the block
    a=[4,3,2,1] (function_aggregator.rs:57-100; Null when never accumulated)."""
    if evals == 0:
        return {"sum(a)/count(a)-merge-passed": [V.NULL, V.NULL], "sum(a)+1-merge-passed": [V.NULL, V("Int64", 1)],
                "(sum(a+1)+2)-merge-passed": [V.NULL, V("Int8", 2)]}.get(name, [V.NULL])
    return {"count-passed": [V("UInt64", 4 * evals)], "max-passed": [V("Int64", 4)], "min-passed": [V("Int64", 1)],
            "sum-passed": [V("Int64", 10 * evals)],
            "sum(a)+1-merge-passed": [V("Int64", 10 * evals), V("Int64", 1)],
            "sum(a)/count(a)-merge-passed": [V("Int64", 10 * evals), V("UInt64", 4 * evals)],
            "(sum(a+1)+2)-merge-passed": [V("Int64", 14 * evals), V("Int8", 2)]}[name]


@pytest.mark.parametrize("name,evals,build,display,expect", AGG_CASES, ids=[c[0] for c in AGG_CASES])
def test_function_aggregator_merge_half_on_product(name, evals, build, display, expect):
    f = build()
    assert str(f) == display
    assert f.accumulate_result() == host_partial(name, 0)
    final = f.clone()
    final.set_depth(0)
    final.merge_state(host_partial(name, evals))
    final.merge_state(host_partial(name, evals - 1))
    assert final.merge_result() == expect


def test_function_return_types_and_nullable():
    b = block_schema()
    assert sum_a().return_type(b) == "Int64"
    assert AggregatorFunction.try_create("count", [FieldFunction.try_create("a")]).return_type(b) == "UInt64"
    f = ArithmeticFunction.try_create("+", [FieldFunction.try_create("a"), ConstantFunction.try_create(V("Int8", 1))])
    assert f.return_type(b) == "Int64" and f.nullable(b) is False
    assert ScalarFunctionFactory.get("<", [FieldFunction.try_create("a"), FieldFunction.try_create("b")]
                                     ).return_type(b) == "Boolean"
    with pytest.raises(FQError):  # arrow's field-not-found text
        FieldFunction.try_create("zz").return_type(b)


def test_factory_errors_and_field_protocol():
    with pytest.raises(FQError, match="^Internal Error: Unsupported Function: avg$"):
        ScalarFunctionFactory.get("avg", [FieldFunction.try_create("a")])
    assert str(ScalarFunctionFactory.get("SUM", [FieldFunction.try_create("a")])) == "Sum(a)"
    # function_field.rs:55-68: a bare field has no aggregate state
    with pytest.raises(FQError, match="^Internal Error: Unsupported aggregate operation for function field$"):
        FieldFunction.try_create("a").accumulate_result()
    with pytest.raises(FQError, match="Unsupported aggregate operation for function ="):
        ScalarFunctionFactory.get("=", [FieldFunction.try_create("a"), FieldFunction.try_create("b")]).merge_result()
    # AggregatorFunction::merge_state reads states[depth] (function_aggregator.rs:108-127)
    f = sum_a()
    f.set_depth(3)
    with pytest.raises(FQError, match="index out of bounds: the len is 1 but the index is 3"):
        f.merge_state([V("Int64", 1)])


def test_device_calls_need_a_gpu():
    # a host-only engine runs the state protocol but never a column: no CPU path
    e = Engine(device=-1)
    b = block_schema()
    with pytest.raises(FQError) as ei:
        sum_a().accumulate(e, b)
    assert ei.value.status == abi.FQ_E_HIP


@pytest.mark.parametrize("text", ["a\x00bc", "\x00", "", "plain", "x" * 300 + "\x00" + "y"])
def test_utf8_scalar_with_nul_bytes_round_trips(text):
    # fq_scalar carries (str, str_len): a Utf8 DataValue may hold NUL bytes and
    # must come back whole through the ABI (ConstantFunction state protocol)
    c = ConstantFunction.try_create(V("Utf8", text))
    assert c.merge_result() == V("Utf8", text)
    assert c.accumulate_result() == [V("Utf8", text)]
    c2 = c.clone()
    c2.merge_state([V("Utf8", text + "\x00tail")])  # a constant keeps its own value (function_constant.rs)
    assert c2.merge_result() == V("Utf8", text)
