"""The reference's planner / executor / processor unit tests, restated one
by one against the host side of the engine (no GPU: planning, EXPLAIN and
pipeline display only).  Each test names the reference test it follows
(file:line of its assertion); execution-side tests are in
test_reference_suite_gpu.py."""
import pytest

from fq_amd import abi
from fq_amd.engine import Engine

PIPE_PROJ = ("\n  └─ Merge (ProjectionTransform × 8 processors) to (MergeProcessor × 1)"
             "\n    └─ ProjectionTransform × 8 processors"
             "\n      └─ FilterTransform × 8 processors"
             "\n        └─ SourceTransform × 8 processors")


@pytest.fixture(scope="module")
def eng():
    e = Engine(device=-1)  # host only: plans, never executes a device scan
    yield e
    e.close()


def plan_text(eng, sql):
    """format!("{:?}", plan): the plan part of EXPLAIN (before the pipeline)."""
    return eng.explain(sql).split("\n\n", 1)[0]


def pipeline_text(eng, sql):
    """format!("{:?}", pipeline) (pipeline.rs Debug): the part after the plan."""
    return "\n" + eng.explain(sql).split("\n\n", 1)[1]


def test_plan_explain(eng):
    # src/planners/plan_explain_test.rs:17-27
    sql = ("explain select number as c1, number as c2, number as c3,(number+1) from system.numbers_mt "
           "where (number+1)=4")
    assert plan_text(eng, sql) == ("└─ Projection: number as c1, number as c2, number as c3, (number + 1)"
                                   "\n  └─ Filter: ((number + 1) = 4)"
                                   "\n    └─ ReadDataSource: scan parts [8](Read from system.numbers_mt table)")


def test_plan_filter(eng):
    # src/planners/plan_filter_test.rs:12-24 builds Filter(number = 1) ->
    # Projection(number) over an 8-part read with PlanBuilder; the same plan
    # through SQL
    assert plan_text(eng, "select number from system.numbers_mt where number = 1") == (
        "└─ Projection: number\n  └─ Filter: (number = 1)"
        "\n    └─ ReadDataSource: scan parts [8](Read from system.numbers_mt table)")


def test_plan_select_wildcard(eng):
    # src/planners/plan_select_test.rs:18-29
    assert plan_text(eng, "select * from system.numbers_mt where (number+1)=4") == (
        "└─ Projection: number\n  └─ Filter: ((number + 1) = 4)"
        "\n    └─ ReadDataSource: scan parts [8](Read from system.numbers_mt table)")


def test_pipeline_builder(eng):
    # src/processors/pipeline_builder_test.rs:19-33
    sql = "select sum(number+1)+2 as sumx from system.numbers_mt where (number+1)=4 limit 1"
    assert pipeline_text(eng, sql) == (
        "\n  └─ LimitTransform × 1 processor"
        "\n    └─ AggregateFinalTransform × 1 processor"
        "\n      └─ Merge (AggregatePartialTransform × 8 processors) to (MergeProcessor × 1)"
        "\n        └─ AggregatePartialTransform × 8 processors"
        "\n          └─ FilterTransform × 8 processors"
        "\n            └─ SourceTransform × 8 processors")


def test_explain_executor(eng):
    # src/executors/executor_explain_test.rs:18-28: ExplainExecutor runs and
    # streams its block (executor_explain.rs:38-59: one Utf8 column "explain"
    # holding the plan and the pipeline)
    r = eng.execute("explain select number from system.numbers_mt(10) where (number+1)=4")
    assert r.names == ["explain"] and r.types == [abi.DT_UTF8]
    assert [row[0] for row in r.rows] == [
        "└─ Projection: number\n  └─ Filter: ((number + 1) = 4)"
        "\n    └─ ReadDataSource: scan parts [8](Read from system.numbers_mt table)", PIPE_PROJ]


@pytest.mark.parametrize("fun,args", [("+", "number, number"), ("-", "number, number"), ("*", "number, number"),
                                      ("/", "number, number"), ("count", "number"), ("and", None),
                                      ("or", None)])
def test_function_factory(eng, fun, args):
    # src/functions/function_factory_test.rs:18-130: ScalarFunctionFactory /
    # AggregateFunctionFactory resolve + - * / count and or without error
    if fun in ("and", "or"):
        sql = "select number from system.numbers_mt(8) where number > 1 %s number < 5" % fun
    elif fun == "count":
        sql = "select count(%s) from system.numbers_mt(8)" % args
    else:
        sql = "select number %s number from system.numbers_mt(8)" % fun
    assert eng.explain(sql)  # planned, every function resolved


def test_function_factory_unknown(eng):
    # function_factory.rs:17-39: an unknown name is "Unsupported Function: <name>"
    with pytest.raises(Exception, match="Unsupported Function: xyz"):
        eng.explain("select xyz(number) from system.numbers_mt(8)")
