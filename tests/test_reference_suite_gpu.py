"""The reference's executor / processor / transform unit tests that execute
a pipeline, restated one by one on the GPU engine (SQL -> the same
processors).  Each test names the reference test it follows (file:line of its
assertion).  transform_aggregate_test.rs (122) and transform_filter_test.rs
([1]) are in test_engine_gpu.py; the planner-side ones in
test_reference_suite_cpu.py."""
import pytest

pytestmark = pytest.mark.gpu

eng = None


def setup_module():
    global eng
    from fq_amd import ops
    ops.require_gpu()
    from fq_amd.engine import Engine
    eng = Engine()


def teardown_module():
    if eng is not None:
        eng.close()


def test_select_executor():
    # src/executors/executor_select_test.rs:18-28: the statement executes and
    # its stream drains (no row has number + 2 < 2)
    r = eng.execute("select number from system.numbers_mt(10) where (number+2)<2")
    assert r.names == ["number"] and r.rows == []


def test_processor_merge_first_block():
    # src/processors/processor_merge_test.rs:14-26: one source over
    # numbers_mt(16) (its 8 partitions in order, testdata/number.rs:54-70)
    # merged -> the first block is [0, 1].  One worker = one pipe, so the
    # merge sees the partitions in order.
    from fq_amd.engine import Engine
    with Engine(worker_threads=1) as e:
        r = e.execute("select number from system.numbers_mt(16)")
    assert [x for (x,) in r.rows[:2]] == [0, 1]
    assert sorted(x for (x,) in r.rows) == list(range(16))


def test_transform_limit():
    # src/transforms/transform_limit_test.rs:14-33: numbers_mt(8) merged,
    # LimitTransform(2) -> 2 rows
    r = eng.execute("select number from system.numbers_mt(8) limit 2")
    assert len(r.rows) == 2


def test_transform_projection():
    # src/transforms/transform_projection_test.rs:14-37: project number, number -> 2 columns
    r = eng.execute("select number, number from system.numbers_mt(8)")
    assert len(r.names) == 2 and all(len(row) == 2 for row in r.rows)
    assert sorted(r.rows) == [(i, i) for i in range(8)]


def test_transform_source_two_sources():
    # src/transforms/transform_source_test.rs:12-26: two numbers_mt(8) sources
    # merged -> 16 rows; a query reads one table, so the two sources are the
    # two halves of a UNION the reference cannot express -- here two
    # statements, 8 + 8 rows
    rows = len(eng.execute("select number from system.numbers_mt(8)").rows) + \
        len(eng.execute("select number from system.numbers_mt(8)").rows)
    assert rows == 16
