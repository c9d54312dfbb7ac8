"""fq_filter_project / fq_predicate_bitmap (FilterTransform -> Projection
fused over one column, hipRTC-specialised) against numpy on seeded inputs,
bit-exact: tile edges (16,384-row tiles, 64-row words), ragged lengths,
empty/full selections, unaligned columns, the map path (no predicate), the
reference's error order (predicate errors on any row first, then expression
errors on kept rows only), and agreement with the unfused fq_compare ->
fq_filter_compact -> fq_arith chain."""
import numpy as np
import pytest

from fq_amd import abi
from fq_amd.expr import COL, chain, predicate, pred_tree

pytestmark = pytest.mark.gpu

ops = None
U64, I64, F64 = abi.DT_UINT64, abi.DT_INT64, abi.DT_FLOAT64


def setup_module():
    global ops
    from fq_amd import ops as _ops
    _ops.require_gpu()
    _ops.jit_config(abi.JIT_AUTO, 1 << 22)
    ops = _ops


def test_two_lookback_launches_side_by_side():
    """The configuration that stalled once in round 5 ("the offset look-back did
    not complete"): look-back launches running together on separate queues, each
    with more workgroups than stay resident beside the other.  Two host threads,
    each on its own HIP stream, run fq_filter_project over its own 4e7-row
    column four times (4,883 tiles, a grid of up to 2,048 workgroups per launch)
    -- every launch completes with numpy's rows.  The single ticket counter
    draws tiles in order, so the lowest unfinished tile's predecessors are all
    held by resident workgroups whatever else shares the GPU (fq_jit.hip)."""
    import threading

    import torch
    n = 40_000_000
    cases = []
    for seed, (mod, lt) in ((0x11, (8, 3)), (0x22, (1000, 500))):
        col = ops.splitmix_column(seed, 0, n)
        host = col.to_numpy()
        keep = host % np.uint64(mod) < np.uint64(lt)
        cases.append((col, predicate(U64, [("%", mod)], "<", lt), host[keep]))
    torch.cuda.synchronize()
    start = threading.Barrier(2)
    errors = []

    def run(col, pred, kept):
        try:
            stream = torch.cuda.Stream()
            with torch.cuda.stream(stream):
                start.wait()
                for _ in range(4):
                    outs = ops.filter_project(col, pred, [chain(U64, [("+", 1)])[0]], stream=stream)
                    got = outs[0].to_numpy()
                    if outs[0].len != len(kept) or not np.array_equal(got, kept + np.uint64(1)):
                        errors.append("rows differ")
        except Exception as e:  # the poll bound reports "did not complete"
            errors.append(repr(e))

    threads = [threading.Thread(target=run, args=c) for c in cases]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in threads), "a look-back launch did not finish"
    assert errors == []


def _u(x):
    return np.asarray(x, dtype=np.uint64)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 16383, 16384, 16385, 16384 * 17 + 5, 1_000_003])
def test_filter_project_numbers_ragged(n):
    host = np.arange(n, dtype=np.uint64) + np.uint64(7)
    col = ops.from_numpy(host)
    pred = predicate(U64, [("%", 8)], "<", 3)
    outs = ops.filter_project(col, pred, [None, chain(U64, [("+", 1)])[0], chain(U64, [("/", 2)])[0]])
    keep = host % np.uint64(8) < np.uint64(3)
    k = host[keep]
    assert [o.len for o in outs] == [len(k)] * 3
    assert np.array_equal(outs[0].to_numpy(), k)
    assert np.array_equal(outs[1].to_numpy(), k + np.uint64(1))
    assert np.array_equal(outs[2].to_numpy(), k // np.uint64(2))


@pytest.mark.parametrize("sel", ["none", "all", "sparse", "dense"])
def test_filter_project_random_selectivity(sel):
    rng = np.random.default_rng(0x5EED)
    n = 300_001
    host = rng.integers(0, 2**63, size=n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n).astype(np.uint64)
    col = ops.from_numpy(host)
    if sel == "none":
        pred, keep = predicate(U64, [], "<", 0), np.zeros(n, bool)
    elif sel == "all":
        pred, keep = predicate(U64, [], ">=", 0), np.ones(n, bool)
    elif sel == "sparse":
        pred, keep = predicate(U64, [("%", 1000)], "=", 999), host % np.uint64(1000) == np.uint64(999)
    else:
        pred, keep = predicate(U64, [("%", 10)], "<", 9), host % np.uint64(10) < np.uint64(9)
    outs = ops.filter_project(col, pred, [chain(U64, [("*", 3), ("-", 5)])[0]])
    k = host[keep]
    assert outs[0].len == len(k)
    assert np.array_equal(outs[0].to_numpy(), k * np.uint64(3) - np.uint64(5))  # u64 wrap


def test_filter_project_tree_predicate_and_float_outputs():
    n = 200_000
    host = np.arange(n, dtype=np.uint64)
    col = ops.from_numpy(host)
    t = pred_tree(U64, [([("%", 8)], "<", 3), ([], ">", 1000), ([("%", 97)], "=", 0)], [0, 1, "and", 2, "or"])
    outs = ops.filter_project(col, t, [chain(U64, [("/", 2.0)])[0], chain(U64, [("-", (5000, "Int64"))])[0]])
    keep = ((host % 8 < 3) & (host > 1000)) | (host % 97 == 0)
    k = host[keep]
    assert outs[0].dtype == F64 and outs[1].dtype == I64
    assert np.array_equal(outs[0].to_numpy(), k.astype(np.float64) / 2.0)
    assert np.array_equal(outs[1].to_numpy(), k.astype(np.int64) - 5000)


def test_filter_project_f64_column():
    rng = np.random.default_rng(7)
    host = rng.standard_normal(100_003)
    col = ops.from_numpy(host)
    pred = predicate(F64, [("*", 2.0)], ">=", 1.5)
    outs = ops.filter_project(col, pred, [None, chain(F64, [("+", COL)])[0]])
    k = host[host * 2.0 >= 1.5]
    assert np.array_equal(outs[0].to_numpy(), k)
    assert np.array_equal(outs[1].to_numpy(), k + k)


@pytest.mark.parametrize("offset", [0, 1])
@pytest.mark.parametrize("n", [1, 2, 3, 1025, 1_000_001])
def test_map_path_no_predicate(n, offset):
    # unaligned column (offset 8 bytes): 8-byte rows instead of 16-byte pairs
    host = np.arange(n + offset, dtype=np.uint64) * np.uint64(3)
    full = ops.from_numpy(host)
    col = ops.DeviceColumn(full.buf, n, U64, offset=8 * offset)
    outs = ops.filter_project(col, None, [chain(U64, [("+", 1)])[0], None, chain(U64, [("%", 7)])[0]])
    h = host[offset:]
    assert [o.len for o in outs] == [n] * 3
    assert np.array_equal(outs[0].to_numpy(), h + np.uint64(1))
    assert np.array_equal(outs[1].to_numpy(), h)
    assert np.array_equal(outs[2].to_numpy(), h % np.uint64(7))


def test_eight_outputs():
    host = np.arange(70_000, dtype=np.uint64)
    col = ops.from_numpy(host)
    pred = predicate(U64, [("%", 3)], "=", 1)
    outs = ops.filter_project(col, pred, [chain(U64, [("+", k)])[0] for k in range(8)])
    k = host[host % 3 == 1]
    for j, o in enumerate(outs):
        assert np.array_equal(o.to_numpy(), k + np.uint64(j))


def test_error_order_predicate_first_then_kept_rows_only():
    host = np.arange(100_000, dtype=np.uint64)
    col = ops.from_numpy(host)
    # predicate divides by zero on row 0: an error whatever the projection
    with pytest.raises(ops.FQError) as ei:
        ops.filter_project(col, predicate(U64, [("/", COL)], ">", 0), [None])
    assert ei.value.status == abi.FQ_E_DIVIDE_BY_ZERO
    assert str(ei.value) == "Internal Error: Divide by zero error"
    # 100 / (number % 8): rows with number % 8 == 0 are kept -> error
    val = chain(U64, [("%", 8), ("/", 100, True)])[0]
    with pytest.raises(ops.FQError) as ei:
        ops.filter_project(col, predicate(U64, [("%", 8)], "<", 3), [val])
    assert ei.value.status == abi.FQ_E_DIVIDE_BY_ZERO
    # ... and filtered out -> no error (the projection sees kept rows only)
    outs = ops.filter_project(col, predicate(U64, [("%", 8)], ">=", 1), [val])
    k = host[host % 8 >= 1]
    assert np.array_equal(outs[0].to_numpy(), np.uint64(100) // (k % np.uint64(8)))


def test_bitmap_predicate_input_and_predicate_bitmap():
    n = 123_457
    host = np.arange(n, dtype=np.uint64) * np.uint64(5)
    col = ops.from_numpy(host)
    pred = predicate(U64, [("%", 7)], "<", 2)
    bm = ops.predicate_bitmap(col, pred)
    keep = host % np.uint64(7) < np.uint64(2)
    assert np.array_equal(bm.to_numpy(), keep)
    # the same bitmap as fq_compare over the materialised lhs
    lhs = ops.arith("%", col, 7)
    assert np.array_equal(ops.compare("<", lhs, 2).to_numpy(), keep)
    p = abi.fq_pred()
    p.kind = abi.PRED_BITMAP
    p.bitmap = bm.ptr
    outs = ops.filter_project(col, p, [chain(U64, [("+", 1)])[0]])
    assert np.array_equal(outs[0].to_numpy(), host[keep] + np.uint64(1))
    # unfused chain: compare -> compact -> arith gives the same rows
    unf = ops.arith("+", ops.filter_compact(col, bm), 1)
    assert np.array_equal(unf.to_numpy(), outs[0].to_numpy())


def test_empty_column():
    col = ops.from_numpy(np.zeros(0, np.uint64))
    outs = ops.filter_project(col, predicate(U64, [], ">", 1), [None])
    assert outs[0].len == 0
