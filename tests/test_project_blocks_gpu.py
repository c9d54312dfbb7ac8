"""fq_filter_project_blocks: FilterTransform -> ProjectionTransform over a
stream of DataBlocks (the reference's per-block loop, transform_filter.rs:38-55
on every numbers block, numbers_stream.rs:29-48, then
transform_projection.rs:45-56), block b's kept rows at output rows
[b * block_rows, + counts[b]).

Checked bit-exact per block: against oracle/fq_ref.py's filter_block +
Function.eval over the reference's own 10,000-row numbers blocks, and against
a numpy restatement of the per-block compaction at block sizes that put block
edges anywhere inside the kernel's 8,192-row tiles (at a tile edge, one row
either side, several tiles per block, one block for the whole column, a short
last block), every selectivity, bitmap / tree predicates, float outputs, eight
outputs, the map path, the error order, and -- at 1.25e8 rows -- per-block
closed forms of the count and of each output's wrapping sum."""
import os
import sys

import numpy as np
import pytest
import torch

from fq_amd import abi
from fq_amd.expr import COL, chain, predicate, pred_tree

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

ops = None
U64, I64, F64 = abi.DT_UINT64, abi.DT_INT64, abi.DT_FLOAT64
TILE = 8192


def setup_module():
    global ops
    from fq_amd import ops as _ops
    _ops.require_gpu()
    _ops.jit_config(abi.JIT_AUTO, 1 << 22)
    ops = _ops


@pytest.fixture(autouse=True, params=[0, 1, 4], ids=["direct", "staged", "staged_quarter"])
def stage(request):
    """Every test three times: kept rows stored straight from registers, staged
    in LDS (a whole tile) then written by consecutive threads, and staged
    through a quarter-tile buffer -- a tile keeping more than a quarter of its
    rows takes several passes (FQ_TUNE_SELECT_BLOCKS_STAGE)."""
    before = ops.tune_get("SELECT_BLOCKS_STAGE")
    ops.tune_set("SELECT_BLOCKS_STAGE", request.param)
    yield request.param
    ops.tune_set("SELECT_BLOCKS_STAGE", before)


def _blocks_of(outs, counts, block_rows):
    """Per output: the list of each block's valid rows (numpy)."""
    res = []
    for o in outs:
        h = o.to_numpy()
        res.append([h[b * block_rows: b * block_rows + int(c)] for b, c in enumerate(counts)])
    return res


def _expect_blocks(host, keep, fns, block_rows):
    exp = []
    for f in fns:
        per = []
        for b0 in range(0, len(host), block_rows):
            blk = host[b0:b0 + block_rows]
            per.append(f(blk[keep[b0:b0 + block_rows]]))
        exp.append(per)
    return exp


def _check(host, keep, pred, values, fns, block_rows, col=None, out_offset=0):
    col = col if col is not None else ops.from_numpy(host)
    outs, counts = ops.filter_project_blocks(col, block_rows, pred, values, out_offset=out_offset)
    nb = -(-len(host) // block_rows)
    assert len(counts) == nb
    want = [int(keep[b0:b0 + block_rows].sum()) for b0 in range(0, len(host), block_rows)]
    assert counts.tolist() == want
    got = _blocks_of(outs, counts, block_rows)
    exp = _expect_blocks(host, keep, fns, block_rows)
    for g, e in zip(got, exp):
        for gb, eb in zip(g, e):
            assert np.array_equal(gb, eb)
    return outs, counts


def test_reference_blocks_against_oracle():
    """numbers_mt rows [begin, begin + 20 blocks): the oracle's filter_block +
    Arith eval on each of the reference's 10,000-row blocks == block b's rows."""
    import fq_ref as R
    begin, nblk = 123_450_000, 20
    where = R.E_bin("<", R.E_bin("%", R.E_field("number"), R.E_const(8)), R.E_const(3))
    exprs = [R.E_bin("+", R.E_field("number"), R.E_const(1)), R.E_bin("/", R.E_field("number"), R.E_const(2))]
    pred_fn = R.to_function(where)
    funcs = [R.to_function(e) for e in exprs]
    col = ops.numbers_column(begin, nblk * 10_000)
    outs, counts = ops.filter_project_blocks(col, 10_000, predicate(U64, [("%", 8)], "<", 3),
                                             [chain(U64, [("+", 1)])[0], chain(U64, [("/", 2)])[0]])
    got = _blocks_of(outs, counts, 10_000)
    blocks = list(R.numbers_blocks(begin, begin + nblk * 10_000 - 1))
    assert len(blocks) == nblk
    for b, (bb, be) in enumerate(blocks):
        blk = R.Block({"number": R.Arr("UInt64", np.arange(bb, be + 1, dtype=np.uint64))})
        kept = R.filter_block(pred_fn, blk)
        assert counts[b] == kept.num_rows()
        for j, f in enumerate(funcs):
            v = f.eval(kept)
            assert v.type == "UInt64"
            assert got[j][b].tolist() == [int(x) for x in v.values]


@pytest.mark.parametrize("block_rows", [TILE, TILE + 1, 10_000, 3 * TILE - 1, 65_536, 1_000_003, 1_000_004])
@pytest.mark.parametrize("n", [1, TILE - 1, TILE, TILE + 1, 10_000 * 17 + 3, 1_000_003])
def test_block_edges_numbers(n, block_rows):
    host = np.arange(n, dtype=np.uint64) + np.uint64(1 << 40)
    keep = host % np.uint64(8) < np.uint64(3)
    _check(host, keep, predicate(U64, [("%", 8)], "<", 3), [None, chain(U64, [("+", 1)])[0]],
           [lambda k: k, lambda k: k + np.uint64(1)], block_rows)


@pytest.mark.parametrize("sel", ["none", "all", "sparse", "dense", "runs"])
def test_block_selectivity(sel):
    rng = np.random.default_rng(0xB10C)
    n = 700_001
    host = rng.integers(0, 2**63, size=n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n).astype(np.uint64)
    if sel == "none":
        pred, keep = predicate(U64, [], "<", 0), np.zeros(n, bool)
    elif sel == "all":
        pred, keep = predicate(U64, [], ">=", 0), np.ones(n, bool)
    elif sel == "sparse":
        pred, keep = predicate(U64, [("%", 1000)], "=", 999), host % np.uint64(1000) == np.uint64(999)
    elif sel == "dense":
        pred, keep = predicate(U64, [("%", 10)], "<", 9), host % np.uint64(10) < np.uint64(9)
    else:  # long kept / dropped runs that straddle tile and block edges
        host = np.arange(n, dtype=np.uint64)
        pred, keep = predicate(U64, [("%", 30_000)], "<", 11_000), host % np.uint64(30_000) < np.uint64(11_000)
    _check(host, keep, pred, [chain(U64, [("*", 3), ("-", 5)])[0]], [lambda k: k * np.uint64(3) - np.uint64(5)],
           10_000)


def test_block_tree_predicate_and_float_outputs():
    n = 250_000
    host = np.arange(n, dtype=np.uint64)
    t = pred_tree(U64, [([("%", 8)], "<", 3), ([], ">", 1000), ([("%", 97)], "=", 0)], [0, 1, "and", 2, "or"])
    keep = ((host % 8 < 3) & (host > 1000)) | (host % 97 == 0)
    outs, _ = _check(host, keep, t, [chain(U64, [("/", 2.0)])[0], chain(U64, [("-", (5000, "Int64"))])[0]],
                     [lambda k: k.astype(np.float64) / 2.0, lambda k: k.astype(np.int64) - 5000], 10_000)
    assert outs[0].dtype == F64 and outs[1].dtype == I64


def test_block_f64_column_and_eight_outputs():
    rng = np.random.default_rng(11)
    host = rng.standard_normal(90_001)
    _check(host, host * 2.0 >= 1.5, predicate(F64, [("*", 2.0)], ">=", 1.5), [None, chain(F64, [("+", COL)])[0]],
           [lambda k: k, lambda k: k + k], 8192)
    h2 = np.arange(70_000, dtype=np.uint64)
    fns = [(lambda j: (lambda k: k + np.uint64(j)))(j) for j in range(8)]
    _check(h2, h2 % 3 == 1, predicate(U64, [("%", 3)], "=", 1), [chain(U64, [("+", j)])[0] for j in range(8)], fns,
           12_345)


def test_block_bitmap_predicate():
    n = 123_457
    host = np.arange(n, dtype=np.uint64) * np.uint64(5)
    col = ops.from_numpy(host)
    bm = ops.predicate_bitmap(col, predicate(U64, [("%", 7)], "<", 2))
    p = abi.fq_pred()
    p.kind = abi.PRED_BITMAP
    p.bitmap = bm.ptr
    keep = host % np.uint64(7) < np.uint64(2)
    _check(host, keep, p, [chain(U64, [("+", 1)])[0]], [lambda k: k + np.uint64(1)], 9_000, col=col)


@pytest.mark.parametrize("n", [1, 10_000, 1_000_001])
def test_block_map_path_no_predicate(n):
    host = np.arange(n, dtype=np.uint64) * np.uint64(3)
    keep = np.ones(n, bool)
    _check(host, keep, None, [chain(U64, [("+", 1)])[0], None], [lambda k: k + np.uint64(1), lambda k: k], 10_000)


def test_block_error_order_and_refusals():
    host = np.arange(100_000, dtype=np.uint64)
    col = ops.from_numpy(host)
    with pytest.raises(ops.FQError) as ei:  # the predicate divides by zero on row 0
        ops.filter_project_blocks(col, 10_000, predicate(U64, [("/", COL)], ">", 0), [None])
    assert ei.value.status == abi.FQ_E_DIVIDE_BY_ZERO
    assert str(ei.value) == "Internal Error: Divide by zero error"
    val = chain(U64, [("%", 8), ("/", 100, True)])[0]  # 100 / (number % 8)
    with pytest.raises(ops.FQError) as ei:  # kept rows with number % 8 == 0
        ops.filter_project_blocks(col, 10_000, predicate(U64, [("%", 8)], "<", 3), [val])
    assert ei.value.status == abi.FQ_E_DIVIDE_BY_ZERO
    keep = host % 8 >= 1  # filtered out: no error, the projection sees kept rows only
    _check(host, keep, predicate(U64, [("%", 8)], ">=", 1), [val], [lambda k: np.uint64(100) // (k % np.uint64(8))],
           10_000, col=col)
    # a block longer than the column: one block (no overflow of len + block_rows)
    outs, counts = ops.filter_project_blocks(col, 2**63 - 1, predicate(U64, [("%", 8)], "<", 3), [None])
    assert counts.tolist() == [int((host % 8 < 3).sum())]
    assert np.array_equal(outs[0].to_numpy()[:counts[0]], host[host % 8 < 3])
    with pytest.raises(ops.FQError) as ei:
        ops.filter_project_blocks(col, TILE - 1, predicate(U64, [], ">", 1), [None])
    assert ei.value.status == abi.FQ_E_INVALID
    outs, counts = ops.filter_project_blocks(ops.from_numpy(np.zeros(0, np.uint64)), 10_000,
                                             predicate(U64, [], ">", 1), [None])
    assert len(counts) == 0


def _block_closed_forms(begin, nb, br):
    """Per block of br rows from `begin`: kept rows with number % 8 < 3, and the
    wrapping sums of number + 1 and number / 2 over them (exact integers)."""
    b = begin + np.arange(nb, dtype=object) * br
    e = b + br - 1
    kept = np.zeros(nb, dtype=object)
    s1 = np.zeros(nb, dtype=object)
    s2 = np.zeros(nb, dtype=object)
    for c in range(3):
        j0 = -((c - b) // 8)  # ceil((b - c) / 8), b >= c
        j1 = (e - c) // 8
        cnt = j1 - j0 + 1
        sj = (j0 + j1) * cnt // 2
        kept += cnt
        s1 += 8 * sj + cnt * (c + 1)
        s2 += 4 * sj + cnt * (c // 2)
    return kept, s1, s2


def test_block_full_size_closed_forms():
    """1.25e8 rows (1 GB) from numbers_mt offset 5e9 in 10,000-row blocks:
    every block's count and each output's wrapping sum over the block's valid
    rows equal their closed forms (size-independent check; sums on the GPU)."""
    begin, br, nb = 5_000_000_000, 10_000, 12_500
    col = ops.numbers_column(begin, br * nb)
    outs, counts = ops.filter_project_blocks(col, br, predicate(U64, [("%", 8)], "<", 3),
                                             [chain(U64, [("+", 1)])[0], chain(U64, [("/", 2)])[0]])
    kept, s1, s2 = _block_closed_forms(begin, nb, br)
    assert counts.tolist() == [int(k) for k in kept]
    cnt = torch.from_numpy(counts).to("cuda")
    mask = torch.arange(br, device="cuda")[None, :] < cnt[:, None]
    for o, s in zip(outs, (s1, s2)):
        v = o.buf[:8 * br * nb].view(torch.int64).view(nb, br)
        got = torch.where(mask, v, torch.zeros_like(v)).sum(dim=1).cpu().numpy().astype(np.uint64)
        assert got.tolist() == [int(x) % (1 << 64) for x in s]



@pytest.mark.parametrize("offset", [0, 1])
@pytest.mark.parametrize("block_rows", [TILE, 10_000, 10_001, 65_536])
def test_block_column_views(offset, block_rows):
    """A column view starting 8 bytes into its buffer (not 16-byte aligned) and
    a 16-byte aligned one, block sizes even and odd."""
    n = 10_000 * 23 + 7
    host = np.arange(n + offset, dtype=np.uint64) * np.uint64(7) + np.uint64(3)
    full = ops.from_numpy(host)
    col = ops.DeviceColumn(full.buf, n, U64, offset=8 * offset)
    h = host[offset:]
    keep = h % np.uint64(5) < np.uint64(2)
    _check(h, keep, predicate(U64, [("%", 5)], "<", 2), [chain(U64, [("+", 1)])[0], None],
           [lambda k: k + np.uint64(1), lambda k: k], block_rows, col=col)


@pytest.mark.parametrize("block_rows", [TILE, 10_000, 10_001])
def test_block_outputs_not_16_byte_aligned(block_rows):
    """Outputs 8 bytes into their buffers: the staged writer stores one row per
    thread instead of 16-byte row pairs; both give the same blocks."""
    n = 10_000 * 31 + 5
    host = np.arange(n, dtype=np.uint64) * np.uint64(3)
    keep = host % np.uint64(8) < np.uint64(3)
    _check(host, keep, predicate(U64, [("%", 8)], "<", 3), [chain(U64, [("+", 1)])[0], None],
           [lambda k: k + np.uint64(1), lambda k: k], block_rows, out_offset=1)


@pytest.mark.parametrize("n_blocks,block_rows,n_cols", [(3000, 64, 1), (20011, 17, 2), (50000, 8, 3), (1025, 1000, 2)])
def test_blocks_compact_multi_chunk_scan(n_blocks, block_rows, n_cols):
    """fq_blocks_compact straight through the C ABI with more blocks than one
    scan chunk holds (the engine's 4e8-row pieces have 40,000 blocks): random
    per-block counts including zeros and full blocks, a short last block, 1-3
    columns -- against numpy's concatenation of each block's valid rows."""
    import ctypes as C

    from fq_amd._lib import check, lib
    rng = np.random.default_rng(n_blocks)
    length = n_blocks * block_rows - block_rows // 2  # the last block is short
    last = length - (n_blocks - 1) * block_rows
    counts = rng.integers(0, block_rows + 1, n_blocks)
    counts[rng.random(n_blocks) < 0.2] = 0
    counts[rng.random(n_blocks) < 0.2] = block_rows
    counts[-1] = min(counts[-1], last)
    cols = [rng.integers(0, 2**63, length, dtype=np.uint64) for _ in range(n_cols)]
    d_in = [ops.from_numpy(c, U64) for c in cols]
    d_out = [ops.empty_column(max(int(counts.sum()), 1), U64) for _ in range(n_cols)]
    d_counts = ops.from_numpy(counts.astype(np.int64), abi.DT_INT64)
    ws = ops.Workspace(lib.fq_blocks_compact_workspace_bytes(n_blocks))
    ins = (C.c_void_p * n_cols)(*[c.ptr for c in d_in])
    outs = (C.c_void_p * n_cols)(*[o.ptr for o in d_out])
    out_len = C.c_int64(-1)
    torch.cuda.synchronize()
    check(lib.fq_blocks_compact(n_cols, ins, length, block_rows, C.c_void_p(d_counts.ptr), outs, C.byref(out_len),
                                ws.ptr, ws.nbytes, C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    assert out_len.value == int(counts.sum())
    for c, o in zip(cols, d_out):
        want = np.concatenate([c[b * block_rows: b * block_rows + int(k)] for b, k in enumerate(counts)])
        got = o.to_numpy()[:out_len.value]
        assert np.array_equal(got, want)
