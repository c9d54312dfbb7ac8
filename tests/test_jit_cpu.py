"""The hipRTC expression specialiser (fuse-query_amd/csrc/fq_jit.hip) on CPU:
every step/compare/predicate shape it can emit is generated and compiled for
gfx950 through fq_jit_prepare (no GPU needed -- the code object is built but
not loaded).  GPU parity of the compiled kernels against the oracle is in
tests/test_kernels_gpu.py, which runs every case interpreted and specialised."""
import ctypes as C
import os

import pytest

from fq_amd import abi, ops
from fq_amd.expr import COL, chain, predicate

ALL = abi.AGG_SUM | abi.AGG_MAX | abi.AGG_MIN | abi.AGG_COUNT
U64, I64, F64 = abi.DT_UINT64, abi.DT_INT64, abi.DT_FLOAT64


@pytest.fixture(autouse=True, scope="module")
def _rtc_available():
    ops.jit_config(abi.JIT_AUTO, 1 << 22)
    if not ops.jit_prepare(U64, value=chain(U64, [("+", 1)])[0]):
        pytest.skip("hipRTC not loadable here")
    if ops.jit_stats()["available"] != 1:
        pytest.skip("hipRTC not loadable here")


VALUE_SHAPES = [
    (U64, [("+", 1)]), (U64, [("-", 1)]), (U64, [("*", 3)]),
    (U64, [("/", 8)]), (U64, [("/", 7)]), (U64, [("/", 3)]), (U64, [("%", 8)]), (U64, [("%", 10)]),
    (U64, [("/", 0)]), (U64, [("%", 0)]), (U64, [("/", 7, True)]), (U64, [("%", COL)]),
    (U64, [("-", (5000, "Int64"))]), (U64, [("*", 3), ("/", 2.0)]), (U64, [("%", 2.5)]),
    (U64, [("+", COL), ("*", COL), ("-", 1, True)]),
    (I64, [("/", (-3, "Int64"))]), (I64, [("%", (7, "Int64"))]), (I64, [("+", 0.5)]),
    (F64, [("*", 2.0), ("+", COL)]), (F64, [("/", 0.0)]), (F64, [("%", 3.0)]),
]


@pytest.mark.parametrize("dt,steps", VALUE_SHAPES, ids=[str(s) for _, s in VALUE_SHAPES])
def test_value_shapes_compile(dt, steps):
    value, _ = chain(dt, steps)
    assert ops.jit_prepare(dt, value=value, mask=ALL)


PRED_SHAPES = [
    (U64, [("%", 8)], "<", 3), (U64, [], ">", 0), (U64, [], "=", COL), (U64, [("+", 1)], ">=", COL),
    (U64, [], "<=", -1), (U64, [("-", 10)], ">", 0.5), (I64, [], "<", (-5, "Int64")),
    (F64, [("*", 2.0)], ">=", 1.5), (F64, [], "=", COL),
]


@pytest.mark.parametrize("dt,lhs,cmp,rhs", PRED_SHAPES, ids=[str(p) for p in PRED_SHAPES])
def test_predicate_shapes_compile_flat_and_block(dt, lhs, cmp, rhs):
    pred = predicate(dt, lhs, cmp, rhs)
    value, _ = chain(dt, [("+", 1)])
    # flat (no sum) and block mode (sum with >1 reference block)
    assert ops.jit_prepare(dt, pred=pred, value=value, mask=abi.AGG_MAX | abi.AGG_COUNT, block_rows=10000)
    assert ops.jit_prepare(dt, pred=pred, mask=ALL, block_rows=10000)


def test_bitmap_predicate_compiles():
    p = abi.fq_pred()
    p.kind = abi.PRED_BITMAP
    assert ops.jit_prepare(U64, pred=p, mask=ALL, block_rows=10000)
    assert ops.jit_prepare(F64, pred=p, mask=abi.AGG_MIN)


def test_unspecialised_shapes():
    # identity scans use the precompiled kernels; narrow columns interpret
    assert not ops.jit_prepare(U64, mask=ALL)
    p = abi.fq_pred()
    p.kind = abi.PRED_BITMAP
    assert not ops.jit_prepare(abi.DT_INT32, pred=p, mask=ALL)
    ops.jit_config(abi.JIT_OFF)
    try:
        assert not ops.jit_prepare(U64, value=chain(U64, [("+", 1)])[0])
    finally:
        ops.jit_config(abi.JIT_AUTO, 1 << 22)


def test_config_roundtrip():
    st0 = ops.jit_stats()
    assert st0["mode"] == abi.JIT_AUTO and st0["min_rows"] == 1 << 22
    with pytest.raises(ops.FQError):
        ops.jit_config(7)


def test_errors():
    from fq_amd._lib import lib
    assert lib.fq_jit_get_stats(None) == abi.FQ_E_INVALID
    assert lib.fq_jit_config(0, -1) != 0
    assert lib.fq_jit_prepare(None, 0, None, None, 0, None) != 0
    c = abi.fq_col(None, 10, abi.DT_UTF8, 0)
    out = C.c_int32(0)
    assert lib.fq_jit_prepare(C.byref(c), 0, None, None, 0, C.byref(out)) != 0


GROUP_SHAPES = [
    ("mod_key_all", U64, [("%", 1000)], [(abi.AGG_COUNT, U64, None), (abi.AGG_SUM, U64, None),
                                         (abi.AGG_MAX, U64, [("+", 1)]), (abi.AGG_MIN, F64, [("*", 1.5)]),
                                         (abi.AGG_SUM, F64, [("/", 3.0)]), (abi.AGG_MAX, F64, [("*", 0.5)])], U64),
    ("signed", U64, [("-", (5, "Int64"))], [(abi.AGG_MIN, I64, [("-", (7, "Int64"))]),
                                           (abi.AGG_MAX, I64, [("-", (7, "Int64"))]),
                                           (abi.AGG_SUM, I64, [("-", (7, "Int64"))])], I64),
    ("identity_key", U64, [], [(abi.AGG_COUNT, U64, None)], U64),
    ("eight_aggs", U64, [("/", 7)], [(abi.AGG_COUNT, U64, None)] * 8, U64),
    ("f64_column", F64, None, [(abi.AGG_SUM, F64, None)], None),
    # dense keys (slot = key): with a COUNT as occupancy, without (key stored)
    ("dense_pow2_no_count", U64, [("*", 3), ("%", 16)], [(abi.AGG_SUM, U64, None), (abi.AGG_MIN, U64, None)], U64),
    ("dense_magic_count", U64, [("%", 4000)], [(abi.AGG_MAX, U64, None), (abi.AGG_COUNT, U64, None)], U64),
    ("dense_too_wide", U64, [("%", 100000)], [(abi.AGG_COUNT, U64, None)], U64),
]


@pytest.mark.parametrize("name,dt,key_steps,aggs,kdt", GROUP_SHAPES, ids=[g[0] for g in GROUP_SHAPES])
def test_groupby_shapes_compile(name, dt, key_steps, aggs, kdt):
    key = chain(dt, key_steps)[0] if key_steps else None
    values = [chain(dt, st)[0] if st else None for _, _, st in aggs]
    spec = [(k, d) for k, d, _ in aggs]
    if kdt is None:  # a Float64 key is outside the device path
        with pytest.raises(ops.FQError):
            ops.group_compile_check(dt, spec, key=key, values=values, key_dtype=F64)
        return
    pred = predicate(dt, [("%", 8)], "<", 3) if dt == U64 else None
    ops.group_compile_check(dt, spec, key=key, values=values, pred=pred, key_dtype=kdt)


@pytest.mark.parametrize("key_steps,log2p", [([("%", 100000)], 8), ([("*", 7), ("%", 100000)], 5),
                                             ([("/", 3)], 6), ([("-", (5, "Int64"))], 1)],
                         ids=["range_bins", "range_bins_p32", "hash_bins", "signed_hash_bins"])
def test_partitioned_groupby_shapes_compile(key_steps, log2p):
    # fq_jit_gpart (block chains) + fq_jit_groupby_bins, range and hash bins
    key, kdt = chain(U64, key_steps)
    aggs = [(abi.AGG_COUNT, U64), (abi.AGG_SUM, U64), (abi.AGG_MAX, U64)]
    pred = predicate(U64, [("%", 8)], "<", 3)
    ops.group_compile_check(U64, aggs, key=key, values=[None] * 3, pred=pred, key_dtype=kdt, log2_parts=log2p)


def test_predicate_tree_shapes_compile():
    from fq_amd.expr import pred_tree
    t = pred_tree(U64, [([("%", 8)], "<", 3), ([], ">", 1000), ([("%", 97)], "=", 0)], [0, 1, "and", 2, "or"])
    value, _ = chain(U64, [("+", 1)])
    assert ops.jit_prepare(U64, pred=t, value=value, mask=abi.AGG_MAX | abi.AGG_COUNT)
    assert ops.jit_prepare(U64, pred=t, value=value, mask=ALL, block_rows=10000)  # block mode
    tf = pred_tree(F64, [([("*", 2.0)], ">=", 1.5), ([], "<", COL)], [0, 1, "or"])
    assert ops.jit_prepare(F64, pred=tf, mask=ALL)
    ops.group_compile_check(U64, [(abi.AGG_COUNT, U64)], key=chain(U64, [("%", 10)])[0], pred=t)
    bad = pred_tree(U64, [([], ">", 1), ([], "<", 5)], [0, 1, "and"])
    bad._tree.prog[2] = 0  # no operator: two values left on the stack
    with pytest.raises(ops.FQError):
        ops.jit_prepare(U64, pred=bad, mask=ALL)


# ---- fused FilterTransform -> ProjectionTransform (fq_filter_project) ------

PROJECT_SHAPES = [
    (U64, None, [None]),
    (U64, None, [chain(U64, [("+", 1)])[0], chain(U64, [("/", 2)])[0]]),
    (U64, ("EXPR", [("+", 1)], "<", 100), [None, chain(U64, [("*", 3)])[0]]),
    (U64, ("EXPR", [("%", 1000)], "=", 999), [chain(U64, [("/", 2.0)])[0]]),
    (U64, ("TREE",), [chain(U64, [("+", 1)])[0], chain(U64, [("-", (5, "Int64"))])[0], None]),
    (I64, ("EXPR", [], "<", (-5, "Int64")), [chain(I64, [("%", (7, "Int64"))])[0]]),
    (F64, ("EXPR", [("*", 2.0)], ">=", 1.5), [None, chain(F64, [("+", COL)])[0]]),
    (U64, None, [chain(U64, [("+", k)])[0] for k in range(8)]),
]


def _project_pred(dt, spec):
    if spec is None:
        return None
    if spec[0] == "TREE":
        from fq_amd.expr import pred_tree
        return pred_tree(U64, [([("%", 8)], "<", 3), ([], ">", 1000)], [0, 1, "and"])
    _, lhs, cmp, rhs = spec
    return predicate(dt, lhs, cmp, rhs)


@pytest.mark.parametrize("i", range(len(PROJECT_SHAPES)))
def test_project_shapes_compile(i):
    # the module (bits, scatter, map kernels) is generated and compiled for
    # gfx950; with no device the call then stops at its first HIP call
    dt, spec, values = PROJECT_SHAPES[i]
    before = ops.jit_stats()["kernels_compiled"]
    st = ops.project_compile_check(dt, _project_pred(dt, spec), values)
    assert st == abi.FQ_E_HIP, (st, ops.lib.fq_last_error())
    assert ops.jit_stats()["kernels_compiled"] == before + 1


@pytest.mark.parametrize("rows,stage", [(8, 1), (16, 1), (16, 2), (32, 2), (32, 4), (16, 0)])
@pytest.mark.parametrize("i", [1, 4, 6])
def test_project_staged_blocks_variant_compiles(i, rows, stage):
    # FQ_TUNE_SELECT_BLOCKS_STAGE: fq_jit_pblocks stages the kept rows in LDS
    # (a 1/stage-tile buffer, passes as needed; 0 = stores from registers)
    dt, spec, values = PROJECT_SHAPES[i]
    try:
        ops.tune_set("SELECT_BLOCKS_STAGE", stage)
        ops.tune_set("SELECT_BLOCKS_ROWS", rows)
        st = ops.project_compile_check(dt, _project_pred(dt, spec), values)
    finally:
        ops.tune_reset()
    assert st == abi.FQ_E_HIP, (st, ops.lib.fq_last_error())


def test_project_rejects_bad_arguments():
    assert ops.project_compile_check(abi.DT_UINT32, None, [None]) == abi.FQ_E_UNSUPPORTED
    assert ops.project_compile_check(U64, None, [None] * 9) == abi.FQ_E_INVALID


# ---- expression trees (FQ_OP_PUSH / FQ_OPERAND_STACK) ----------------------
from fq_amd.expr import PUSH, STACK  # noqa: E402

TREE_SHAPES = [
    (U64, [("+", 1), PUSH, ("/", 2), ("+", STACK, True)]),                       # (x+1)+(x/2)
    (U64, [("+", 1), PUSH, ("+", 2), ("*", STACK, True), ("%", 1000003)]),       # ((x+1)*(x+2))%p
    (U64, [("/", 3), PUSH, ("%", 7), ("*", 2), ("-", STACK, True)]),            # (x/3)-(x%7)*2
    (U64, [("+", 1), PUSH, ("/", 2.0), ("+", STACK, True)]),                     # u64 + f64
    (U64, [("+", 1), PUSH, ("+", 2), PUSH, ("%", 5), ("-", STACK, True), ("*", STACK, True)]),  # depth 2
    (U64, [("-", (5, "Int64")), PUSH, ("*", 3), ("+", STACK, True)]),            # i64 + u64 -> i64
    (I64, [("*", (3, "Int64")), PUSH, ("%", (7, "Int64")), ("/", STACK, True)]),
    (F64, [("*", 2.0), PUSH, ("+", COL), ("/", STACK, True)]),
]


@pytest.mark.parametrize("dt,steps", TREE_SHAPES, ids=[str(s) for _, s in TREE_SHAPES])
def test_tree_shapes_compile(dt, steps):
    value, _ = chain(dt, steps)
    assert ops.jit_prepare(dt, value=value, mask=ALL)
    pred = predicate(dt, steps, "<", 100)
    assert ops.jit_prepare(dt, pred=pred, mask=ALL, block_rows=10000)
    assert ops.project_compile_check(dt, pred, [value, None]) == abi.FQ_E_HIP


def test_tree_lowering_rejects_unbalanced_and_deep():
    unbalanced, _ = chain(U64, [("+", 1), PUSH, ("+", 2)])
    unbalanced.out_dtype = U64
    with pytest.raises(ops.FQError):
        ops.jit_prepare(U64, value=unbalanced, mask=ALL)
    deep = chain(U64, [PUSH, PUSH, PUSH, ("+", STACK, True), ("+", STACK, True), ("+", STACK, True)])[0]
    with pytest.raises(ops.FQError):
        ops.jit_prepare(U64, value=deep, mask=ALL)


@pytest.mark.parametrize("i", range(5))
def test_oracle_tree_matches_numpy(i):
    # the C oracle's tree evaluation (oracle/fq_oracle.c eval_chain) against a
    # direct numpy/python evaluation of the same tree
    import numpy as np
    import oracle_c
    host = np.arange(1, 20_001, dtype=np.uint64) * np.uint64(7919)
    dt, steps = TREE_SHAPES[i]
    value, vdt = chain(dt, steps)
    st = oracle_c.column_partial(host, dt, 10000, [(abi.AGG_MAX, value), (abi.AGG_MIN, value)])
    x = [int(v) for v in host]
    M = 2**64

    def ev(v):
        if i == 0:
            return (v + 1 + v // 2) % M
        if i == 1:
            return ((v + 1) * (v + 2) % M) % 1000003
        if i == 2:
            return (v // 3 - (v % 7) * 2) % M
        if i == 3:
            return float(v + 1) + v / 2.0
        return ((v + 1) * ((v + 2) - v % 5)) % M
    vals = [ev(v) for v in x]
    from fq_amd.expr import from_bits
    assert from_bits(st[0].bits, vdt) == max(vals)
    assert from_bits(st[1].bits, vdt) == min(vals)


MANY_THREADS = r"""
import sys, threading
sys.path.insert(0, sys.argv[1])
from fq_amd import abi, ops
from fq_amd.expr import chain, predicate
U64 = abi.DT_UINT64
errors = []

def compile_shape(j):
    try:
        key, kdt = chain(U64, [("+", 1)] * (1 + j % 4) + [("%", 100000)])
        aggs = [(abi.AGG_COUNT, U64)] + [(abi.AGG_MAX, U64)] * (j // 4 % 4)
        pred = predicate(U64, [("%", 8)], "<", 3) if j >= 16 else None
        ops.group_compile_check(U64, aggs, key=key, values=[None] * len(aggs), pred=pred, key_dtype=kdt,
                                log2_parts=6)
    except Exception as e:
        errors.append(e)

for r in range(2):
    ts = [threading.Thread(target=compile_shape, args=(r * 8 + w,)) for w in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
assert not errors, errors
print("compiled", ops.jit_stats()["kernels_compiled"])
"""


def test_compiles_from_many_threads():
    # hipRTC is loaded into a link-map namespace of its own; compiles issued
    # from many fresh threads (the engine's workers) crashed the process inside
    # hipRTC until every call went through its one compiler thread (fq_jit.hip
    # RtcThread).  16 distinct shapes (key chain length x aggregate count x
    # predicate), each compiled on a thread of its own, 8 at a time, in a child
    # process without the comgr cache (cached code objects never reach the
    # compiler; the namespace's libc reads the environment only when loaded).
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd")
    env = dict(os.environ, AMD_COMGR_CACHE="0")
    r = subprocess.run([sys.executable, "-c", MANY_THREADS, pkg], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "compiled 16" in r.stdout, r.stdout
