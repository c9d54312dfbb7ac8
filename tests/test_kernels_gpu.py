"""Parity of the gfx950 kernels (through the C ABI) against the C oracle and
numpy, on seeded inputs at sizes the oracle finishes in seconds.

Bit-exact for integer results; float sums within the tolerance written in
each test (reduction order differs from arrow's lane-wise simd sum)."""
import ctypes as C

import numpy as np
import pytest

from fq_amd import abi
from fq_amd.expr import COL, chain, predicate, to_bits

import oracle_c
from replay import as_tuple, replay

pytestmark = pytest.mark.gpu

ops = None


def setup_module():
    global ops
    from fq_amd import ops as _ops
    _ops.require_gpu()
    ops = _ops


ALL = abi.AGG_SUM | abi.AGG_MAX | abi.AGG_MIN | abi.AGG_COUNT
AGGS = [abi.AGG_SUM, abi.AGG_MAX, abi.AGG_MIN, abi.AGG_COUNT]


@pytest.fixture(autouse=True, params=["interp", "jit"])
def jit_mode(request):
    """Every case runs twice: on the precompiled program-interpreting scan and
    on the hipRTC-specialised scan (fq_jit.hip) for the same shape."""
    if request.param == "jit":
        ops.jit_config(abi.JIT_ALWAYS, 0)
    else:
        ops.jit_config(abi.JIT_OFF)
    yield request.param
    ops.jit_config(abi.JIT_AUTO, 1 << 22)


def check_against_oracle(host, dtype, block_rows, pred=None, value=None, gpu_col=None):
    """One device block vs the oracle's per-block loop over the same column."""
    col = gpu_col if gpu_col is not None else ops.from_numpy(host, dtype)
    aggs = [(op, value) for op in AGGS]
    try:
        exp = [as_tuple(s) for s in oracle_c.column_partial(host, dtype, block_rows, aggs, pred)]
        exp_err = None
    except oracle_c.OracleError as e:
        exp, exp_err = None, e
    st = ops.aggregate(col, block_rows, pred, value, ALL)
    if exp_err is not None:
        with pytest.raises(oracle_c.OracleError) as ei:
            for op in AGGS:
                replay(op, st)
        assert str(ei.value) == str(exp_err)
        return st
    got = [replay(op, st) for op in AGGS]
    assert got == exp, (got, exp, ops.state_values(st))
    return st


def test_fill_numbers_matches_numbers_stream():
    for begin, n in [(0, 1), (5, 17), (1_250_000_000, 100_003), (2**40, 4097)]:
        c = ops.numbers_column(begin, n)
        assert np.array_equal(c.to_numpy(), np.arange(begin, begin + n, dtype=np.uint64))


def test_fill_splitmix_matches_oracle():
    c = ops.splitmix_column(0x5EED, 123, 1000)
    L = oracle_c.lib()
    exp = np.array([L.fqo_splitmix64(0x5EED, 123 + i) for i in range(1000)], dtype=np.uint64)
    assert np.array_equal(c.to_numpy(), exp)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 7, 16, 63, 64, 65, 1000, 10000, 10001, 123457, 1 << 20])
def test_identity_u64_all_aggs(n):
    host = np.random.default_rng(n).integers(0, 2**64, size=n, dtype=np.uint64)
    st = check_against_oracle(host, abi.DT_UINT64, 10000)
    if n:
        assert st.sum == int(host.sum(dtype=np.uint64))  # numpy wraps mod 2^64
        assert st.max == int(host.max()) and st.min == int(host.min()) and st.count == n


def test_misaligned_column_head_and_tail():
    host = np.arange(1, 1 + 100_003, dtype=np.uint64) * np.uint64(7919)
    base = ops.from_numpy(np.concatenate([np.zeros(1, np.uint64), host]))
    col = ops.DeviceColumn(base.buf, host.shape[0], abi.DT_UINT64, offset=8)  # 8-byte aligned only
    check_against_oracle(host, abi.DT_UINT64, 10000, gpu_col=col)


@pytest.mark.parametrize("dt,npdt", [(abi.DT_INT64, np.int64), (abi.DT_INT32, np.int32),
                                     (abi.DT_UINT8, np.uint8), (abi.DT_INT16, np.int16),
                                     (abi.DT_UINT32, np.uint32)])
def test_identity_small_and_signed_types(dt, npdt):
    rng = np.random.default_rng(7)
    info = np.iinfo(npdt)
    host = rng.integers(info.min, info.max, size=50_001, dtype=npdt, endpoint=True)
    st = ops.aggregate(ops.from_numpy(host, dt), 0, None, None, ALL)
    v = ops.state_values(st)
    # arrow sum on T wraps in T (simd add); compare modulo the width
    mod = 1 << (8 * host.dtype.itemsize)
    assert (v["sum"] - int(host.astype(object).sum())) % mod == 0
    assert v["max"] == int(host.max()) and v["min"] == int(host.min()) and v["count"] == host.shape[0]


def test_f64_sum_tolerance_minmax_exact():
    rng = np.random.default_rng(11)
    host = rng.standard_normal(1_000_003) * 1e3
    st = ops.aggregate(ops.from_numpy(host), 0, None, None, ALL)
    v = ops.state_values(st)
    exp = float(np.sum(host.astype(np.float64)))
    # tolerance: |err| <= 1e-12 * sum(|x|) (order-of-summation bound, n ~ 1e6)
    assert abs(v["sum"] - exp) <= 1e-12 * float(np.abs(host).sum())
    assert v["max"] == float(host.max()) and v["min"] == float(host.min())


def test_numbers_plus_one_with_mod_predicate():
    # C4 shape: max(number+1) WHERE (number%8)<3 over one numbers_mt partition
    n = 250_000
    host = np.arange(1_000_000, 1_000_000 + n, dtype=np.uint64)
    value, _ = chain(abi.DT_UINT64, [("+", 1)])
    pred = predicate(abi.DT_UINT64, [("%", 8)], "<", 3)
    check_against_oracle(host, abi.DT_UINT64, 10000, pred=pred, value=value)


@pytest.mark.parametrize("d", [1, 2, 3, 7, 8, 10, 641, 999, 1000, 1001, 4095, 10000, 65521, 65535, 65537,
                               1 << 33, (1 << 63) + 1, 2**64 - 1, 0x1234567890abcdef])
def test_div_mod_by_constant_magic(d):
    # '%' by d <= 65535 runs on 32-bit halves (K_MODM32_U), larger d on the
    # 64-bit multiply-high magic
    rng = np.random.default_rng(d & 0xffff)
    host = rng.integers(0, 2**64, size=70_001, dtype=np.uint64)
    host[:8] = [0, 1, d - 1 if d > 1 else 0, 2**64 - 1, 2**32 - 1, 2**32, (2**32 * d - 1) % 2**64, 2**63]
    for sym, ref in (("/", host // np.uint64(d)), ("%", host % np.uint64(d))):
        value, _ = chain(abi.DT_UINT64, [(sym, d)])
        st = ops.aggregate(ops.from_numpy(host), 0, None, value, ALL)
        assert st.flags == 0
        assert st.sum == int(ref.sum(dtype=np.uint64)), sym
        assert st.max == int(ref.max()) and st.min == int(ref.min()), sym


def test_div_by_zero_constant_and_column():
    host = np.arange(0, 20_000, dtype=np.uint64)
    value, _ = chain(abi.DT_UINT64, [("/", 0)])
    check_against_oracle(host, abi.DT_UINT64, 10000, value=value)  # error path
    value2, _ = chain(abi.DT_UINT64, [("/", 7, True)])  # 7 / number: zero at row 0
    check_against_oracle(host, abi.DT_UINT64, 10000, value=value2)
    # zero divisor only in rows the predicate drops -> no error (eval on filtered block)
    pred = predicate(abi.DT_UINT64, [], ">", 0)
    check_against_oracle(host, abi.DT_UINT64, 10000, pred=pred, value=value2)


def test_filtered_sum_empty_block_semantics():
    host = np.arange(0, 50_000, dtype=np.uint64)
    value, _ = chain(abi.DT_UINT64, [])
    # only the first block has rows with number < 5 -> later blocks empty -> Sum errors
    pred = predicate(abi.DT_UINT64, [], "<", 5)
    st = check_against_oracle(host, abi.DT_UINT64, 10000, pred=pred)
    assert st.flags & abi.STATE_ANY_EMPTY
    # every block keeps rows -> fine
    pred2 = predicate(abi.DT_UINT64, [("%", 10)], "=", 3)
    check_against_oracle(host, abi.DT_UINT64, 10000, pred=pred2)
    # single block, nothing passes -> Sum state None, Min/Max None
    pred3 = predicate(abi.DT_UINT64, [], ">", 10**12)
    check_against_oracle(host[:7000], abi.DT_UINT64, 10000, pred=pred3)


def test_mixed_types_chain_f64_and_i64():
    host = np.arange(0, 30_000, dtype=np.uint64)
    v1, _ = chain(abi.DT_UINT64, [("*", 3), ("/", 2.0)])  # u64 * u64 -> / f64 -> Float64
    st = ops.aggregate(ops.from_numpy(host), 10000, None, v1, ALL)
    ref = host.astype(np.float64) * 3 / 2.0
    v = ops.state_values(st)
    assert v["dtype"] == abi.DT_FLOAT64
    assert abs(v["sum"] - ref.sum()) <= 1e-12 * abs(ref).sum()
    assert v["max"] == ref.max() and v["min"] == ref.min()
    v2, _ = chain(abi.DT_UINT64, [("-", (5000, "Int64"))])  # UInt64 - Int64 -> Int64
    check_against_oracle(host, abi.DT_UINT64, 10000, value=v2)


def test_random_column_matches_oracle_loop():
    seed, n = 0x5EED, 300_000
    col = ops.splitmix_column(seed, 0, n)
    host = col.to_numpy()
    value, _ = chain(abi.DT_UINT64, [("%", 1000003), ("*", 13)])
    pred = predicate(abi.DT_UINT64, [("%", 8)], "<", 3)
    check_against_oracle(host, abi.DT_UINT64, 10000, pred=pred, value=value, gpu_col=col)


def test_arith_compare_filter_elementwise():
    rng = np.random.default_rng(3)
    a = rng.integers(0, 2**64, size=10_007, dtype=np.uint64)
    b = rng.integers(1, 2**20, size=10_007, dtype=np.uint64)
    A, B = ops.from_numpy(a), ops.from_numpy(b)
    assert np.array_equal(ops.arith("+", A, B).to_numpy(), a + b)
    assert np.array_equal(ops.arith("-", A, B).to_numpy(), a - b)
    assert np.array_equal(ops.arith("*", A, B).to_numpy(), a * b)
    assert np.array_equal(ops.arith("/", A, B).to_numpy(), a // b)
    assert np.array_equal(ops.arith("%", A, B).to_numpy(), a % b)
    assert np.array_equal(ops.arith("-", 1, B).to_numpy(), np.uint64(1) - b)
    m = ops.compare("<", B, 1000)
    assert np.array_equal(m.to_numpy(), b < 1000)
    m2 = ops.compare(">", 1000, B)  # scalar-array: flipped operator
    assert np.array_equal(m2.to_numpy(), b < 1000)
    kept = ops.filter_compact(A, m)
    assert np.array_equal(kept.to_numpy(), a[b < 1000])


def test_arith_div_zero_error_text():
    A = ops.from_numpy(np.array([4, 3, 2, 1], np.uint64))
    Z = ops.from_numpy(np.array([1, 0, 3, 4], np.uint64))
    with pytest.raises(ops.FQError) as ei:
        ops.arith("/", A, Z)
    assert str(ei.value) == "Internal Error: Divide by zero error"
    assert ei.value.status == abi.FQ_E_DIVIDE_BY_ZERO


def test_filter_compaction_large_ragged():
    n = 3 * 16384 + 77
    rng = np.random.default_rng(9)
    x = rng.integers(0, 2**64, size=n, dtype=np.uint64)
    X = ops.from_numpy(x)
    for thr in (0, 2**62, 2**63, 2**64 - 1):
        m = ops.compare("<", X, (thr, "UInt64"))
        kept = ops.filter_compact(X, m)
        assert np.array_equal(kept.to_numpy(), x[x < np.uint64(thr)])


@pytest.mark.parametrize("shape", ["c4", "chain_f64", "div_col", "block_sum", "bitmap"])
def test_specialised_scan_bit_identical_to_interpreter(shape, jit_mode):
    """Same grid, same per-lane order: the fq_agg_state bytes must match."""
    if jit_mode != "jit":
        pytest.skip("compares both modes itself")
    n = 3_000_017
    col = ops.splitmix_column(0xC4, 0, n)
    br, pred, value, mask = 0, None, None, ALL
    if shape == "c4":
        value, _ = chain(abi.DT_UINT64, [("+", 1)])
        pred = predicate(abi.DT_UINT64, [("%", 8)], "<", 3)
        mask = abi.AGG_MAX | abi.AGG_COUNT
    elif shape == "chain_f64":
        value, _ = chain(abi.DT_UINT64, [("%", 1000), ("*", 0.5), ("+", COL)])
    elif shape == "div_col":
        value, _ = chain(abi.DT_UINT64, [("%", 977), ("/", COL, True)])
    elif shape == "block_sum":
        pred = predicate(abi.DT_UINT64, [("%", 10)], "=", 3)
        br = 10000
    else:
        bm = ops.compare("<", col, 2**63)
        pred = abi.fq_pred()
        pred.kind = abi.PRED_BITMAP
        pred.bitmap = bm.ptr
    before = ops.jit_stats()["jit_launches"]
    got = bytes(ops.aggregate(col, br, pred, value, mask))
    assert ops.jit_stats()["jit_launches"] == before + 1
    ops.jit_config(abi.JIT_OFF)
    exp = bytes(ops.aggregate(col, br, pred, value, mask))
    assert got == exp


def test_unknown_aggregate_mask_bits_are_refused():
    """agg_mask carries FQ_AGG_* bits only (round 5's in-launch finalize flag
    0x100 is gone with its variant)."""
    col = ops.numbers_column(0, 100_000)
    with pytest.raises(Exception, match="unknown bits"):
        ops.aggregate(col, 0, None, None, ALL | 0x100)


def _trunc_divmod(a, b):
    q = (np.abs(a) // np.abs(b)) * (np.sign(a) * np.sign(b))
    return q, a - q * b


@pytest.mark.parametrize("n", [4096 * 3, 4096 * 3 + 1, 512 * 7 + 63, 200_003])
@pytest.mark.parametrize("dt", [abi.DT_UINT64, abi.DT_INT64, abi.DT_FLOAT64])
def test_elementwise_vector_fast_paths(n, dt, jit_mode):
    """64-bit same-type operands take the 16-byte vector kernels for whole
    tiles and the generic kernels for the rest; both must agree with numpy
    (arrow semantics: wrapping ints, truncating integer division)."""
    if jit_mode != "interp":
        pytest.skip("no expression program involved")
    rng = np.random.default_rng(n + dt)
    if dt == abi.DT_UINT64:
        a = rng.integers(0, 2**64, size=n, dtype=np.uint64)
        b = rng.integers(1, 2**40, size=n, dtype=np.uint64)
        k = (12345, "UInt64")
    elif dt == abi.DT_INT64:
        a = rng.integers(-2**62, 2**62, size=n, dtype=np.int64)
        b = rng.integers(-2**30, 2**30, size=n, dtype=np.int64)
        b[b == 0] = 7
        k = (-977, "Int64")
    else:
        a = rng.standard_normal(n) * 1e6
        b = rng.standard_normal(n)
        a[::97] = np.nan
        k = 0.75
    A, B = ops.from_numpy(a, dt), ops.from_numpy(b, dt)
    kv = np.array([k[0] if isinstance(k, tuple) else k], dtype=a.dtype)[0]
    with np.errstate(all="ignore"):
        for sym in "+-*/%":
            for lhs, rhs, x, y in ((A, B, a, b), (A, k, a, kv), (k, B, kv, b)):
                got = ops.arith(sym, lhs, rhs).to_numpy()
                if sym == "+":
                    exp = x + y
                elif sym == "-":
                    exp = x - y
                elif sym == "*":
                    exp = x * y
                elif dt == abi.DT_FLOAT64:
                    exp = x / y if sym == "/" else np.fmod(x, y)
                elif dt == abi.DT_UINT64:
                    exp = x // y if sym == "/" else x % y
                else:
                    q, r = _trunc_divmod(np.asarray(x, np.int64), np.asarray(y, np.int64))
                    exp = q if sym == "/" else r
                exp = np.broadcast_to(exp, (n,))
                if dt == abi.DT_FLOAT64:
                    assert np.array_equal(got, exp, equal_nan=True), sym
                else:
                    assert np.array_equal(got, exp), sym
        for sym, f in (("=", np.equal), ("<", np.less), ("<=", np.less_equal), (">", np.greater),
                       (">=", np.greater_equal)):
            assert np.array_equal(ops.compare(sym, A, B).to_numpy(), f(a, b)), sym
            assert np.array_equal(ops.compare(sym, A, k).to_numpy(), f(a, kv)), sym
    # misaligned slices (8-byte offset) fall back to the generic kernels
    As = ops.DeviceColumn(A.buf, n - 1, dt, offset=8)
    Bs = ops.DeviceColumn(B.buf, n - 1, dt, offset=8)
    with np.errstate(all="ignore"):
        assert np.array_equal(ops.arith("+", As, Bs).to_numpy(), (a[1:] + b[1:]), equal_nan=dt == abi.DT_FLOAT64)
    assert np.array_equal(ops.compare("<", As, Bs).to_numpy(), a[1:] < b[1:])


def test_elementwise_fast_path_div_zero_in_tile_and_tail():
    n = 4096 * 2 + 100
    a = np.arange(n, dtype=np.uint64)
    for zero_at in (5, 4096 + 17, n - 3):  # inside a vector tile / in the generic tail
        b = np.ones(n, np.uint64)
        b[zero_at] = 0
        with pytest.raises(ops.FQError) as ei:
            ops.arith("%", ops.from_numpy(a), ops.from_numpy(b))
        assert str(ei.value) == "Internal Error: Divide by zero error"


def test_filter_compaction_many_tiles(jit_mode):
    """> 16 x 512 tiles: every wave of the tile-count scan walks several
    512-entry chunks, the last one ragged."""
    if jit_mode != "interp":
        pytest.skip("no expression program involved")
    n = 16384 * 9001 + 77
    X = ops.splitmix_column(0xF1, 0, n)
    x = X.to_numpy()
    thr = np.uint64(5 * 2**61)
    kept = ops.filter_compact(X, ops.compare("<", X, (int(thr), "UInt64")))
    assert np.array_equal(kept.to_numpy(), x[x < thr])


@pytest.mark.parametrize("n", [1, 63, 64, 127, 128, 129, 16384 * 3 + 1, 16384 * 5 + 128, 1_000_003])
def test_filter_compaction_vector_path_edges(n, jit_mode):
    """16-byte-aligned 8-byte columns take the pairwise vector scatter; odd
    lengths end on a row whose pair partner is past the column."""
    if jit_mode != "interp":
        pytest.skip("no expression program involved")
    rng = np.random.default_rng(n)
    for dt, npdt in ((abi.DT_UINT64, np.uint64), (abi.DT_FLOAT64, np.float64), (abi.DT_INT64, np.int64)):
        x = rng.integers(0, 2**40, size=n).astype(npdt)
        X = ops.from_numpy(x, dt)
        for thr in (0.0, 0.3, 0.97, 1.0):
            keep = rng.random(n) < thr
            keep[-1] = True  # the last row (odd lengths: no pair partner)
            m = ops.from_numpy(keep.astype(np.uint64), abi.DT_UINT64)
            bm = ops.compare("=", m, 1)
            got = ops.filter_compact(X, bm).to_numpy()
            assert np.array_equal(got, x[keep]), (dt, thr)
    # 8-byte-offset output: aligned input takes the pairwise register scatter
    x = rng.integers(0, 2**40, size=n).astype(np.uint64)
    keep = rng.random(n) < 0.4
    keep[-1] = True
    X = ops.from_numpy(x)
    bm = ops.compare("=", ops.from_numpy(keep.astype(np.uint64)), 1)
    out = ops.empty_column(n + 1, abi.DT_UINT64)
    ws = ops.Workspace(ops.lib.fq_filter_workspace_bytes(n))
    kept = C.c_int64(0)
    ops.check(ops.lib.fq_filter_compact(C.byref(X.col()), C.c_void_p(bm.ptr), C.c_void_p(out.ptr + 8),
                                        C.byref(kept), ws.ptr, ws.nbytes, None))
    assert kept.value == int(keep.sum())
    got = out.buf[8: 8 + 8 * kept.value].cpu().numpy().view(np.uint64)
    assert np.array_equal(got, x[keep])
    # misaligned (8-byte offset) input keeps the scalar scatter
    X = ops.from_numpy(np.arange(n + 1, dtype=np.uint64))
    Xs = ops.DeviceColumn(X.buf, n, abi.DT_UINT64, offset=8)
    bm = ops.compare("<", Xs, 2**63)
    assert np.array_equal(ops.filter_compact(Xs, bm).to_numpy(), np.arange(1, n + 1, dtype=np.uint64))


@pytest.mark.parametrize("block_rows,n,offset", [(10000, 100_001, 0), (9999, 99_990, 0), (10000, 60_000, 1),
                                                  (2, 1001, 0), (64, 6401, 0)])
def test_block_mode_vector_and_scalar_paths(block_rows, n, offset):
    """Filtered sum (block mode): even block sizes on an aligned column take
    16-byte loads, odd ones / misaligned columns 8-byte loads; every block's
    emptiness must match the reference's per-block state machine."""
    host = np.arange(5, 5 + n + offset, dtype=np.uint64)
    X = ops.from_numpy(host)
    col = ops.DeviceColumn(X.buf, n, abi.DT_UINT64, offset=8 * offset) if offset else X
    h = host[offset:]
    value, _ = chain(abi.DT_UINT64, [("+", 1)])
    for pred in (predicate(abi.DT_UINT64, [("%", 8)], "<", 3),     # every block keeps rows
                 predicate(abi.DT_UINT64, [], "<", 5 + block_rows)):  # only the first block does
        check_against_oracle(h, abi.DT_UINT64, block_rows, pred=pred, value=value, gpu_col=col)


TREES = [
    ("and", [([("%", 8)], "<", 3), ([], ">", 1000)], [0, 1, "and"]),
    ("or", [([], "<", 5000), ([("%", 97)], "=", 0)], [0, 1, "or"]),
    ("nested", [([("%", 8)], "<", 3), ([], ">", 10), ([], "=", 5), ([("/", 3)], ">=", 2)],
     [0, 1, "and", 2, "or", 3, "and"]),
]


@pytest.mark.parametrize("name,leaves,prog", TREES, ids=[t[0] for t in TREES])
def test_predicate_tree_scan_matches_numpy(name, leaves, prog, jit_mode):
    """FQ_PRED_TREE (LogicFunction over comparisons) in the fused scan,
    interpreted (truth table) and specialised (boolean expression)."""
    from fq_amd.expr import pred_tree
    n = 1_000_003
    x = np.arange(3, 3 + n, dtype=np.uint64)
    col = ops.from_numpy(x)
    pred = pred_tree(abi.DT_UINT64, leaves, prog)
    value, _ = chain(abi.DT_UINT64, [("+", 1)])
    masks = []
    for steps, cmp, rhs in leaves:
        v = x.copy()
        for sym, k in steps:
            v = v % np.uint64(k) if sym == "%" else v // np.uint64(k)
        masks.append({"<": v < rhs, ">": v > rhs, "=": v == rhs, ">=": v >= rhs}[cmp])
    st = []
    for t in prog:
        if isinstance(t, str):
            b, a = st.pop(), st.pop()
            st.append(a & b if t == "and" else a | b)
        else:
            st.append(masks[t])
    m = st[0]
    y = (x + np.uint64(1))[m]
    s = ops.aggregate(col, 0, pred, value, ALL)  # one block
    assert s.count == int(m.sum())
    assert s.sum == int(y.sum(dtype=np.uint64)) and s.max == int(y.max()) and s.min == int(y.min())
    # many reference blocks: flat for max/count, block mode for sum
    s2 = ops.aggregate(col, 10000, pred, value, abi.AGG_MAX | abi.AGG_COUNT)
    assert s2.count == int(m.sum()) and s2.max == int(y.max())
