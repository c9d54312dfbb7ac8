"""TEST INFRASTRUCTURE ONLY: ctypes binding of the C oracle (fq_oracle.c).

Used by tests/ as the parity checker and by bench.py's cpu_baseline leg.
It borrows the struct layouts of include/fq_gpu.h through fq_amd.abi but never
calls the product library.

Also restates AggregateFinalTransform's merge of the partial states
(src/transforms/transform_aggregate_final.rs:50-78 ->
AggregatorFunction::merge_state, src/functions/function_aggregator.rs:106-139)
with the reference's DataValue semantics (Null absorbs, typed None makes the
Sum merge fail, min/max skip None).
"""
import ctypes as C
import os
import struct
import subprocess

from fq_amd import abi

_HERE = os.path.dirname(os.path.abspath(__file__))

FQO_NULL, FQO_NONE, FQO_SOME = 0, 1, 2
SRC_NUMBERS, SRC_SPLITMIX = 0, 1


class fqo_state(C.Structure):
    _fields_ = [("kind", C.c_int32), ("dtype", C.c_int32), ("bits", C.c_uint64)]


def _path(native=False):
    return os.path.join(_HERE, "build", "libfq_oracle_native.so" if native else "libfq_oracle.so")


def build(native=False):
    subprocess.run(["make", "-s", "-C", _HERE] + (["native"] if native else []), check=True)
    return _path(native)


def load(native=False):
    p = _path(native)
    if not os.path.exists(p):
        build(native)
    lib = C.CDLL(p)
    P = C.POINTER
    lib.fqo_num_partitions.restype = C.c_int32
    lib.fqo_num_partitions.argtypes = [C.c_uint64]
    lib.fqo_partition_range.restype = None
    lib.fqo_partition_range.argtypes = [C.c_uint64, C.c_int32, P(C.c_uint64), P(C.c_uint64)]
    lib.fqo_partition_rows.restype = C.c_uint64
    lib.fqo_partition_rows.argtypes = [C.c_uint64, C.c_int32]
    lib.fqo_splitmix64.restype = C.c_uint64
    lib.fqo_splitmix64.argtypes = [C.c_uint64, C.c_uint64]
    lib.fqo_numbers_partial.restype = C.c_int32
    lib.fqo_numbers_partial.argtypes = [
        C.c_uint64, C.c_int32, C.c_uint64, C.c_int32, C.c_int32, P(abi.fq_pred), C.c_int32,
        P(C.c_int32), P(abi.fq_expr), C.c_int32, P(fqo_state), P(C.c_int32), C.c_char_p, C.c_int32]
    lib.fqo_numbers_partial_split.restype = C.c_int32
    lib.fqo_numbers_partial_split.argtypes = [
        C.c_uint64, P(abi.fq_pred), C.c_int32, P(C.c_int32), P(abi.fq_expr), C.c_int32, C.c_int32, P(fqo_state),
        C.c_char_p, C.c_int32]
    lib.fqo_column_partial.restype = C.c_int32
    lib.fqo_column_partial.argtypes = [
        C.c_void_p, C.c_int32, C.c_int64, C.c_int64, P(abi.fq_pred), C.c_int32, P(C.c_int32),
        P(abi.fq_expr), P(fqo_state), C.c_char_p, C.c_int32]
    lib.fqo_numbers_group.restype = C.c_int32
    lib.fqo_numbers_group.argtypes = [
        C.c_uint64, C.c_int32, C.c_uint64, P(abi.fq_pred), P(abi.fq_expr), C.c_int32, P(C.c_int32), P(C.c_int32),
        P(abi.fq_expr), C.c_int32, C.c_uint64, C.c_void_p, C.c_void_p, P(C.c_uint64), C.c_char_p, C.c_int32]
    lib.fqo_numbers_project.restype = C.c_int32
    lib.fqo_numbers_project.argtypes = [C.c_uint64, P(abi.fq_pred), C.c_int32, P(abi.fq_expr), C.c_int32,
                                        P(C.c_uint64), P(C.c_uint64), C.c_char_p, C.c_int32]
    return lib


_LIB = None


def lib(native=False):
    global _LIB
    if native:
        return load(True)
    if _LIB is None:
        _LIB = load(False)
    return _LIB


class OracleError(Exception):
    def __init__(self, status, msg):
        super().__init__(msg)
        self.status = status


def partitions(total):
    L = lib()
    out = []
    for p in range(L.fqo_num_partitions(total)):
        b, e = C.c_uint64(0), C.c_uint64(0)
        L.fqo_partition_range(total, p, C.byref(b), C.byref(e))
        out.append((b.value, e.value, L.fqo_partition_rows(total, p)))
    return out


def _identity(dtype):
    e = abi.fq_expr()
    e.n_steps = 0
    e.out_dtype = dtype
    return e


def numbers_partial(total, aggs, pred=None, src=SRC_NUMBERS, seed=0, p0=0, p1=None, threads=0,
                    native=False):
    """aggs: [(agg_op, fq_expr or None)].  Returns (states[part][agg], statuses, err)."""
    L = lib(native)
    if p1 is None:
        p1 = L.fqo_num_partitions(total)
    n = len(aggs)
    ops = (C.c_int32 * n)(*[a for a, _ in aggs])
    args = (abi.fq_expr * n)(*[(e if e is not None else _identity(abi.DT_UINT64)) for _, e in aggs])
    np_ = p1 - p0
    states = (fqo_state * (np_ * n))()
    st = (C.c_int32 * np_)()
    err = C.create_string_buffer(512)
    L.fqo_numbers_partial(total, src, seed, p0, p1, C.byref(pred) if pred is not None else None, n,
                          ops, args, threads, states, st, err, 512)
    rows = [[states[i * n + a] for a in range(n)] for i in range(np_)]
    return rows, list(st), err.value.decode()


def numbers_partial_split(total, aggs, pred=None, threads=0, slices=1, native=False):
    """numbers_partial with every partition's blocks cut into `slices` tasks
    (fqo_numbers_partial_split): (states[task][agg], err)."""
    L = lib(native)
    n = len(aggs)
    ops = (C.c_int32 * n)(*[a for a, _ in aggs])
    args = (abi.fq_expr * n)(*[(e if e is not None else _identity(abi.DT_UINT64)) for _, e in aggs])
    nt = L.fqo_num_partitions(total) * slices
    states = (fqo_state * (nt * n))()
    err = C.create_string_buffer(512)
    rc = L.fqo_numbers_partial_split(total, C.byref(pred) if pred is not None else None, n, ops, args, threads,
                                     slices, states, err, 512)
    return [[states[i * n + a] for a in range(n)] for i in range(nt)], rc, err.value.decode()


def column_partial(arr, dtype, block_rows, aggs, pred=None):
    """Partial states over a host numpy column (64-bit dtypes)."""
    L = lib()
    n = len(aggs)
    ops = (C.c_int32 * n)(*[a for a, _ in aggs])
    args = (abi.fq_expr * n)(*[(e if e is not None else _identity(dtype)) for _, e in aggs])
    states = (fqo_state * n)()
    err = C.create_string_buffer(512)
    rc = L.fqo_column_partial(arr.ctypes.data, dtype, arr.shape[0], block_rows,
                              C.byref(pred) if pred is not None else None, n, ops, args, states,
                              err, 512)
    if rc:
        raise OracleError(rc, err.value.decode())
    return [states[a] for a in range(n)]


def numbers_group(total, key, aggs, pred=None, src=SRC_NUMBERS, seed=0, threads=0, cap_groups=1 << 20,
                  native=False):
    """GROUP BY over numbers_mt(total): key = fq_expr over the column (None =
    the column), aggs = [(agg_op, state dtype, fq_expr or None)].  Returns
    (keys uint64[groups], states uint64[groups, len(aggs)]), unordered."""
    import numpy as np
    L = lib(native)
    n = len(aggs)
    ops = (C.c_int32 * n)(*[a for a, _, _ in aggs])
    dts = (C.c_int32 * n)(*[d for _, d, _ in aggs])
    args = (abi.fq_expr * n)(*[(e if e is not None else _identity(abi.DT_UINT64)) for _, _, e in aggs])
    k = key if key is not None else _identity(abi.DT_UINT64)
    keys = np.zeros(cap_groups, np.uint64)
    states = np.zeros((cap_groups, n), np.uint64)
    groups = C.c_uint64(0)
    err = C.create_string_buffer(512)
    rc = L.fqo_numbers_group(total, src, seed, C.byref(pred) if pred is not None else None, C.byref(k), n, ops, dts,
                             args, threads, cap_groups, keys.ctypes.data, states.ctypes.data, C.byref(groups), err,
                             512)
    if rc:
        raise OracleError(rc, err.value.decode())
    g = groups.value
    return keys[:g], states[:g]


def numbers_project(total, outs, pred=None, threads=0, native=False):
    """Filter -> Projection over numbers_mt(total): outs = [fq_expr or None].
    Returns (kept rows, [wrapping sum of each output's value bits])."""
    L = lib(native)
    n = len(outs)
    ex = (abi.fq_expr * n)(*[(e if e is not None else _identity(abi.DT_UINT64)) for e in outs])
    kept = C.c_uint64(0)
    sums = (C.c_uint64 * n)()
    err = C.create_string_buffer(512)
    rc = L.fqo_numbers_project(total, C.byref(pred) if pred is not None else None, n, ex, threads, C.byref(kept),
                               sums, err, 512)
    if rc:
        raise OracleError(rc, err.value.decode())
    return kept.value, list(sums)


# ---------------------------------------------------------------------------
# AggregateFinal merge (DataValue semantics)
# ---------------------------------------------------------------------------
def _f(bits):
    return struct.unpack("<d", struct.pack("<Q", bits))[0]


def _b(f):
    return struct.unpack("<Q", struct.pack("<d", f))[0]


def merge_states(op, states):
    """AggregatorFunction::merge_state over partial states in order.
    Returns an fqo_state-like tuple (kind, dtype, bits) or raises OracleError."""
    kind, dtype, bits = FQO_NULL, abi.DT_NULL, 0
    for s in states:
        if op in (abi.AGG_SUM, abi.AGG_COUNT):
            # data_value_arithmetic_op(Add, state, val)
            if kind == FQO_NULL:
                kind, dtype, bits = s.kind, s.dtype, s.bits
                continue
            if s.kind == FQO_NULL:
                continue
            if kind == FQO_NONE or s.kind == FQO_NONE:
                raise OracleError(abi.FQ_E_INTERNAL,
                                  "Internal Error: DataValue to array cannot be NONE NULL")
            if dtype == abi.DT_FLOAT64:
                bits = _b(_f(bits) + _f(s.bits))
            else:
                bits = (bits + s.bits) & 0xFFFFFFFFFFFFFFFF
        else:
            if kind == FQO_NULL:
                kind, dtype, bits = s.kind, s.dtype, s.bits
                continue
            if s.kind in (FQO_NULL, FQO_NONE):
                continue
            if kind == FQO_NONE:
                kind, bits = s.kind, s.bits
                continue
            a, b = bits, s.bits
            if dtype == abi.DT_FLOAT64:
                x, y = _f(a), _f(b)
                take = (x != x) or (y == y and (y > x if op == abi.AGG_MAX else y < x))
            elif dtype == abi.DT_INT64:
                sa = a - (1 << 64) if a >> 63 else a
                sb = b - (1 << 64) if b >> 63 else b
                take = sb > sa if op == abi.AGG_MAX else sb < sa
            else:
                take = b > a if op == abi.AGG_MAX else b < a
            if take:
                bits = b
    return kind, dtype, bits


def numbers_query(total, aggs, pred=None, src=SRC_NUMBERS, seed=0, threads=0):
    """Full Source -> Filter -> AggregatePartial x P -> Merge -> AggregateFinal
    for a list of single aggregators.  Returns [(kind, dtype, value)] or raises."""
    rows, st, err = numbers_partial(total, aggs, pred, src, seed, threads=threads)
    for s in st:
        if s:
            raise OracleError(s, err)
    out = []
    for a, (op, _) in enumerate(aggs):
        kind, dt, bits = merge_states(op, [r[a] for r in rows])
        out.append((kind, dt, bits))
    return out
