"""Tensor-level wrappers over the C ABI of include/fq_gpu.h.

PyTorch only provides device memory and the current HIP stream here; every
computation is one of the library's gfx950 kernels.  All functions raise
FQError (status + the reference's error text) on failure, and raise
immediately when no GPU is present -- there is no CPU fallback.
"""
import ctypes as C

import numpy as np
import torch

from . import abi
from ._lib import FQError, check, last_error, lib  # noqa: F401
from .expr import from_bits, to_bits

NP_DTYPES = {
    abi.DT_INT8: np.int8, abi.DT_INT16: np.int16, abi.DT_INT32: np.int32,
    abi.DT_INT64: np.int64, abi.DT_UINT8: np.uint8, abi.DT_UINT16: np.uint16,
    abi.DT_UINT32: np.uint32, abi.DT_UINT64: np.uint64, abi.DT_FLOAT32: np.float32,
    abi.DT_FLOAT64: np.float64,
}
DT_OF_NP = {np.dtype(v): k for k, v in NP_DTYPES.items()}
ELEM_SIZE = {k: np.dtype(v).itemsize for k, v in NP_DTYPES.items()}


def require_gpu():
    if not torch.cuda.is_available():
        raise FQError(abi.FQ_E_HIP, "fq_amd: no GPU visible (the device path has no CPU fallback)")


def _stream(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


class DeviceColumn:
    """An Arrow-layout column in HBM (values buffer, no nulls).  Boolean
    columns are LSB-first bitmaps in uint64 words."""

    def __init__(self, buf, length, dtype, offset=0):
        self.buf = buf  # torch uint8 tensor owning the bytes
        self.len = int(length)
        self.dtype = dtype
        self.offset = offset

    @property
    def ptr(self):
        return self.buf.data_ptr() + self.offset

    def col(self):
        return abi.fq_col(C.c_void_p(self.ptr), self.len, self.dtype, 0)

    def nbytes(self):
        if self.dtype == abi.DT_BOOLEAN:
            return ((self.len + 63) // 64) * 8
        return self.len * ELEM_SIZE[self.dtype]

    def to_numpy(self):
        nb = self.nbytes()
        host = self.buf[self.offset:self.offset + nb].cpu().numpy()
        if self.dtype == abi.DT_BOOLEAN:
            words = host.view(np.uint64)
            bits = np.unpackbits(words.view(np.uint8), bitorder="little")
            return bits[: self.len].astype(bool)
        return host.view(NP_DTYPES[self.dtype]).copy()


def empty_column(n, dtype, device=None):
    require_gpu()
    nb = ((n + 63) // 64) * 8 if dtype == abi.DT_BOOLEAN else n * ELEM_SIZE[dtype]
    buf = torch.empty(max(nb, 16), dtype=torch.uint8, device=device or "cuda")
    return DeviceColumn(buf, n, dtype)


class _RawDevice:
    """A device allocation presented to torch through __cuda_array_interface__."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 2}


_hip = None


def contiguous_column(n, dtype):
    """A column in physically contiguous HBM (hipExtMallocWithFlags with
    hipDeviceMallocContiguous), freed with its tensor.  Output buffers of the
    block-stream Filter -> Projection run faster more often in such memory
    (profiles/r03_s3_output_placement.txt); the kernels accept any device memory."""
    global _hip
    require_gpu()
    import weakref
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so.7")  # torch's HIP runtime, already loaded (see _lib._load)
        _hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
        _hip.hipFree.argtypes = [C.c_void_p]
    nb = max(((n + 63) // 64) * 8 if dtype == abi.DT_BOOLEAN else n * ELEM_SIZE[dtype], 16)
    p = C.c_void_p()
    rc = _hip.hipExtMallocWithFlags(C.byref(p), nb, 0x4)  # hipDeviceMallocContiguous
    if rc != 0:
        raise FQError(abi.FQ_E_HIP, "hipExtMallocWithFlags(hipDeviceMallocContiguous, %d bytes) failed: %d" % (nb, rc))
    buf = torch.as_tensor(_RawDevice(p.value, nb), device="cuda")
    fin = weakref.finalize(buf, _hip.hipFree, C.c_void_p(p.value))
    fin.atexit = False  # never call into HIP during interpreter shutdown; process exit releases it
    return DeviceColumn(buf, n, dtype)


def device_view(ptr, nbytes):
    """A torch uint8 tensor over device memory the library owns (no copy, not
    freed by torch): e.g. a block of fq_engine_execute_blocks."""
    require_gpu()
    return torch.as_tensor(_RawDevice(int(ptr), max(int(nbytes), 1)), device="cuda")


def device_block_to_numpy(b):
    """An fq_device_block's columns as numpy, one list of per-block arrays per
    column (block-stream layout) or one array per column (plain)."""
    cols = [b.columns[j] for j in range(b.n_columns)]
    if b.block_rows > 0:
        counts = device_view(b.d_counts, 8 * b.n_blocks).cpu().numpy().view(np.int64).copy() if b.n_blocks else \
            np.zeros(0, np.int64)
    out = []
    for c in cols:
        h = device_view(c.data, c.len * ELEM_SIZE[c.dtype]).cpu().numpy().view(NP_DTYPES[c.dtype]).copy() \
            if c.len else np.zeros(0, NP_DTYPES[c.dtype])
        if b.block_rows > 0:
            out.append([h[k * b.block_rows: k * b.block_rows + int(n)] for k, n in enumerate(counts)])
        else:
            out.append(h[:b.rows])
    return out


def from_numpy(arr, dtype=None):
    require_gpu()
    arr = np.ascontiguousarray(arr)
    dt = dtype if dtype is not None else DT_OF_NP[arr.dtype]
    raw = arr.view(np.uint8).reshape(-1) if arr.size else np.zeros(16, np.uint8)
    buf = torch.from_numpy(raw.copy()).to("cuda")
    return DeviceColumn(buf, arr.shape[0], dt)


def numbers_column(begin, count, stream=None):
    """SourceTransform of one numbers_mt range: [begin, begin+count)."""
    c = empty_column(count, abi.DT_UINT64)
    check(lib.fq_fill_numbers_u64(C.c_void_p(c.ptr), begin, count, _stream(stream)))
    return c


def splitmix_column(seed, first_index, count, stream=None):
    c = empty_column(count, abi.DT_UINT64)
    check(lib.fq_fill_splitmix64(C.c_void_p(c.ptr), seed, first_index, count, _stream(stream)))
    return c


class Workspace:
    def __init__(self, nbytes):
        require_gpu()
        self.buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device="cuda")
        self.nbytes = self.buf.numel()

    @property
    def ptr(self):
        return C.c_void_p(self.buf.data_ptr())


def aggregate_async(col, block_rows=0, pred=None, value=None, mask=0xF, ws=None, out=None,
                    stream=None):
    """Launch fq_aggregate; returns the device tensor holding the fq_agg_state."""
    require_gpu()
    ws = ws or Workspace(lib.fq_aggregate_workspace_bytes(col.len))
    if out is None:
        out = torch.empty(48, dtype=torch.uint8, device="cuda")
    c = col.col()
    check(lib.fq_aggregate(C.byref(c), block_rows, C.byref(pred) if pred is not None else None,
                           C.byref(value) if value is not None else None, mask,
                           C.c_void_p(out.data_ptr()), ws.ptr, ws.nbytes, _stream(stream)))
    return out


def state_from_device(t):
    raw = t.cpu().numpy().tobytes()
    return abi.fq_agg_state.from_buffer_copy(raw)


def aggregate(col, block_rows=0, pred=None, value=None, mask=0xF, ws=None, stream=None):
    """Fused AggregatePartial over one device block -> host fq_agg_state."""
    t = aggregate_async(col, block_rows, pred, value, mask, ws, None, stream)
    return state_from_device(t)


def state_values(st):
    """fq_agg_state -> dict(sum, max, min, count, blocks, flags) of Python values."""
    dt = st.dtype
    return {
        "sum": from_bits(st.sum, dt), "max": from_bits(st.max, dt),
        "min": from_bits(st.min, dt), "count": st.count, "blocks": st.blocks,
        "flags": st.flags, "dtype": dt,
    }


def _side(x):
    """DeviceColumn -> (fq_col, None); python scalar / (value, dtype) -> (None, fq_value)."""
    if isinstance(x, DeviceColumn):
        return x.col(), None
    if isinstance(x, abi.fq_value):
        return None, x
    from .expr import literal
    val, dt = literal(x)
    if val is None:
        return None, abi.fq_value(dt, 0, 0)
    return None, abi.fq_value(dt, 1, to_bits(val, dt))


def arith(op_sym, lhs, rhs, stream=None):
    """ArithmeticFunction::eval on device columns / scalars -> DeviceColumn."""
    require_gpu()
    lc, ls = _side(lhs)
    rc, rs = _side(rhs)
    ldt = lc.dtype if lc is not None else ls.dtype
    rdt = rc.dtype if rc is not None else rs.dtype
    out_dt = C.c_int32(0)
    check(lib.fq_arith_result_type(abi.OP_BY_SYM[op_sym], ldt, rdt, C.byref(out_dt)))
    n = lc.len if lc is not None else (rc.len if rc is not None else 1)
    out = empty_column(n, out_dt.value)
    oc = out.col()
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    check(lib.fq_arith(abi.OP_BY_SYM[op_sym], C.byref(lc) if lc is not None else None,
                       C.byref(ls) if ls is not None else None, C.byref(rc) if rc is not None else None,
                       C.byref(rs) if rs is not None else None, C.byref(oc),
                       C.c_void_p(flag.data_ptr()), _stream(stream)))
    return out


def compare(cmp_sym, lhs, rhs, stream=None):
    """ComparisonFunction::eval -> Boolean DeviceColumn (LSB-first bitmap)."""
    require_gpu()
    lc, ls = _side(lhs)
    rc, rs = _side(rhs)
    n = lc.len if lc is not None else (rc.len if rc is not None else 1)
    out = empty_column(n, abi.DT_BOOLEAN)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    check(lib.fq_compare(abi.CMP_BY_SYM[cmp_sym], C.byref(lc) if lc is not None else None,
                         C.byref(ls) if ls is not None else None,
                         C.byref(rc) if rc is not None else None,
                         C.byref(rs) if rs is not None else None, C.c_void_p(out.ptr), n,
                         C.c_void_p(flag.data_ptr()), _stream(stream)))
    return out


def logic(op, lhs, rhs, stream=None):
    """LogicFunction::eval: 'and' / 'or' of two Boolean DeviceColumns."""
    require_gpu()
    out = empty_column(lhs.len, abi.DT_BOOLEAN)
    check(lib.fq_logic(0 if op == "and" else 1, C.c_void_p(lhs.ptr), C.c_void_p(rhs.ptr), C.c_void_p(out.ptr),
                       lhs.len, _stream(stream)))
    return out


def filter_compact(col, bitmap, stream=None):
    """FilterTransform: keep rows whose bit is set, in order -> DeviceColumn."""
    require_gpu()
    out = empty_column(col.len, col.dtype)
    ws = Workspace(lib.fq_filter_workspace_bytes(col.len))
    n = C.c_int64(0)
    c = col.col()
    check(lib.fq_filter_compact(C.byref(c), C.c_void_p(bitmap.ptr), C.c_void_p(out.ptr), C.byref(n),
                                ws.ptr, ws.nbytes, _stream(stream)))
    out.len = n.value
    return out


def filter_project(col, pred, values, stream=None):
    """FilterTransform -> ProjectionTransform fused (fq_filter_project): the
    kept rows of `col` (pred None = all) through each fq_expr of `values`
    (None = the column itself) -> [DeviceColumn] in row order."""
    require_gpu()
    n_out = len(values)
    exprs = (abi.fq_expr * n_out)()
    outs = []
    for j, v in enumerate(values):
        if v is None:
            v = abi.fq_expr()
            v.n_steps = 0
            v.out_dtype = col.dtype
        exprs[j] = v
        outs.append(empty_column(col.len, v.out_dtype))
    ptrs = (C.c_void_p * max(n_out, 1))(*[o.ptr for o in outs])
    ws = Workspace(lib.fq_filter_project_workspace_bytes(col.len))
    n = C.c_int64(0)
    c = col.col()
    check(lib.fq_filter_project(C.byref(c), C.byref(pred) if pred is not None else None, exprs, n_out, ptrs,
                                C.byref(n), ws.ptr, ws.nbytes, _stream(stream)))
    for o in outs:
        o.len = n.value
    return outs


def filter_project_blocks(col, block_rows, pred, values, stream=None, out_offset=0):
    """FilterTransform -> ProjectionTransform over a stream of DataBlocks of
    block_rows rows (fq_filter_project_blocks): -> ([DeviceColumn of col.len
    rows per output], per-block kept counts as an int64 numpy array).  Block
    b's kept rows are rows [b * block_rows, + counts[b]) of each output.
    out_offset: each output a view that many 8-byte rows into its buffer
    (tests: outputs not 16-byte aligned)."""
    require_gpu()
    n_out = len(values)
    exprs = (abi.fq_expr * n_out)()
    outs = []
    for j, v in enumerate(values):
        if v is None:
            v = abi.fq_expr()
            v.n_steps = 0
            v.out_dtype = col.dtype
        exprs[j] = v
        if out_offset:
            full = empty_column(col.len + out_offset, v.out_dtype)
            outs.append(DeviceColumn(full.buf, col.len, v.out_dtype, offset=8 * out_offset))
        else:
            outs.append(empty_column(col.len, v.out_dtype))
    ptrs = (C.c_void_p * max(n_out, 1))(*[o.ptr for o in outs])
    nb =(1 if block_rows >= col.len else -(-col.len // block_rows)) if block_rows > 0 and col.len > 0 else 0
    counts = Workspace(max(8 * nb, 8))
    ws = Workspace(lib.fq_filter_project_blocks_workspace_bytes())
    n = C.c_int64(0)
    c = col.col()
    check(lib.fq_filter_project_blocks(C.byref(c), block_rows, C.byref(pred) if pred is not None else None, exprs,
                                       n_out, ptrs, counts.ptr, C.byref(n), ws.ptr, ws.nbytes, _stream(stream)))
    cnt = counts.buf[:8 * nb].view(torch.int64).cpu().numpy() if nb else np.zeros(0, np.int64)
    assert int(cnt.sum()) == n.value
    return outs, cnt


def predicate_bitmap(col, pred, stream=None):
    """FilterTransform's predicate as a Boolean column (fq_predicate_bitmap)."""
    require_gpu()
    out = empty_column(col.len, abi.DT_BOOLEAN)
    flag = Workspace(4)
    c = col.col()
    check(lib.fq_predicate_bitmap(C.byref(c), C.byref(pred), C.c_void_p(out.ptr), flag.ptr, _stream(stream)))
    return out


def project_compile_check(col_dtype, pred=None, values=(None,)):
    """Generate + compile the fused projection module for this shape without
    running it (no GPU needed: gfx950 code object only).  Returns the
    fq_status of fq_filter_project on a fake column (FQ_E_HIP when there is no
    device after a successful compile)."""
    exprs = (abi.fq_expr * len(values))()
    for j, v in enumerate(values):
        if v is None:
            v = abi.fq_expr()
            v.out_dtype = col_dtype
        exprs[j] = v
    fake = (C.c_void_p * len(values))(*([C.c_void_p(256)] * len(values)))
    c = abi.fq_col(C.c_void_p(256), 1 << 20, col_dtype, 0)
    n = C.c_int64(0)
    return lib.fq_filter_project(C.byref(c), C.byref(pred) if pred is not None else None, exprs, len(values), fake,
                                 C.byref(n), C.c_void_p(256), lib.fq_filter_project_workspace_bytes(1 << 20), None)


def state_merge(states):
    arr = (abi.fq_agg_state * len(states))(*states)
    out = abi.fq_agg_state()
    check(lib.fq_state_merge(arr, len(states), C.byref(out)))
    return out


# ---- expression specialisation (include/fq_gpu.h fq_jit_*) ----
def jit_config(mode, min_rows=1 << 22):
    """Process-wide JIT policy: abi.JIT_OFF / JIT_AUTO / JIT_ALWAYS."""
    check(lib.fq_jit_config(mode, int(min_rows)))


def jit_stats():
    st = abi.fq_jit_stats()
    check(lib.fq_jit_get_stats(C.byref(st)))
    return {f: getattr(st, f) for f, _ in abi.fq_jit_stats._fields_}


def jit_prepare(dtype, pred=None, value=None, mask=abi.AGG_SUM, block_rows=0, length=1 << 30):
    """Compile the specialised scan for this shape ahead of time (works
    without a GPU: the source is then only compiled for gfx950).  Returns
    True if the shape has a specialised kernel."""
    c = abi.fq_col(None, int(length), dtype, 0)
    out = C.c_int32(0)
    check(lib.fq_jit_prepare(C.byref(c), int(block_rows), C.byref(pred) if pred is not None else None,
                             C.byref(value) if value is not None else None, mask, C.byref(out)))
    return bool(out.value)


# ---- GROUP BY hash aggregation (include/fq_gpu.h fq_group_*) ----
class GroupTable:
    """A device hash table of groups: key -> one 64-bit state per aggregate.
    aggs: [(abi.AGG_*, state dtype)]; Count's state dtype is UInt64."""

    def __init__(self, capacity, aggs, key_dtype=abi.DT_UINT64, stream=None):
        require_gpu()
        cap = 64
        while cap < capacity:
            cap *= 2
        self.desc = abi.fq_group_table()
        self.desc.capacity = cap
        self.desc.key_dtype = key_dtype
        self.desc.n_aggs = len(aggs)
        for i, (k, dt) in enumerate(aggs):
            self.desc.kinds[i] = k
            self.desc.dtypes[i] = dt
        self.buf = torch.empty(lib.fq_group_table_bytes(cap, len(aggs)), dtype=torch.uint8, device="cuda")
        self.desc.d_mem = self.buf.data_ptr()
        self.aggs = list(aggs)
        check(lib.fq_group_table_init(C.byref(self.desc), _stream(stream)))

    def aggregate(self, col, pred=None, key=None, values=None, stream=None, log2_parts=0, narrow=False):
        """fq_group_aggregate, or with log2_parts > 0 the radix-partitioned
        fq_group_aggregate_partitioned (2^log2_parts bins; narrow: the caller
        vouches every value lies within 2^31 of the first, FQ_GROUP_NARROW_ROWS)."""
        c = col.col()
        vals = (abi.fq_expr * abi.MAX_GROUP_AGGS)()
        for i, v in enumerate(values or []):
            if v is not None:
                vals[i] = v
        p = C.byref(pred) if pred is not None else None
        k = C.byref(key) if key is not None else None
        if not log2_parts:
            check(lib.fq_group_aggregate(C.byref(self.desc), C.byref(c), p, k, vals, _stream(stream)))
            return
        ws = Workspace(lib.fq_group_partition_workspace_bytes(col.len, log2_parts))
        lp = log2_parts | (abi.GROUP_NARROW_ROWS if narrow else 0)
        check(lib.fq_group_aggregate_partitioned(C.byref(self.desc), C.byref(c), p, k, vals, lp, ws.ptr,
                                                 ws.nbytes, _stream(stream)))
        self._ws = ws  # alive until the next call (the launch is asynchronous)

    def merge(self, keys, states, stream=None):
        """fq_group_table_merge: host uint64 keys[n] and per-aggregate uint64
        states[n] (state bits) folded into this table."""
        n = len(keys)
        dk = torch.from_numpy(np.ascontiguousarray(keys, dtype=np.uint64).view(np.int64)).cuda()
        ds = [torch.from_numpy(np.ascontiguousarray(s, dtype=np.uint64).view(np.int64)).cuda() for s in states]
        ptrs = (C.c_void_p * max(len(ds), 1))(*[t.data_ptr() for t in ds])
        check(lib.fq_group_table_merge(C.byref(self.desc), C.c_void_p(dk.data_ptr()), ptrs, n, _stream(stream)))
        torch.cuda.synchronize()

    def count(self, stream=None):
        n = C.c_int64(0)
        check(lib.fq_group_table_count(C.byref(self.desc), C.byref(n), _stream(stream)))
        return n.value

    def extract(self, stream=None):
        """-> (keys uint64[g], [states uint64[g] per aggregate]) in slot order."""
        g = self.count(stream)
        n = max(g, 1)
        keys = torch.empty(n, dtype=torch.int64, device="cuda")
        sts = [torch.empty(n, dtype=torch.int64, device="cuda") for _ in self.aggs]
        ptrs = (C.c_void_p * len(sts))(*[t.data_ptr() for t in sts])
        out = C.c_int64(0)
        check(lib.fq_group_table_extract(C.byref(self.desc), C.c_void_p(keys.data_ptr()), ptrs, n, C.byref(out),
                                         _stream(stream)))
        k = keys[: out.value].cpu().numpy().view(np.uint64)
        return k, [t[: out.value].cpu().numpy().view(np.uint64) for t in sts]


def group_compile_check(col_dtype, aggs, key=None, values=None, pred=None, key_dtype=abi.DT_UINT64, log2_parts=0):
    """Generate + compile the group-by kernel for a shape (no GPU needed: a
    zero-length call compiles the source for gfx950 without loading it);
    log2_parts > 0 through fq_group_aggregate_partitioned (range bins for a
    `% d` key, else hash bins)."""
    d = abi.fq_group_table()
    d.d_mem = 0x1000  # never dereferenced for a zero-length column
    d.capacity = 64
    d.key_dtype = key_dtype
    d.n_aggs = len(aggs)
    for i, (k, dt) in enumerate(aggs):
        d.kinds[i] = k
        d.dtypes[i] = dt
    c = abi.fq_col(None, 0, col_dtype, 0)
    vals = (abi.fq_expr * abi.MAX_GROUP_AGGS)()
    for i, v in enumerate(values or []):
        if v is not None:
            vals[i] = v
    p = C.byref(pred) if pred is not None else None
    k = C.byref(key) if key is not None else None
    if log2_parts:
        check(lib.fq_group_aggregate_partitioned(C.byref(d), C.byref(c), p, k, vals, log2_parts, None, 0, None))
    else:
        check(lib.fq_group_aggregate(C.byref(d), C.byref(c), p, k, vals, None))


def tune_set(name, value):
    """fq_tune_set by knob name (abi.TUNE); tuning tools only."""
    check(lib.fq_tune_set(abi.TUNE[name], int(value)))


def tune_get(name):
    return int(lib.fq_tune_get(abi.TUNE[name]))


def tune_reset():
    check(lib.fq_tune_reset())


