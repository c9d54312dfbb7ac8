"""Python binding of include/fq_engine.h: run SQL through the C++ pipeline
(Source -> Filter -> AggregatePartial x P -> Merge -> AggregateFinal, or
Projection / Limit) on the gfx950 kernels.

    with Engine() as e:
        r = e.execute("SELECT sum(number)/count(number), max(number), min(number) "
                      "FROM system.numbers_mt(10000000000)")
        r.names  -> ['Sum(number) / Count(number)', 'Max(number)', 'Min(number)']
        r.rows   -> [(1310651184, 9999999999, 0)]
"""
import ctypes as C
import gc

import numpy as np

from . import abi
from ._lib import FQError, check, last_error, lib
from .expr import from_bits

P = C.POINTER

OPT_WORKER_THREADS, OPT_MODULO, OPT_PROFILE, OPT_STREAMS, OPT_CHUNK_ROWS, OPT_GROUP_CHUNK_ROWS = 1, 2, 3, 4, 5, 6
OPT_FAULT_PIPE = 7  # testing: merged pipe k (1-based) fails its device-context setup
PROFILE_PAIRS, PROFILE_SPAN = 1, 2  # FQ_OPT_PROFILE values

ENGINE_SYMBOLS = [
    "fq_engine_create", "fq_engine_destroy", "fq_engine_set_option", "fq_engine_materialize_numbers",
    "fq_engine_release_numbers", "fq_engine_trim_memory", "fq_engine_execute", "fq_engine_explain", "fq_engine_execute_partial",
    "fq_engine_execute_final", "fq_engine_get_stats", "fq_engine_reset_stats", "fq_result_num_rows",
    "fq_result_num_columns", "fq_result_column_name", "fq_result_column_type", "fq_result_value",
    "fq_result_text", "fq_result_free", "fq_result_mysql_type", "fq_result_values", "fq_engine_partial_state_bytes",
    "fq_engine_execute_blocks", "fq_block_stream_next", "fq_block_stream_free", "fq_engine_execute_row",
]


class fq_engine_stats(C.Structure):
    _fields_ = [("scan_launches", C.c_uint64), ("scan_rows", C.c_uint64), ("scan_bytes", C.c_uint64),
                ("scan_ms", C.c_double), ("queries", C.c_uint64), ("plan_ms", C.c_double),
                ("exec_ms", C.c_double), ("first_launch_ms", C.c_double), ("partial_ms", C.c_double),
                ("exchange_ms", C.c_double), ("final_ms", C.c_double), ("exchanges", C.c_uint64),
                ("exchange_rounds", C.c_uint64), ("exchange_bytes", C.c_uint64),
                ("cached_block_bytes", C.c_uint64), ("cached_workspace_bytes", C.c_uint64),
                ("project_launches", C.c_uint64), ("project_rows", C.c_uint64), ("project_kept", C.c_uint64),
                ("project_bytes", C.c_uint64), ("project_ms", C.c_double), ("tail_ms", C.c_double),
                ("complete_ms", C.c_double)]


class fq_device_block(C.Structure):
    _fields_ = [("n_columns", C.c_int32), ("pipe", C.c_int32), ("names", P(C.c_char_p)), ("columns", P(abi.fq_col)),
                ("rows", C.c_int64), ("block_rows", C.c_int64), ("n_blocks", C.c_int64), ("d_counts", C.c_void_p)]


_protos = {
    "fq_engine_create": (C.c_int32, [C.c_int32, P(C.c_void_p)]),
    "fq_engine_destroy": (None, [C.c_void_p]),
    "fq_engine_set_option": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int64]),
    "fq_engine_materialize_numbers": (C.c_int32, [C.c_void_p, C.c_uint64, C.c_int32, C.c_int32]),
    "fq_engine_release_numbers": (C.c_int32, [C.c_void_p]),
    "fq_engine_trim_memory": (C.c_int32, [C.c_void_p]),
    "fq_engine_execute": (C.c_int32, [C.c_void_p, C.c_char_p, P(C.c_void_p)]),
    "fq_engine_execute_row": (C.c_int32, [C.c_void_p, C.c_char_p, P(abi.fq_value), C.c_int32, P(C.c_int32)]),
    "fq_engine_explain": (C.c_int32, [C.c_void_p, C.c_char_p, C.c_char_p, C.c_size_t, P(C.c_size_t)]),
    "fq_engine_execute_partial": (C.c_int32, [C.c_void_p, C.c_char_p, C.c_int32, C.c_int32, C.c_void_p,
                                              C.c_size_t, P(C.c_size_t)]),
    "fq_engine_execute_final": (C.c_int32, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_size_t, C.c_int32,
                                            P(C.c_void_p)]),
    "fq_engine_partial_state_bytes": (C.c_int32, [C.c_void_p, C.c_char_p, P(C.c_size_t)]),
    "fq_engine_get_stats": (C.c_int32, [C.c_void_p, P(fq_engine_stats)]),
    "fq_engine_execute_blocks": (C.c_int32, [C.c_void_p, C.c_char_p, C.c_int32, C.c_int32, P(C.c_void_p)]),
    "fq_block_stream_next": (C.c_int32, [C.c_void_p, P(fq_device_block), P(C.c_int32)]),
    "fq_block_stream_free": (None, [C.c_void_p]),
    "fq_engine_reset_stats": (C.c_int32, [C.c_void_p]),
    "fq_result_num_rows": (C.c_int64, [C.c_void_p]),
    "fq_result_num_columns": (C.c_int32, [C.c_void_p]),
    "fq_result_column_name": (C.c_char_p, [C.c_void_p, C.c_int32]),
    "fq_result_column_type": (C.c_int32, [C.c_void_p, C.c_int32]),
    "fq_result_value": (C.c_int32, [C.c_void_p, C.c_int64, C.c_int32, P(abi.fq_value)]),
    "fq_result_text": (C.c_char_p, [C.c_void_p, C.c_int64, C.c_int32]),
    "fq_result_values": (C.c_int32, [C.c_void_p, C.c_int32, P(abi.fq_value), C.c_int64]),
    "fq_result_free": (None, [C.c_void_p]),
    "fq_result_mysql_type": (C.c_int32, [C.c_void_p, C.c_int32, P(C.c_int32)]),
}
for _n, (_r, _a) in _protos.items():
    _f = getattr(lib, _n)
    _f.restype = _r
    _f.argtypes = _a


_VALUE_NP = np.dtype([("dtype", "<i4"), ("is_some", "<i4"), ("bits", "<u8")])


def _column_values(ptr, c, nrow):
    """One column of a result as Python values (None for NULL), fetched in
    one fq_result_values call (numpy conversion for long columns)."""
    if nrow == 0:
        return []
    arr = (abi.fq_value * nrow)()
    check(lib.fq_result_values(ptr, c, arr, nrow))
    if nrow <= 64:  # aggregate results: a plain loop beats numpy's setup cost
        return [from_bits(v.bits, v.dtype) if v.is_some else None for v in arr]
    a = np.frombuffer(arr, dtype=_VALUE_NP)
    dts = np.unique(a["dtype"])
    if len(dts) == 1 and bool(a["is_some"].all()):
        dt, bits = int(dts[0]), a["bits"]
        if dt in (abi.DT_FLOAT32, abi.DT_FLOAT64):
            return bits.view(np.float64).tolist()
        if dt in (abi.DT_INT8, abi.DT_INT16, abi.DT_INT32, abi.DT_INT64):
            return bits.view(np.int64).tolist()
        if dt == abi.DT_BOOLEAN:
            return (bits != 0).tolist()
        return bits.tolist()
    return [from_bits(int(b), int(d)) if s else None for d, s, b in zip(a["dtype"], a["is_some"], a["bits"])]


class Result:
    """A query result: column names/types as the reference names them and
    rows of Python values (None for NULL)."""

    def __init__(self, ptr):
        try:
            ncol = lib.fq_result_num_columns(ptr)
            nrow = lib.fq_result_num_rows(ptr)
            self.names = [lib.fq_result_column_name(ptr, c).decode() for c in range(ncol)]
            self.types = [lib.fq_result_column_type(ptr, c) for c in range(ncol)]
            cols = []
            for c in range(ncol):
                if self.types[c] == abi.DT_UTF8:
                    vals = []
                    for r in range(nrow):
                        t = lib.fq_result_text(ptr, r, c)
                        vals.append(t.decode() if t is not None else None)
                    cols.append(vals)
                    continue
                cols.append(_column_values(ptr, c, nrow))
            self.columns = cols
            # 1e5-row results: the cyclic GC would rescan the young tuples
            # over and over while they are built (5x the build itself)
            gc_was = gc.isenabled()
            if nrow > 10000:
                gc.disable()
            try:
                self.rows = list(zip(*cols)) if cols else [() for _ in range(nrow)]
            finally:
                if gc_was:
                    gc.enable()
            # what the reference's MySQL writer sends (mysql_stream.rs:21-84) is
            # read on first use (mysql_types / mysql_error), like the text form
            self._mysql = None
            # the text form is built on first use (the handle stays open until then)
            self._ptr, ptr = ptr, None
            self._text = None
        finally:
            if ptr is not None:
                lib.fq_result_free(ptr)

    def _mysql_info(self):
        if self._mysql is None:
            types, err = [], None
            for c in range(len(self.names)):
                t = C.c_int32(0)
                if lib.fq_result_mysql_type(self._handle(), c, C.byref(t)) != 0:
                    err = last_error()
                    break
                types.append(t.value)
            self._mysql = (types, err)
        return self._mysql

    @property
    def mysql_types(self):
        """Column types the reference's MySQL writer declares (mysql_stream.rs:30-62)."""
        return self._mysql_info()[0]

    @property
    def mysql_error(self):
        """The error that writer raises for this result, or None."""
        return self._mysql_info()[1]

    def _handle(self):
        if self._ptr is None:
            raise RuntimeError("result handle already released")
        return self._ptr

    @property
    def text_rows(self):
        """Every value as arrow's array_value_to_string (fq_result_text)."""
        if self._text is None:
            ncol, nrow = len(self.names), len(self.rows)
            self._text = [tuple((lambda t: t.decode() if t is not None else None)(lib.fq_result_text(self._ptr, r, c))
                                for c in range(ncol)) for r in range(nrow)]
            self._mysql_info()  # everything read from the handle before it goes
            self._free()
        return self._text

    def _free(self):
        if getattr(self, "_ptr", None) is not None:
            lib.fq_result_free(self._ptr)
            self._ptr = None

    def __del__(self):
        try:
            self._free()
        except Exception:  # interpreter shutdown
            pass

    def __repr__(self):
        return "Result(names=%r, rows=%r)" % (self.names, self.rows[:10])


class BlockStream:
    """fq_engine_execute_blocks: a row pipeline's output as device DataBlocks
    (include/fq_engine.h).  Iterating yields fq_device_block structs; each is
    valid until the next one is pulled (or the stream is closed)."""

    def __init__(self, engine, sql, rank=0, world=1):
        h = C.c_void_p()
        check(lib.fq_engine_execute_blocks(engine.h, sql.encode(), rank, world, C.byref(h)))
        self.h = h
        self.engine = engine
        engine._streams.add(self)  # Engine.close() closes the streams still open

    def next(self):
        """The next fq_device_block, or None at the end."""
        b, has = fq_device_block(), C.c_int32(0)
        check(lib.fq_block_stream_next(self.h, C.byref(b), C.byref(has)))
        return b if has.value else None

    def __iter__(self):
        while True:
            b = self.next()
            if b is None:
                return
            yield b

    def close(self):
        if getattr(self, "h", None):
            lib.fq_block_stream_free(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine:
    def __init__(self, device=0, worker_threads=8, modulo=True, profile=False, streams=1):
        import weakref
        self._streams = weakref.WeakSet()  # open BlockStreams
        h = C.c_void_p()
        check(lib.fq_engine_create(device, C.byref(h)))
        self.h = h
        self.set_option(OPT_WORKER_THREADS, worker_threads)
        self.set_option(OPT_MODULO, 1 if modulo else 0)
        # profile: False / True (= 1, an event pair per scan launch) / PROFILE_SPAN
        # (= 2, one span from a query's first scan to its last, fq_engine.h)
        self.set_option(OPT_PROFILE, int(profile))
        self.set_option(OPT_STREAMS, streams)

    def set_option(self, opt, value):
        check(lib.fq_engine_set_option(self.h, opt, int(value)))

    def close(self):
        if getattr(self, "h", None):
            for st in list(getattr(self, "_streams", ())):  # before the engine they run on
                st.close()
            lib.fq_engine_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def materialize_numbers(self, total, rank=0, world=1):
        check(lib.fq_engine_materialize_numbers(self.h, int(total), rank, world))

    def release_numbers(self):
        check(lib.fq_engine_release_numbers(self.h))

    def trim_memory(self):
        """fq_engine_trim_memory: idle cached device blocks back to the driver."""
        check(lib.fq_engine_trim_memory(self.h))

    def execute(self, sql):
        out = C.c_void_p()
        check(lib.fq_engine_execute(self.h, sql.encode(), C.byref(out)))
        return Result(out)

    def execute_row(self, sql, cap=16):
        """fq_engine_execute_row: a one-row statement's values (fq_value list)."""
        row = (abi.fq_value * cap)()
        n = C.c_int32(0)
        check(lib.fq_engine_execute_row(self.h, sql.encode() if isinstance(sql, str) else sql, row, cap, C.byref(n)))
        return [row[i] for i in range(min(n.value, cap))]

    def execute_blocks(self, sql, rank=0, world=1):
        """The row pipeline's output blocks, left in HBM (BlockStream); rank of
        world: this rank's numbers_mt partitions only."""
        return BlockStream(self, sql, rank, world)

    def explain(self, sql):
        n = C.c_size_t(0)
        check(lib.fq_engine_explain(self.h, sql.encode(), None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value + 1)
        check(lib.fq_engine_explain(self.h, sql.encode(), buf, n.value + 1, C.byref(n)))
        return buf.value.decode()

    def execute_partial(self, sql, rank, world):
        """Serialised merged partial states of this rank's shard (bytes)."""
        n = C.c_size_t(0)
        # one reusable buffer (a fresh 1 MB buffer per step would be zero-filled
        # inside the timed loop of a multi-GPU bench)
        buf = getattr(self, "_pbuf", None)
        if buf is None:
            buf = self._pbuf = C.create_string_buffer(1 << 16)
        while True:
            cap = len(buf)
            st = lib.fq_engine_execute_partial(self.h, sql.encode(), rank, world, buf, cap, C.byref(n))
            if st == abi.FQ_E_INVALID and n.value > cap:
                buf = self._pbuf = C.create_string_buffer(n.value)
                continue
            check(st)
            return C.string_at(buf, n.value)

    def partial_state_bytes(self, sql):
        """fq_engine_partial_state_bytes: the partial states' size on every rank
        (0 when it depends on the data, GROUP BY)."""
        n = C.c_size_t(0)
        check(lib.fq_engine_partial_state_bytes(self.h, sql.encode(), C.byref(n)))
        return n.value

    def execute_final(self, sql, states, stride=None):
        """AggregateFinal over per-rank serialised states (list of bytes, rank order)."""
        stride = stride or max(len(s) for s in states)
        blob = b"".join(s.ljust(stride, b"\0") for s in states)
        out = C.c_void_p()
        check(lib.fq_engine_execute_final(self.h, sql.encode(), blob, stride, len(states), C.byref(out)))
        return Result(out)

    def stats(self):
        s = fq_engine_stats()
        check(lib.fq_engine_get_stats(self.h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in fq_engine_stats._fields_}

    def reset_stats(self):
        check(lib.fq_engine_reset_stats(self.h))


__all__ = ["Engine", "Result", "BlockStream", "FQError", "last_error", "ENGINE_SYMBOLS"]
