"""The reference's Function API over the C ABI's Function handles
(include/fq_engine.h "Function handles"; src/functions/function.rs:28-131).

    FieldFunction.try_create("a")                      function_field.rs:20-25
    ConstantFunction.try_create(DataValue("Int8", 1))  function_constant.rs:18-20
    ArithmeticFunction.try_create("+", [l, r])         function_arithmetic.rs:24-34
    ComparisonFunction.try_create("<", [l, r])         function_comparison.rs
    AggregatorFunction.try_create("sum", [arg])        function_aggregator.rs:24-36
    ScalarFunctionFactory.get(name, args)              function_factory.rs:14-40

A Function is a handle to the engine's C++ object: eval/accumulate run on the
engine's GPU (there is no CPU path), accumulate_result/merge_state/
merge_result are the host-side state protocol.  DataValue mirrors
data_value.rs:20-38: DataValue(type, value) with value None for `X(None)`,
and DataValue.NULL for the untyped DataValue::Null.  Errors raise FQError
with the reference's display text.
"""
import ctypes as C

from . import abi
from ._lib import FQError, check, lib
from .engine import Engine
from .expr import from_bits, to_bits

OPT = C.c_void_p
P = C.POINTER

SCALAR_NULL, SCALAR_NONE, SCALAR_SOME = 0, 1, 2


class fq_scalar(C.Structure):
    # str is a raw address: Utf8 payloads carry str_len and may hold NUL bytes
    # (a c_char_p field would hand back a copy cut at the first NUL)
    _fields_ = [("kind", C.c_int32), ("dtype", C.c_int32), ("bits", C.c_uint64), ("str", C.c_void_p),
                ("str_len", C.c_uint64)]


class fq_block(C.Structure):
    _fields_ = [("n_columns", C.c_int32), ("names", P(C.c_char_p)), ("columns", P(abi.fq_col)),
                ("block_rows", C.c_int64), ("filter", OPT)]


FUNCTION_SYMBOLS = [
    "fq_function_field", "fq_function_constant", "fq_function_create", "fq_function_clone", "fq_function_free",
    "fq_function_display", "fq_function_set_depth", "fq_function_return_type", "fq_function_nullable",
    "fq_function_eval", "fq_function_accumulate", "fq_function_accumulate_result", "fq_function_merge_state",
    "fq_function_merge_result", "fq_data_value_arithmetic_op", "fq_data_value_aggregate_op",
    "fq_functions_accumulate",
]

_protos = {
    "fq_function_field": (C.c_int32, [C.c_char_p, P(OPT)]),
    "fq_function_constant": (C.c_int32, [P(fq_scalar), P(OPT)]),
    "fq_function_create": (C.c_int32, [C.c_char_p, P(OPT), C.c_int32, P(OPT)]),
    "fq_function_clone": (C.c_int32, [OPT, P(OPT)]),
    "fq_function_free": (None, [OPT]),
    "fq_function_display": (C.c_int32, [OPT, C.c_char_p, C.c_size_t, P(C.c_size_t)]),
    "fq_function_set_depth": (C.c_int32, [OPT, C.c_uint64]),
    "fq_function_return_type": (C.c_int32, [OPT, P(fq_block), P(C.c_int32)]),
    "fq_function_nullable": (C.c_int32, [OPT, P(fq_block), P(C.c_int32)]),
    "fq_function_eval": (C.c_int32, [OPT, OPT, P(fq_block), C.c_void_p, C.c_size_t, P(C.c_size_t),
                                     P(C.c_int32), P(C.c_int64), P(C.c_int32), P(fq_scalar)]),
    "fq_function_accumulate": (C.c_int32, [OPT, OPT, P(fq_block)]),
    "fq_functions_accumulate": (C.c_int32, [OPT, P(OPT), C.c_int32, P(fq_block)]),
    "fq_function_accumulate_result": (C.c_int32, [OPT, P(fq_scalar), C.c_size_t, P(C.c_size_t)]),
    "fq_function_merge_state": (C.c_int32, [OPT, P(fq_scalar), C.c_size_t]),
    "fq_function_merge_result": (C.c_int32, [OPT, P(fq_scalar)]),
    "fq_data_value_arithmetic_op": (C.c_int32, [C.c_int32, P(fq_scalar), P(fq_scalar), P(fq_scalar)]),
    "fq_data_value_aggregate_op": (C.c_int32, [C.c_uint32, P(fq_scalar), P(fq_scalar), P(fq_scalar)]),
}
for _n, (_r, _a) in _protos.items():
    _f = getattr(lib, _n)
    _f.restype = _r
    _f.argtypes = _a


class DataValue:
    """data_value.rs:20-38: `type` is the DataType name ("Int64", "Utf8", ...),
    `value` the payload (None for X(None)); DataValue.NULL is DataValue::Null."""

    __slots__ = ("type", "value")

    def __init__(self, type_, value=None):
        self.type = type_
        self.value = value

    def is_null(self):
        return self.type == "Null"

    def __eq__(self, o):
        return isinstance(o, DataValue) and self.type == o.type and self.value == o.value

    def __hash__(self):
        return hash((self.type, self.value))

    def __repr__(self):
        if self.type == "Null":
            return "DataValue::Null"
        return "%s(%r)" % (self.type, self.value)

    def to_scalar(self):
        s = fq_scalar()
        if self.type == "Null":
            s.kind = SCALAR_NULL
            return s
        s.dtype = abi.DT_BY_NAME[self.type]
        if self.value is None:
            s.kind = SCALAR_NONE
            return s
        s.kind = SCALAR_SOME
        if s.dtype == abi.DT_UTF8:
            raw = self.value.encode()
            s._buf = C.create_string_buffer(raw, max(1, len(raw)))  # the scalar keeps its bytes alive
            s.str = C.addressof(s._buf)
            s.str_len = len(raw)
        else:
            s.bits = to_bits(self.value, s.dtype)
        return s

    @staticmethod
    def from_scalar(s):
        if s.kind == SCALAR_NULL:
            return DataValue.NULL
        name = abi.DT_NAMES[s.dtype]
        if s.kind == SCALAR_NONE:
            return DataValue(name, None)
        if s.dtype == abi.DT_UTF8:
            return DataValue(name, C.string_at(s.str, s.str_len).decode() if s.str_len else "")
        return DataValue(name, from_bits(s.bits, s.dtype))


DataValue.NULL = DataValue("Null", None)


def data_value_arithmetic_op(op, left, right):
    """data_value_arithmetic.rs:10-27 (op "+", "-", "*", "/")."""
    out = fq_scalar()
    check(lib.fq_data_value_arithmetic_op(abi.OP_BY_SYM[op], C.byref(left.to_scalar()), C.byref(right.to_scalar()),
                                          C.byref(out)))
    return DataValue.from_scalar(out)


def data_value_aggregate_op(op, left, right):
    """data_value_aggregate.rs:8-101 (op "min", "max", "sum", "count")."""
    out = fq_scalar()
    check(lib.fq_data_value_aggregate_op(abi.AGG_BY_NAME[op], C.byref(left.to_scalar()), C.byref(right.to_scalar()),
                                         C.byref(out)))
    return DataValue.from_scalar(out)


class DataBlock:
    """data_block.rs:10-62 over device columns: names -> ops.DeviceColumn.
    The columns stay owned by the caller (borrowed for each call).

    block_rows > 0: the columns hold the reference's blocks of that many rows
    (a numbers_mt partition of 10,000-row blocks) and accumulate replays the
    per-block state machine; filter: a pending FilterTransform (a Boolean
    Function) -- the block holds the rows where it is true, block by block."""

    def __init__(self, names, columns, block_rows=0, filter=None):
        assert len(names) == len(columns)
        self.names = list(names)
        self.columns = list(columns)
        self.block_rows = int(block_rows)
        self.filter = filter

    def num_rows(self):
        return self.columns[0].len if self.columns else 0

    def _abi(self):
        n = len(self.names)
        names = (C.c_char_p * max(n, 1))(*[s.encode() for s in self.names])
        cols = (abi.fq_col * max(n, 1))(*[c.col() if c.buf is not None else abi.fq_col(None, c.len, c.dtype, 0)
                                          for c in self.columns])
        b = fq_block(n, names, cols, self.block_rows, self.filter.h if self.filter is not None else None)
        b._keep = (names, cols, self.filter)
        return b


def _sync_torch():
    import torch

    if torch.cuda.is_initialized():
        torch.cuda.synchronize()


class Function:
    """A handle to one of the engine's Function objects."""

    def __init__(self, h):
        self.h = h

    def __del__(self):
        try:
            if self.h:
                lib.fq_function_free(self.h)
                self.h = None
        except Exception:  # interpreter shutdown
            pass

    def clone(self):
        out = OPT()
        check(lib.fq_function_clone(self.h, C.byref(out)))
        return Function(out)

    def __str__(self):
        n = C.c_size_t(0)
        lib.fq_function_display(self.h, None, 0, C.byref(n))
        buf = C.create_string_buffer(n.value + 1)
        check(lib.fq_function_display(self.h, buf, n.value + 1, C.byref(n)))
        return buf.value.decode()

    __repr__ = __str__

    def set_depth(self, depth):
        check(lib.fq_function_set_depth(self.h, depth))

    def return_type(self, block):
        out = C.c_int32()
        check(lib.fq_function_return_type(self.h, C.byref(block._abi()), C.byref(out)))
        return abi.DT_NAMES[out.value]

    def nullable(self, block):
        out = C.c_int32()
        check(lib.fq_function_nullable(self.h, C.byref(block._abi()), C.byref(out)))
        return bool(out.value)

    def eval(self, engine, block):
        """DataColumnarValue: an ops.DeviceColumn (array) or a DataValue (scalar)."""
        import torch

        from . import ops

        _sync_torch()  # the block's columns were written on torch's queue
        b = block._abi()
        nbytes, dt, ln, is_arr, sc = C.c_size_t(0), C.c_int32(0), C.c_int64(0), C.c_int32(0), fq_scalar()
        cap = max(8, ((block.num_rows() + 63) // 64) * 8, block.num_rows() * 8)
        out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        st = lib.fq_function_eval(engine.h, self.h, C.byref(b), C.c_void_p(out.data_ptr()), cap, C.byref(nbytes),
                                  C.byref(dt), C.byref(ln), C.byref(is_arr), C.byref(sc))
        check(st)
        if not is_arr.value:
            return DataValue.from_scalar(sc)
        return ops.DeviceColumn(out, ln.value, dt.value)

    def accumulate(self, engine, block):
        _sync_torch()
        check(lib.fq_function_accumulate(engine.h, self.h, C.byref(block._abi())))

    @staticmethod
    def accumulate_all(engine, funcs, block):
        """transform_aggregate_partial.rs:53-58 for one block -- every function's
        accumulate -- through fq_functions_accumulate: the aggregators sharing an
        argument (and the block's filter) read the column once."""
        _sync_torch()
        arr = (OPT * max(1, len(funcs)))(*[f.h for f in funcs])
        check(lib.fq_functions_accumulate(engine.h, arr, len(funcs), C.byref(block._abi())))

    def accumulate_result(self):
        n = C.c_size_t(0)
        st = lib.fq_function_accumulate_result(self.h, None, 0, C.byref(n))
        if st != abi.FQ_E_INVALID or n.value == 0:
            check(st)
        arr = (fq_scalar * max(1, n.value))()
        check(lib.fq_function_accumulate_result(self.h, arr, n.value, C.byref(n)))
        return [DataValue.from_scalar(arr[i]) for i in range(n.value)]

    def merge_state(self, states):
        scalars = [s.to_scalar() for s in states]  # they own the Utf8 bytes the array points at
        arr = (fq_scalar * max(1, len(states)))(*scalars)
        check(lib.fq_function_merge_state(self.h, arr, len(states)))
        del scalars

    def merge_result(self):
        out = fq_scalar()
        check(lib.fq_function_merge_result(self.h, C.byref(out)))
        return DataValue.from_scalar(out)


class ScalarFunctionFactory:
    @staticmethod
    def get(name, args):
        arr = (OPT * max(1, len(args)))(*[a.h for a in args])
        out = OPT()
        check(lib.fq_function_create(name.encode(), arr, len(args), C.byref(out)))
        return Function(out)


class FieldFunction:
    @staticmethod
    def try_create(name):
        out = OPT()
        check(lib.fq_function_field(name.encode(), C.byref(out)))
        return Function(out)


class ConstantFunction:
    @staticmethod
    def try_create(value):
        out = OPT()
        s = value.to_scalar()
        check(lib.fq_function_constant(C.byref(s), C.byref(out)))
        return Function(out)


class ArithmeticFunction:
    @staticmethod
    def try_create(op, args):
        return ScalarFunctionFactory.get(op, args)


class ComparisonFunction:
    @staticmethod
    def try_create(op, args):
        return ScalarFunctionFactory.get(op, args)


class AggregatorFunction:
    @staticmethod
    def try_create(op, args):
        return ScalarFunctionFactory.get(op, args)


__all__ = ["DataValue", "DataBlock", "Function", "FieldFunction", "ConstantFunction", "ArithmeticFunction",
           "ComparisonFunction", "AggregatorFunction", "ScalarFunctionFactory", "data_value_arithmetic_op",
           "data_value_aggregate_op", "FUNCTION_SYMBOLS", "FQError", "Engine"]
