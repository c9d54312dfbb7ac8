"""TEST INFRASTRUCTURE ONLY -- semantic CPU restatement of the reference's
hot path in numpy, for small inputs (the parity checker for expression trees
and error texts; oracle/fq_oracle.c is the fast one for the numbers_mt loop).
Never imported by the product package.

Restates (dantengsky/fuse-query, /root/reference):
  numerical_coercion / equal_coercion   src/datavalues/data_type.rs:27-98
  arrow cast (num-traits NumCast)       via data_array_arithmetic.rs:39-40
  data_array_arithmetic_op              src/datavalues/data_array_arithmetic.rs:14-55
  data_array_comparison_op              src/datavalues/data_array_comparison.rs:14-94
  data_array_aggregate_op               src/datavalues/data_array_aggregate.rs:14-163
  data_value_arithmetic_op              src/datavalues/data_value_arithmetic.rs:10-27
  data_value_aggregate_op               src/datavalues/data_value_aggregate.rs:8-101
  DataValue::to_array                   src/datavalues/data_value.rs:77-111
  Field/Constant/Alias/Arithmetic/Comparison/Aggregator functions
                                        src/functions/*.rs (depth rule: plan_expression.rs:40-75)
  numbers_mt partitions + blocks        src/datasources/system/numbers_{table,stream}.rs
  Filter / Projection / Limit / AggregatePartial / AggregateFinal
                                        src/transforms/*.rs, src/datastreams/stream_limit.rs
Pinned by tests/golden/reference_vectors.json (the reference's own test tables).
The '%' operator is this build's EXTENSION (the reference has no such function).
"""
import math

import numpy as np

NUMERIC = ["Int8", "Int16", "Int32", "Int64", "UInt8", "UInt16", "UInt32", "UInt64", "Float32", "Float64"]
NP = {"Int8": np.int8, "Int16": np.int16, "Int32": np.int32, "Int64": np.int64, "UInt8": np.uint8,
      "UInt16": np.uint16, "UInt32": np.uint32, "UInt64": np.uint64, "Float32": np.float32,
      "Float64": np.float64}
ORDER = ["Float64", "Float32", "Int64", "Int32", "Int16", "Int8", "UInt64", "UInt32", "UInt16", "UInt8"]
ARITH = {"+", "-", "*", "/", "%"}
CMP = {"=", "<", "<=", ">", ">="}
FLIP = {"=": "=", "<": ">", "<=": ">=", ">": "<", ">=": "<="}
AGG_DEBUG = {"min": "Min", "max": "Max", "sum": "Sum", "count": "Count"}


class RefError(Exception):
    """A FuseQueryError; str() is its Display text."""


def internal(msg):
    return RefError("Internal Error: " + msg)


def is_int(t):
    return t in NP and not t.startswith("Float")


def is_signed(t):
    return t.startswith("Int")


def int_range(t):
    info = np.iinfo(NP[t])
    return int(info.min), int(info.max)


# ---------------------------------------------------------------------------
# values and arrays
# ---------------------------------------------------------------------------
class Value:
    """DataValue: type 'Null' is DataValue::Null; value None is X(None)."""
    __slots__ = ("type", "value")

    def __init__(self, type_, value=None):
        self.type = type_
        self.value = value

    @staticmethod
    def null():
        return Value("Null", None)

    def is_untyped_null(self):
        return self.type == "Null"

    def __eq__(self, o):
        if not isinstance(o, Value) or self.type != o.type:
            return False
        if self.value is None or o.value is None:
            return self.value is None and o.value is None
        if isinstance(self.value, float) and math.isnan(self.value):
            return isinstance(o.value, float) and math.isnan(o.value)
        return self.value == o.value

    def __repr__(self):
        return "Value(%s, %r)" % (self.type, self.value)

    def debug(self):
        if self.type == "Null":
            return "Null"
        if self.value is None:
            return "NULL"
        if self.type == "Boolean":
            return "true" if self.value else "false"
        if self.type.startswith("Float"):
            return fmt_float(self.value, self.type == "Float32")
        return str(self.value)


def fmt_float(d, f32=False):
    if d != d:
        return "NaN"
    if math.isinf(d):
        return "inf" if d > 0 else "-inf"
    if d == 0:
        return "-0" if math.copysign(1, d) < 0 else "0"
    for p in range(1, 18):
        s = "%.*e" % (p - 1, d)
        back = float(s)
        if (np.float32(back) == np.float32(d)) if f32 else back == d:
            break
    neg = s.startswith("-")
    s = s.lstrip("-")
    mant, exp = s.split("e")
    exp = int(exp)
    digits = mant.replace(".", "").rstrip("0") or "0"
    n = len(digits)
    if exp < 0:
        out = "0." + "0" * (-exp - 1) + digits
    elif exp >= n - 1:
        out = digits + "0" * (exp - (n - 1))
    else:
        out = digits[: exp + 1] + "." + digits[exp + 1:]
    return ("-" if neg else "") + out


class Arr:
    """An arrow array restated: values (numpy for numerics, list otherwise)
    plus a validity mask (None = all valid)."""
    __slots__ = ("type", "values", "valid")

    def __init__(self, type_, values, valid=None):
        self.type = type_
        if type_ in NP:
            values = np.asarray(values, dtype=NP[type_])
        self.values = values
        self.valid = valid

    def __len__(self):
        return len(self.values)

    def is_valid(self, i):
        return self.valid is None or bool(self.valid[i])

    def get(self, i):
        if not self.is_valid(i):
            return Value(self.type, None)
        v = self.values[i]
        if self.type in NP:
            v = float(v) if self.type.startswith("Float") else int(v)
        elif self.type == "Boolean":
            v = bool(v)
        return Value(self.type, v)

    def to_list(self):
        return [self.get(i).value for i in range(len(self))]

    def take(self, mask):
        mask = np.asarray(mask, dtype=bool)
        if self.type in NP:
            vals = self.values[mask]
        else:
            vals = [v for v, m in zip(self.values, mask) if m]
        valid = None if self.valid is None else np.asarray(self.valid)[mask]
        return Arr(self.type, vals, valid)

    def slice(self, n):
        vals = self.values[:n]
        valid = None if self.valid is None else self.valid[:n]
        return Arr(self.type, vals, valid)


def to_array(v, size):
    """DataValue::to_array (data_value.rs:77-111)."""
    if v.type == "Null":
        return Arr("Null", [None] * size, np.zeros(size, bool))
    if v.value is None:
        raise internal("DataValue to array cannot be NONE NULL")
    if v.type in NP:
        return Arr(v.type, np.full(size, v.value, dtype=NP[v.type]))
    return Arr(v.type, [v.value] * size)


# ---------------------------------------------------------------------------
# coercion + cast
# ---------------------------------------------------------------------------
def numerical_coercion(op, l, r):
    if l not in NP or r not in NP:
        raise internal("Unsupported (%s) %s (%s)" % (l, op, r))
    if l == r:
        return l
    for t in ORDER:
        if l == t or r == t:
            return t
    raise internal("Unsupported (%s) %s (%s)" % (l, op, r))


def equal_coercion(op, l, r):
    if l == r:
        return l
    return numerical_coercion(op, l, r)


def cast(a, to):
    """arrow::compute::cast between numeric types: out-of-range -> null."""
    if a.type == to:
        return a
    if a.type not in NP or to not in NP:
        raise internal("cast %s -> %s not restated" % (a.type, to))
    src = a.values
    valid = np.ones(len(src), bool) if a.valid is None else np.asarray(a.valid).copy()
    if to.startswith("Float"):
        out = src.astype(NP[to])
    else:
        lo, hi = int_range(to)
        if a.type.startswith("Float"):
            with np.errstate(invalid="ignore"):
                t = np.trunc(src.astype(np.float64))
                ok = np.isfinite(t) & (t >= float(lo)) & (t < float(hi) + 1.0)
            t = np.where(ok, t, 0)
            out = t.astype(NP[to]) if not is_signed(to) else t.astype(np.int64).astype(NP[to])
        elif is_signed(a.type):
            s = src.astype(np.int64)
            ok = (s >= lo) & ((s < 0) | (s.astype(np.uint64) <= np.uint64(hi)))
            out = np.where(ok, s, 0).astype(NP[to])
        else:
            u = src.astype(np.uint64)
            ok = u <= np.uint64(hi)
            out = np.where(ok, u, 0).astype(NP[to])
        valid &= ok
    return Arr(to, out, None if valid.all() else valid)


def _both_valid(a, b):
    if a.valid is None and b.valid is None:
        return None
    va = np.ones(len(a), bool) if a.valid is None else a.valid
    vb = np.ones(len(b), bool) if b.valid is None else b.valid
    return va & vb


# ---------------------------------------------------------------------------
# array kernels
# ---------------------------------------------------------------------------
def _int_div(a, b, t, mod):
    """Rust '/' and '%' (truncating) on same-typed int arrays; b has no zeros."""
    with np.errstate(all="ignore"):
        if not is_signed(t):
            return (a % b) if mod else (a // b)
        ua = np.abs(a.astype(np.int64)).astype(np.uint64)
        ua = np.where(a.astype(np.int64) == np.iinfo(np.int64).min, np.uint64(1) << np.uint64(63), ua)
        ub = np.abs(b.astype(np.int64)).astype(np.uint64)
        q = (ua // ub).astype(np.uint64)
        neg = (a.astype(np.int64) < 0) != (b.astype(np.int64) < 0)
        q = np.where(neg, (np.uint64(0) - q), q).astype(np.int64)
        if not mod:
            return q.astype(NP[t])
        r = (a.astype(np.int64) - (q * b.astype(np.int64))).astype(NP[t])
        return r


def arith_arrays(op, l, r):
    """arrow add/subtract/multiply/divide on same-typed arrays (+ '%')."""
    t = l.type
    valid = _both_valid(l, r)
    a, b = l.values, r.values
    if op in ("/", "%"):
        vz = (b == 0) if valid is None else ((b == 0) & valid)
        if np.any(vz):
            raise internal("Divide by zero error")
        b = np.where(b == 0, np.ones(1, dtype=b.dtype), b)
    with np.errstate(all="ignore"):
        if op == "+":
            out = a + b
        elif op == "-":
            out = a - b
        elif op == "*":
            out = a * b
        elif t.startswith("Float"):
            out = a / b if op == "/" else np.fmod(a, b)
        else:
            out = _int_div(a, b, t, op == "%")
    return Arr(t, np.asarray(out, dtype=NP[t]), valid)


def data_array_arithmetic_op(op, left, right):
    """left/right: Arr or Value (DataColumnarValue)."""
    if isinstance(left, Arr) and isinstance(right, Arr):
        la, ra = left, right
    elif isinstance(left, Arr):
        la, ra = left, to_array(right, len(left))
    elif isinstance(right, Arr):
        la, ra = to_array(left, len(right)), right
    else:
        la, ra = to_array(left, 1), to_array(right, 1)
    ct = numerical_coercion(op, la.type, ra.type)
    return arith_arrays(op, cast(la, ct), cast(ra, ct))


def _cmp(op, a, b):
    return {"=": a == b, "<": a < b, "<=": a <= b, ">": a > b, ">=": a >= b}[op]


def _cmp_arrays(op, l, r):
    if l.type == "Utf8":
        vals = [_cmp(op, x, y) for x, y in zip(l.values, r.values)]
        return Arr("Boolean", vals, _both_valid(l, r))
    if l.type not in NP:
        names = {"=": "eq", "<": "lt", "<=": "lt_eq", ">": "gt", ">=": "gt_eq"}
        raise internal("Unsupported arithmetic_compute::%s for data type: %s" % (names[op], l.type))
    return Arr("Boolean", list(_cmp(op, l.values, r.values)), _both_valid(l, r))


def data_array_comparison_op(op, left, right):
    if isinstance(left, Arr) and isinstance(right, Arr):
        ct = equal_coercion(op, left.type, right.type)
        return _cmp_arrays(op, cast(left, ct), cast(right, ct))
    if isinstance(left, Arr):
        ct = equal_coercion(op, left.type, right.type)
        s = cast(to_array(right, 1), ct)
        return _cmp_arrays(op, cast(left, ct), _bcast(s, len(left)))
    if isinstance(right, Arr):  # scalar-array: operator flipped (:76-84)
        ct = equal_coercion(op, right.type, left.type)
        s = cast(to_array(left, 1), ct)
        return _cmp_arrays(FLIP[op], cast(right, ct), _bcast(s, len(right)))
    raise internal("Cannot do data_array %s, left:%s, right:%s" % (op, left.type, right.type))


def data_array_logic_op(op, left, right):
    """data_array_logic.rs:10-31: and/or of two Boolean ARRAYS (arrow
    compute::and / or via array_boolean_op!, macros.rs:212-218)."""
    if not (isinstance(left, Arr) and isinstance(right, Arr)):
        raise internal("Cannot do data_array %s, left:%s, right:%s" % (op, left.type, right.type))
    for a in (left, right):
        if a.type != "Boolean":  # downcast_array! (macros.rs:5-16)
            raise internal("Cannot downcast_array from datatype:%s item to:BooleanArray" % a.type)
    if len(left) != len(right):
        raise internal("Cannot perform bitwise operation on arrays of different length")
    lv, rv = left.values, right.values
    out = [(bool(a) and bool(b)) if op == "and" else (bool(a) or bool(b)) for a, b in zip(lv, rv)]
    return Arr("Boolean", out)


def _bcast(one, n):
    if one.type in NP:
        return Arr(one.type, np.repeat(one.values, n), None if one.valid is None else np.repeat(one.valid, n))
    return Arr(one.type, list(one.values) * n, one.valid)


def data_array_aggregate_op(op, a):
    """min/max/sum/count over one array -> Value (None when no valid value)."""
    if op == "count":
        return Value("UInt64", len(a))
    if a.type not in NP and not (a.type == "Utf8" and op in ("min", "max")):
        raise internal("Unsupported data_array_%s for data type: %s" % (op, a.type))
    idx = [i for i in range(len(a)) if a.is_valid(i)] if a.valid is not None else None
    if a.type == "Utf8":
        vals = [v for i, v in enumerate(a.values) if a.is_valid(i)]
        if not vals:
            return Value("Utf8", None)
        return Value("Utf8", min(vals) if op == "min" else max(vals))
    vals = a.values if idx is None else a.values[idx]
    if len(vals) == 0:
        return Value(a.type, None)
    if op == "sum":
        if a.type.startswith("Float"):
            s = float(np.sum(vals.astype(np.float64))) if a.type == "Float64" else float(np.sum(vals))
            return Value(a.type, s)
        with np.errstate(over="ignore"):
            s = vals.sum(dtype=NP[a.type])
        return Value(a.type, int(s))
    # min_max_helper: fold from m[0], replace when cmp(n, item)
    n = vals[0]
    for it in vals[1:]:
        if (op == "min" and n > it) or (op == "max" and n < it):
            n = it
    return Value(a.type, float(n) if a.type.startswith("Float") else int(n))


def data_value_arithmetic_op(op, l, r):
    if l.is_untyped_null():
        return r
    if r.is_untyped_null():
        return l
    out = data_array_arithmetic_op(op, to_array(l, 1), to_array(r, 1))
    return out.get(0)


def data_value_aggregate_op(op, l, r):
    if l.is_untyped_null():
        return r
    if r.is_untyped_null():
        return l
    if l.type != r.type or (l.type not in NP and not (l.type == "Utf8" and op in ("min", "max"))):
        raise internal("Unsupported data_value_%s for data type: left:%s, right:%s" % (op, l.type, r.type))
    if op == "count":
        return Value("UInt64", 1)
    a, b = l.value, r.value
    if a is None and b is None:
        return Value(l.type, None)
    if b is None:
        return l
    if a is None:
        return r
    if op == "sum":
        if l.type.startswith("Float"):
            return Value(l.type, a + b)
        lo, hi = int_range(l.type)
        v = (a + b - lo) % (hi - lo + 1) + lo
        return Value(l.type, v)
    if l.type.startswith("Float"):  # f64::min/max ignore NaN
        if a != a:
            return r
        if b != b:
            return l
    return Value(l.type, min(a, b) if op == "min" else max(a, b))


# ---------------------------------------------------------------------------
# functions (src/functions/)
# ---------------------------------------------------------------------------
class Block:
    def __init__(self, cols):
        self.cols = dict(cols)

    def num_rows(self):
        return len(next(iter(self.cols.values()))) if self.cols else 0

    def column_by_name(self, name):
        if name not in self.cols:
            raise internal('Invalid argument error: Unable to get field named "%s". Valid fields: [%s]' % (
                name, ", ".join('"%s"' % k for k in self.cols)))
        return self.cols[name]

    def take(self, mask):
        return Block({k: v.take(mask) for k, v in self.cols.items()})


class Fn:
    depth = 0

    def set_depth(self, d):
        self.depth = d

    def accumulate(self, block):
        pass


class Field(Fn):
    def __init__(self, name):
        self.name = name

    def display(self):
        return self.name

    def return_type(self, schema):
        return schema[self.name]

    def eval(self, block):
        return block.column_by_name(self.name)

    def accumulate(self, block):
        block.column_by_name(self.name)

    def _err(self, *a):
        raise internal("Unsupported aggregate operation for function field")

    accumulate_result = merge_state = merge_result = _err

    def clone(self):
        f = Field(self.name)
        f.depth = self.depth
        return f


class Const(Fn):
    def __init__(self, value):
        self.value = value

    def display(self):
        return self.value.debug()

    def return_type(self, schema):
        return self.value.type

    def eval(self, block):
        return self.value

    def accumulate_result(self):
        return [self.value]

    def merge_state(self, states):
        pass

    def merge_result(self):
        return self.value

    def clone(self):
        return Const(self.value)


class Alias(Fn):
    def __init__(self, alias, func):
        self.alias, self.func = alias, func

    def display(self):
        return self.alias

    def return_type(self, s):
        return self.func.return_type(s)

    def eval(self, b):
        return self.func.eval(b)

    def accumulate(self, b):
        self.func.accumulate(b)

    def accumulate_result(self):
        return self.func.accumulate_result()

    def merge_state(self, s):
        self.func.merge_state(s)

    def merge_result(self):
        return self.func.merge_result()

    def clone(self):
        a = Alias(self.alias, self.func.clone())
        a.depth = self.depth
        return a


class Arith(Fn):
    def __init__(self, op, left, right):
        self.op, self.left, self.right = op, left, right

    def display(self):
        return "%s %s %s" % (self.left.display(), self.op, self.right.display())

    def return_type(self, s):
        return numerical_coercion(self.op, self.left.return_type(s), self.right.return_type(s))

    def set_depth(self, d):
        self.left.set_depth(d)
        self.right.set_depth(d + 1)
        self.depth = d

    def eval(self, b):
        return data_array_arithmetic_op(self.op, self.left.eval(b), self.right.eval(b))

    def accumulate(self, b):
        self.left.accumulate(b)
        self.right.accumulate(b)

    def accumulate_result(self):
        return self.left.accumulate_result() + self.right.accumulate_result()

    def merge_state(self, s):
        self.left.merge_state(s)
        self.right.merge_state(s)

    def merge_result(self):
        return data_value_arithmetic_op(self.op, self.left.merge_result(), self.right.merge_result())

    def clone(self):
        a = Arith(self.op, self.left.clone(), self.right.clone())
        a.depth = self.depth
        return a


class Compare(Fn):
    def __init__(self, op, left, right):
        self.op, self.left, self.right = op, left, right

    def display(self):
        return "%s %s %s" % (self.left.display(), self.op, self.right.display())

    def return_type(self, s):
        return "Boolean"

    def eval(self, b):
        return data_array_comparison_op(self.op, self.left.eval(b), self.right.eval(b))

    def accumulate(self, b):
        self.left.accumulate(b)
        self.right.accumulate(b)

    def _err(self, *a):
        raise internal("Unsupported aggregate operation for function %s" % self.op)

    accumulate_result = merge_state = merge_result = _err

    def clone(self):
        c = Compare(self.op, self.left.clone(), self.right.clone())
        c.depth = self.depth
        return c


class Logic(Fn):
    """LogicFunction (function_logic.rs:17-87)."""
    def __init__(self, op, left, right):
        self.op, self.left, self.right = op, left, right

    def display(self):
        return "%s %s %s" % (self.left.display(), self.op, self.right.display())

    def return_type(self, s):
        return "Boolean"

    def eval(self, b):
        return data_array_logic_op(self.op, self.left.eval(b), self.right.eval(b))

    def accumulate(self, b):
        self.left.accumulate(b)
        self.right.accumulate(b)

    def _err(self, *a):
        raise internal("Unsupported aggregate operation for function %s" % self.op)

    accumulate_result = merge_state = merge_result = _err

    def clone(self):
        c = Logic(self.op, self.left.clone(), self.right.clone())
        c.depth = self.depth
        return c


class Agg(Fn):
    def __init__(self, op, arg):
        self.op, self.arg = op, arg
        self.state = Value.null()

    def display(self):
        return "%s(%s)" % (AGG_DEBUG[self.op], self.arg.display())

    def return_type(self, s):
        return "UInt64" if self.op == "count" else self.arg.return_type(s)

    def eval(self, b):
        return self.arg.eval(b)

    def accumulate(self, b):
        rows = b.num_rows()
        val = self.arg.eval(b)
        if self.op == "count":
            self.state = data_value_arithmetic_op("+", self.state, Value("UInt64", rows))
            return
        arr = val if isinstance(val, Arr) else to_array(val, rows)
        delta = data_array_aggregate_op(self.op, arr)
        if self.op == "sum":
            self.state = data_value_arithmetic_op("+", self.state, delta)
        else:
            self.state = data_value_aggregate_op(self.op, self.state, delta)

    def accumulate_result(self):
        return [self.state]

    def merge_state(self, states):
        if self.depth >= len(states):
            raise internal("index out of bounds: the len is %d but the index is %d" % (len(states), self.depth))
        v = states[self.depth]
        if self.op in ("count", "sum"):
            self.state = data_value_arithmetic_op("+", self.state, v)
        else:
            self.state = data_value_aggregate_op(self.op, self.state, v)

    def merge_result(self):
        return self.state

    def clone(self):
        a = Agg(self.op, self.arg.clone())
        a.depth = self.depth
        a.state = self.state
        return a


def factory(name, args, modulo=True):
    n = name.lower()
    if n in ARITH and (n != "%" or modulo):
        return Arith(n, args[0], args[1])
    if n in CMP:
        return Compare(n, args[0], args[1])
    if n in ("and", "or"):
        return Logic(n, args[0], args[1])
    if n in AGG_DEBUG:
        return Agg(n, args[0])
    raise internal("Unsupported Function: %s" % name)


def set_depths(f, depth=0):
    """plan_to_function's depth assignment for a tree built with the helpers
    below (binary right child depth+1; function args depth+1 then set to depth)."""
    f.set_depth(depth)
    return f


# expression builders mirroring ExpressionPlan -> plan_to_function
def E_field(n):
    return ("field", n)


def E_const(v, t=None):
    if t is None:
        t = "UInt64" if isinstance(v, int) and v >= 0 else ("Int64" if isinstance(v, int) else "Float64")
    return ("const", Value(t, v))


def E_bin(op, l, r):
    return ("bin", op, l, r)


def E_fn(name, *args):
    return ("fn", name, list(args))


def E_alias(a, e):
    return ("alias", a, e)


def to_function(e, depth=0, modulo=True):
    k = e[0]
    if k == "field":
        return Field(e[1])
    if k == "const":
        return Const(e[1])
    if k == "bin":
        l = to_function(e[2], depth, modulo)
        r = to_function(e[3], depth + 1, modulo)
        f = factory(e[1], [l, r], modulo)
        f.set_depth(depth)
        return f
    if k == "fn":
        args = []
        for a in e[2]:
            f = to_function(a, depth + 1, modulo)
            f.set_depth(depth)
            args.append(f)
        f = factory(e[1], args, modulo)
        f.set_depth(depth)
        return f
    if k == "alias":
        f = to_function(e[2], depth, modulo)
        f.set_depth(depth)
        return Alias(e[1], f)
    raise ValueError(e)


def is_aggregate(e):
    if e[0] == "alias":
        return is_aggregate(e[2])
    if e[0] == "bin":
        return is_aggregate(e[2]) or is_aggregate(e[3])
    if e[0] == "fn":
        return e[1].lower() in ("max", "min", "avg", "count", "sum")
    return False


# ---------------------------------------------------------------------------
# numbers_mt + transforms
# ---------------------------------------------------------------------------
def generate_parts(total):
    chunk = total // 8
    if chunk == 0:
        return [(0, total - 1)]
    parts = []
    for p in range(8):
        s, e = p * chunk, (p + 1) * chunk - 1
        if p == 7:
            e += total % 8
        parts.append((s, e))
    return parts


def numbers_blocks(begin, end):
    count = end - begin + 1
    nb, rem = divmod(count, 10000)
    if nb == 0:
        yield (begin, end)
        return
    for i in range(nb):
        bb = begin + 10000 * i
        be = begin + 10000 * (i + 1) - 1
        if i == nb - 1 and rem > 0:
            be = bb + rem
        yield (bb, be)


def numbers_stream(total, parts=None):
    for (b, e) in (parts if parts is not None else generate_parts(total)):
        for (bb, be) in numbers_blocks(b, e):
            yield Block({"number": Arr("UInt64", np.arange(bb, be + 1, dtype=np.uint64))})


def filter_block(pred_fn, block):
    """FilterTransform::expression_executor."""
    res = pred_fn.eval(block)
    if not isinstance(res, Arr):
        res = to_array(res, block.num_rows())
    if res.type != "Boolean":
        raise internal("cannot downcast to boolean array")
    mask = [bool(v) and res.is_valid(i) for i, v in enumerate(res.values)]
    return block.take(mask)


def aggregate_query(total, exprs, where=None, modulo=True, parts=None):
    """Source x P -> Filter -> AggregatePartial x P -> Merge (partition order)
    -> AggregateFinal.  exprs: expression tuples.  Returns [Value] or raises."""
    if where is not None and is_aggregate(where):
        raise internal("Aggregate function ... is found in WHERE in query")
    parts = parts if parts is not None else generate_parts(total)
    partials = []
    for p in parts:
        funcs = [to_function(e, modulo=modulo) for e in exprs]
        pred = to_function(where, modulo=modulo) if where is not None else None
        for b in numbers_stream(total, [p]):
            if pred is not None:
                b = filter_block(pred, b)
            for f in funcs:
                f.accumulate(b)
        partials.append([f.accumulate_result() for f in funcs])
    finals = [to_function(e, modulo=modulo) for e in exprs]
    for states in partials:
        for f, s in zip(finals, states):
            f.merge_state(s)
    out = []
    for f in finals:
        v = f.merge_result()
        if not v.is_untyped_null() and v.value is None:
            raise internal("DataValue to array cannot be NONE NULL")
        out.append(v)
    return out


def projection_blocks(total, exprs, where=None, modulo=True):
    """The non-aggregate stream as the reference yields it, per partition:
    for every 10,000-row numbers block (numbers_stream.rs:27-83),
    FilterTransform::expression_executor (transform_filter.rs:38-55) then each
    projected expression (transform_projection.rs:45-56,
    stream_expression.rs:38-50).  Returns [partition][block][column] -> list of
    values (empty blocks kept)."""
    out = []
    for p in generate_parts(total):
        funcs = [to_function(e, modulo=modulo) for e in exprs]
        pred = to_function(where, modulo=modulo) if where is not None else None
        blocks = []
        for b in numbers_stream(total, [p]):
            if pred is not None:
                b = filter_block(pred, b)
            cols = []
            for f in funcs:
                v = f.eval(b)
                a = v if isinstance(v, Arr) else to_array(v, b.num_rows())
                cols.append([a.get(i).value for i in range(b.num_rows())])
            blocks.append(cols)
        out.append(blocks)
    return out


def projection_query(total, exprs, where=None, limit=None, modulo=True):
    """Rows in partition order (the reference's merge order is arrival order)."""
    rows = []
    for p in generate_parts(total):
        funcs = [to_function(e, modulo=modulo) for e in exprs]
        pred = to_function(where, modulo=modulo) if where is not None else None
        got = 0
        for b in numbers_stream(total, [p]):
            if limit is not None and got >= limit:
                break
            if pred is not None:
                b = filter_block(pred, b)
            cols = []
            for f in funcs:
                v = f.eval(b)
                cols.append(v if isinstance(v, Arr) else to_array(v, b.num_rows()))
            n = b.num_rows()
            for i in range(n):
                if limit is not None and got >= limit:
                    break
                rows.append(tuple(c.get(i).value for c in cols))
                got += 1
    return rows


def aggregate_partial_states(total, exprs, parts, where=None, modulo=True):
    """What one rank ships for its partitions `parts`: AggregatePartial per
    partition, merged in partition order, as accumulate_result() per expr."""
    merged = [to_function(e, modulo=modulo) for e in exprs]
    for p in parts:
        funcs = [to_function(e, modulo=modulo) for e in exprs]
        pred = to_function(where, modulo=modulo) if where is not None else None
        for b in numbers_stream(total, [p]):
            if pred is not None:
                b = filter_block(pred, b)
            for f in funcs:
                f.accumulate(b)
        for m, f in zip(merged, funcs):
            m.merge_state(f.accumulate_result())
    return [m.accumulate_result() for m in merged]


def group_by_query(total, key_expr, exprs, where=None, modulo=True):
    """GROUP BY -- NOT a restatement: the reference plans group_expr
    (plan_parser.rs:284-308) but PipelineBuilder ignores it
    (pipeline_builder.rs:50-66), so there is no reference behaviour to
    follow.  This is the semantics the device path implements, stated with
    the reference's own Function machinery: rows are filtered, grouped by the
    value of key_expr, every AggregatorFunction accumulates each block's rows
    of its group (function_aggregator.rs:57-100) and the aggregate
    expressions are merge_result()-ed per group.  Parity unpinned.
    Returns [(key, value...)] sorted by key."""
    key_fn = to_function(key_expr, modulo=modulo)
    pred = to_function(where, modulo=modulo) if where is not None else None
    groups = {}
    for b in numbers_stream(total):
        if pred is not None:
            b = filter_block(pred, b)
        if b.num_rows() == 0:
            continue
        kv = key_fn.eval(b)
        karr = kv if isinstance(kv, Arr) else to_array(kv, b.num_rows())
        keys = np.asarray(karr.values)
        for k in np.unique(keys):
            sub = b.take(list(keys == k))
            fs = groups.get(int(k))
            if fs is None:
                fs = groups[int(k)] = [to_function(e, modulo=modulo) for e in exprs]
            for f in fs:
                f.accumulate(sub)
    out = []
    for k in sorted(groups):
        row = [k]
        for f in groups[k]:
            row.append(f.merge_result().value)
        out.append(tuple(row))
    return out


def _agg_leaves(f, out):
    if isinstance(f, Agg):
        out.append(f)
    for attr in ("left", "right", "func"):
        g = getattr(f, attr, None)
        if isinstance(g, Fn):
            _agg_leaves(g, out)
    return out


def group_by_partial_states(total, key_expr, exprs, parts, where=None, modulo=True):
    """What one rank ships for a GROUP BY over its partitions `parts`: per
    group [key Value, state of every aggregate leaf (left to right)], sorted
    by key (the engine's exchange rows; see group_by_query)."""
    key_fn = to_function(key_expr, modulo=modulo)
    pred = to_function(where, modulo=modulo) if where is not None else None
    groups = {}
    ktype = None
    for b in numbers_stream(total, parts):
        if pred is not None:
            b = filter_block(pred, b)
        if b.num_rows() == 0:
            continue
        kv = key_fn.eval(b)
        karr = kv if isinstance(kv, Arr) else to_array(kv, b.num_rows())
        ktype = karr.type
        keys = np.asarray(karr.values)
        for k in np.unique(keys):
            sub = b.take(list(keys == k))
            fs = groups.get(int(k))
            if fs is None:
                fs = groups[int(k)] = [to_function(e, modulo=modulo) for e in exprs]
            for f in fs:
                f.accumulate(sub)
    rows = []
    for k in sorted(groups):
        leaves = []
        for f in groups[k]:
            _agg_leaves(f, leaves)
        rows.append([Value(ktype, k)] + [a.state for a in leaves])
    return rows
