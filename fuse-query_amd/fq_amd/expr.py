"""Builders for the fused-expression descriptors of include/fq_gpu.h.

A fused expression is the chain an ArithmeticFunction tree evaluates to when
every operator has a Constant or the column as its other child
(src/functions/function_arithmetic.rs:64-72).  Step types follow
numerical_coercion (src/datavalues/data_type.rs:27-90); comparison types
follow equal_coercion (:92-98).  Constants are typed like the SQL planner
types literals (src/planners/plan_parser.rs:216-229): int >= 0 -> UInt64,
int < 0 -> Int64, float -> Float64; or pass (value, "Int8") explicitly.
"""
import ctypes as C
import struct

from . import abi

_ORDER = [abi.DT_FLOAT64, abi.DT_FLOAT32, abi.DT_INT64, abi.DT_INT32, abi.DT_INT16,
          abi.DT_INT8, abi.DT_UINT64, abi.DT_UINT32, abi.DT_UINT16, abi.DT_UINT8]
_NUMERIC = set(_ORDER)


class CoercionError(Exception):
    pass


def numerical_coercion(op, l, r):
    """data_type.rs:27-90; raises with the reference's error text."""
    if l not in _NUMERIC or r not in _NUMERIC:
        raise CoercionError("Internal Error: Unsupported (%s) %s (%s)" % (
            abi.DT_NAMES[l], op, abi.DT_NAMES[r]))
    if l == r:
        return l
    for t in _ORDER:
        if l == t or r == t:
            return t
    raise CoercionError("unreachable")


def equal_coercion(op, l, r):
    if l == r:
        return l
    return numerical_coercion(op, l, r)


def to_bits(value, dtype):
    """fq_value encoding: ints sign/zero-extended to 64 bits, floats binary64."""
    if dtype in (abi.DT_FLOAT32, abi.DT_FLOAT64):
        return struct.unpack("<Q", struct.pack("<d", float(value)))[0]
    if dtype == abi.DT_BOOLEAN:
        return 1 if value else 0
    return int(value) & 0xFFFFFFFFFFFFFFFF


def from_bits(bits, dtype):
    if dtype in (abi.DT_FLOAT32, abi.DT_FLOAT64):
        return struct.unpack("<d", struct.pack("<Q", bits & 0xFFFFFFFFFFFFFFFF))[0]
    if dtype in (abi.DT_INT8, abi.DT_INT16, abi.DT_INT32, abi.DT_INT64):
        b = bits & 0xFFFFFFFFFFFFFFFF
        return b - (1 << 64) if b >> 63 else b
    if dtype == abi.DT_BOOLEAN:
        return bool(bits)
    return bits & 0xFFFFFFFFFFFFFFFF


def literal(v):
    """(value, dtype) of a constant, typed like the SQL planner."""
    if isinstance(v, tuple):
        val, dt = v
        return val, (abi.DT_BY_NAME[dt] if isinstance(dt, str) else dt)
    if isinstance(v, bool):
        return v, abi.DT_BOOLEAN
    if isinstance(v, int):
        return v, (abi.DT_UINT64 if v >= 0 else abi.DT_INT64)
    if isinstance(v, float):
        return v, abi.DT_FLOAT64
    raise TypeError("unsupported constant %r" % (v,))


COL = "col"  # operand marker: the column itself
STACK = "stack"  # operand marker: the value pushed by the matching ("push",) step
PUSH = ("push",)  # step: push acc, restart from the column (expression trees)


def chain(col_dtype, steps):
    """steps: [(sym, operand[, reversed])]; operand = constant or COL.
    Returns (fq_expr, out_dtype)."""
    e = abi.fq_expr()
    acc = col_dtype
    stack = []
    if len(steps) > abi.MAX_STEPS:
        raise ValueError("too many steps")
    for i, st in enumerate(steps):
        if st[0] == "push":  # tree: keep acc (the left subtree), restart from the column
            s = e.steps[i]
            s.op, s.operand, s.reversed, s.dtype, s.bits = abi.OP_PUSH, abi.OPERAND_CONST, 0, col_dtype, 0
            stack.append(acc)
            acc = col_dtype
            continue
        sym, operand = st[0], st[1]
        rev = bool(st[2]) if len(st) > 2 else False
        if operand is STACK or operand == STACK:
            odt = stack.pop()
            okind, obits = abi.OPERAND_STACK, 0
        elif operand is COL or operand == COL:
            odt = col_dtype
            okind, obits = abi.OPERAND_COLUMN, 0
        else:
            val, odt = literal(operand)
            okind = abi.OPERAND_CONST
        dt = numerical_coercion(sym, odt, acc) if rev else numerical_coercion(sym, acc, odt)
        if okind == abi.OPERAND_CONST:
            obits = to_bits(val, dt)
        s = e.steps[i]
        s.op = abi.OP_BY_SYM[sym]
        s.operand = okind
        s.reversed = 1 if rev else 0
        s.dtype = dt
        s.bits = obits
        acc = dt
    e.n_steps = len(steps)
    e.out_dtype = acc
    return e, acc


def predicate(col_dtype, lhs_steps, cmp_sym, rhs, flipped=False):
    """cmp(chain(lhs_steps)(x), rhs) with rhs a constant or COL.  flipped=True
    builds the scalar-array form `rhs cmp chain` (the reference flips the
    operator, data_array_comparison.rs:76-84)."""
    p = abi.fq_pred()
    p.kind = abi.PRED_EXPR
    lhs, ldt = chain(col_dtype, lhs_steps)
    p.lhs = lhs
    if rhs is COL or rhs == COL:
        rdt = col_dtype
        p.rhs_operand = abi.OPERAND_COLUMN
    else:
        val, rdt = literal(rhs)
        p.rhs_operand = abi.OPERAND_CONST
    cdt = equal_coercion(cmp_sym, ldt, rdt)
    cmp = abi.CMP_BY_SYM[cmp_sym]
    p.cmp = abi.CMP_FLIP[cmp] if flipped else cmp
    p.cmp_dtype = cdt
    if p.rhs_operand == abi.OPERAND_CONST:
        p.rhs_bits = to_bits(val, cdt)
    return p


def pred_tree(col_dtype, leaves, prog):
    """and/or predicate tree (FQ_PRED_TREE): leaves = [(lhs_steps, cmp_sym,
    rhs)], prog = postfix tokens: leaf indices and "and" / "or"."""
    t = abi.fq_pred_tree()
    if not 1 <= len(leaves) <= abi.MAX_PRED_LEAVES:
        raise ValueError("1..%d leaves" % abi.MAX_PRED_LEAVES)
    t.n_leaves = len(leaves)
    for i, (steps, cmp_sym, rhs) in enumerate(leaves):
        p = predicate(col_dtype, steps, cmp_sym, rhs)
        lf = t.leaves[i]
        lf.cmp, lf.cmp_dtype, lf.rhs_operand, lf.rhs_bits, lf.lhs = p.cmp, p.cmp_dtype, p.rhs_operand, p.rhs_bits, p.lhs
    toks = [(abi.PRED_AND if x == "and" else abi.PRED_OR) if isinstance(x, str) else int(x) for x in prog]
    t.n_prog = len(toks)
    for i, x in enumerate(toks):
        t.prog[i] = x
    pr = abi.fq_pred()
    pr.kind = abi.PRED_TREE
    pr.tree = C.pointer(t)
    pr._tree = t  # keep the tree alive with the predicate
    return pr
