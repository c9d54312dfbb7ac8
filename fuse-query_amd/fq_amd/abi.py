"""ctypes mirror of include/fq_gpu.h (layouts and constants only).

Nothing in this module computes anything; it is shared by the product
wrappers (fq_amd.ops / fq_amd.engine) and by the test-side oracle binding so
both speak the same struct layout.
"""
import ctypes as C

FQ_ABI_VERSION = 3

# status (src/error.rs:10-22)
FQ_OK = 0
FQ_E_INTERNAL = 1
FQ_E_PLAN = 2
FQ_E_DIVIDE_BY_ZERO = 3
FQ_E_UNSUPPORTED = 4
FQ_E_HIP = 5
FQ_E_RCCL = 6
FQ_E_INVALID = 7

# DataType
DT_NULL, DT_BOOLEAN, DT_INT8, DT_INT16, DT_INT32, DT_INT64 = 0, 1, 2, 3, 4, 5
DT_UINT8, DT_UINT16, DT_UINT32, DT_UINT64, DT_FLOAT32, DT_FLOAT64, DT_UTF8 = 6, 7, 8, 9, 10, 11, 12

DT_NAMES = {
    DT_NULL: "Null", DT_BOOLEAN: "Boolean", DT_INT8: "Int8", DT_INT16: "Int16",
    DT_INT32: "Int32", DT_INT64: "Int64", DT_UINT8: "UInt8", DT_UINT16: "UInt16",
    DT_UINT32: "UInt32", DT_UINT64: "UInt64", DT_FLOAT32: "Float32",
    DT_FLOAT64: "Float64", DT_UTF8: "Utf8",
}
DT_BY_NAME = {v: k for k, v in DT_NAMES.items()}

# operators (src/datavalues/data_value_operator.rs)
OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_MOD = 0, 1, 2, 3, 4
OP_PUSH = 5  # expression trees: push acc, acc = the column
OP_BY_SYM = {"+": OP_ADD, "-": OP_SUB, "*": OP_MUL, "/": OP_DIV, "%": OP_MOD}
CMP_EQ, CMP_LT, CMP_LTEQ, CMP_GT, CMP_GTEQ = 0, 1, 2, 3, 4
CMP_BY_SYM = {"=": CMP_EQ, "<": CMP_LT, "<=": CMP_LTEQ, ">": CMP_GT, ">=": CMP_GTEQ}
CMP_FLIP = {CMP_EQ: CMP_EQ, CMP_LT: CMP_GT, CMP_LTEQ: CMP_GTEQ, CMP_GT: CMP_LT, CMP_GTEQ: CMP_LTEQ}

AGG_MIN, AGG_MAX, AGG_SUM, AGG_COUNT = 1, 2, 4, 8
AGG_BY_NAME = {"min": AGG_MIN, "max": AGG_MAX, "sum": AGG_SUM, "count": AGG_COUNT}

OPERAND_CONST, OPERAND_COLUMN, OPERAND_STACK = 0, 1, 2
MAX_STACK = 2
PRED_NONE, PRED_EXPR, PRED_BITMAP = 0, 1, 2
MAX_STEPS = 8

STATE_ANY_EMPTY = 1
STATE_DIV_ZERO = 2
STATE_CAST_NULL = 4


class fq_value(C.Structure):
    _fields_ = [("dtype", C.c_int32), ("is_some", C.c_int32), ("bits", C.c_uint64)]


class fq_col(C.Structure):
    _fields_ = [("data", C.c_void_p), ("len", C.c_int64), ("dtype", C.c_int32),
                ("reserved", C.c_int32)]


class fq_step(C.Structure):
    _fields_ = [("op", C.c_int32), ("operand", C.c_int32), ("reversed", C.c_int32),
                ("dtype", C.c_int32), ("bits", C.c_uint64)]


class fq_expr(C.Structure):
    _fields_ = [("n_steps", C.c_int32), ("out_dtype", C.c_int32),
                ("steps", fq_step * MAX_STEPS)]


MAX_PRED_LEAVES = 4
PRED_TREE = 3
PRED_AND, PRED_OR = 100, 101


class fq_pred_leaf(C.Structure):
    _fields_ = [("cmp", C.c_int32), ("cmp_dtype", C.c_int32), ("rhs_operand", C.c_int32),
                ("reserved", C.c_int32), ("rhs_bits", C.c_uint64), ("lhs", fq_expr)]


class fq_pred_tree(C.Structure):
    _fields_ = [("n_leaves", C.c_int32), ("n_prog", C.c_int32), ("prog", C.c_int32 * (2 * MAX_PRED_LEAVES)),
                ("leaves", fq_pred_leaf * MAX_PRED_LEAVES)]


class fq_pred(C.Structure):
    _fields_ = [("kind", C.c_int32), ("cmp", C.c_int32), ("cmp_dtype", C.c_int32),
                ("rhs_operand", C.c_int32), ("rhs_bits", C.c_uint64), ("lhs", fq_expr),
                ("bitmap", C.c_void_p), ("tree", C.POINTER(fq_pred_tree))]


class fq_agg_state(C.Structure):
    _fields_ = [("sum", C.c_uint64), ("max", C.c_uint64), ("min", C.c_uint64),
                ("count", C.c_uint64), ("blocks", C.c_uint64), ("flags", C.c_uint32),
                ("dtype", C.c_int32)]


class fq_jit_stats(C.Structure):
    _fields_ = [("kernels_compiled", C.c_int64), ("jit_launches", C.c_int64),
                ("interp_launches", C.c_int64), ("compile_ms", C.c_double),
                ("available", C.c_int32), ("mode", C.c_int32), ("min_rows", C.c_int64)]


JIT_OFF, JIT_AUTO, JIT_ALWAYS = 0, 1, 2

MAX_GROUP_AGGS = 8
GROUP_NARROW_ROWS = 0x10000  # fq_group_aggregate_partitioned: 4-byte partition rows
FQ_E_TABLE_FULL = 8


class fq_group_table(C.Structure):
    _fields_ = [("d_mem", C.c_void_p), ("capacity", C.c_int64), ("key_dtype", C.c_int32),
                ("n_aggs", C.c_int32), ("kinds", C.c_int32 * MAX_GROUP_AGGS),
                ("dtypes", C.c_int32 * MAX_GROUP_AGGS)]

assert C.sizeof(fq_agg_state) == 48
assert C.sizeof(fq_step) == 24


# launch-shape knobs (fq_tune_set; tuning tools only)
TUNE = {
    "SCAN_WG_PER_CU": 0, "EW_WG_PER_CU": 1, "BLOCK_U": 2, "SELECT_WG_PER_CU": 3, "SELECT_BLOCKS_WG_PER_CU": 4,
    "SELECT_BLOCKS_ROWS": 5, "SELECT_BLOCKS_STAGE": 6, "BLOCK_CACHE": 7, "POOL_SPIN_US": 8, "GROUP_THREADS": 9,
    "GROUP_LDS_KB": 10, "GROUP_WG_PER_CU": 11, "GROUP_CLUSTER": 12, "GROUP_CHUNKED": 13, "GROUP_RANGE_BINS": 14,
    "GROUP_NARROW": 15, "GPART_WG_PER_CU": 16, "GBINS_WG_PER_CU": 17,
}
