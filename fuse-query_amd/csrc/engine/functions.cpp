// Expression tree over device columns + the fused aggregate driver.
#include "functions.h"

#include <string.h>

#include <algorithm>

#include "../fq_common.h"

namespace fq {

static bool is_chain_dtype(DataType dt) {
    return dt == FQ_DT_UINT64 || dt == FQ_DT_INT64 || dt == FQ_DT_FLOAT64;
}

std::string FusedChain::key() const {
    std::string k = column + ":" + std::to_string(col_dtype) + ":" + std::to_string(out_dtype);
    for (int i = 0; i < expr.n_steps; ++i) {
        const fq_step &s = expr.steps[i];
        k += "/" + std::to_string(s.op) + "," + std::to_string(s.operand) + "," + std::to_string(s.reversed) +
             "," + std::to_string(s.dtype) + "," + std::to_string(s.bits);
    }
    return k;
}

std::string FusedPred::key() const {
    auto leaf = [this](const fq_expr &lhs, int32_t cmp, int32_t cdt, int32_t ro, uint64_t rb) {
        FusedChain c;
        c.column = column;
        c.col_dtype = col_dtype;
        c.expr = lhs;
        c.out_dtype = lhs.out_dtype;
        return c.key() + "?" + std::to_string(cmp) + "," + std::to_string(cdt) + "," + std::to_string(ro) + "," +
               std::to_string(rb);
    };
    if (pred.kind != FQ_PRED_TREE) return leaf(pred.lhs, pred.cmp, pred.cmp_dtype, pred.rhs_operand, pred.rhs_bits);
    std::string k = "T";
    for (int i = 0; i < tree.n_prog; ++i) k += std::to_string(tree.prog[i]) + ",";
    for (int i = 0; i < tree.n_leaves; ++i) {
        const fq_pred_leaf &l = tree.leaves[i];
        k += "[" + leaf(l.lhs, l.cmp, l.cmp_dtype, l.rhs_operand, l.rhs_bits) + "]";
    }
    return k;
}

// ---------------------------------------------------------------------------
// device element-wise ops (data_array_arithmetic_op / data_array_comparison_op)
// ---------------------------------------------------------------------------
static void side(const ColumnarValue &v, fq_col &c, fq_value &s, bool &is_col) {
    is_col = v.is_array;
    if (v.is_array) c = v.array.abi();
    else s = v.scalar.to_abi();
}

static void none_check(const ColumnarValue &v) {
    if (!v.is_array && v.scalar.kind == DataValue::kNone) throw_internal("DataValue to array cannot be NONE NULL");
    if (!v.is_array && v.scalar.kind == DataValue::kStruct)
        throw_internal("DataValue to array cannot be NONE " + v.scalar.debug());
}

static Column device_arith(int32_t op, const ColumnarValue &l, const ColumnarValue &r, ExecCtx &ctx) {
    none_check(l);
    none_check(r);
    if (!l.is_array && !r.is_array) {
        // both to_array(1): one-row result (data_array_arithmetic.rs:277-279)
        int32_t ct = 0;
        check_fq(fq_arith_result_type(op, l.scalar.data_type(), r.scalar.data_type(), &ct));
        const DataValue v = data_value_arithmetic_op(op, l.scalar, r.scalar);
        if (v.kind != DataValue::kSome)
            throw_status(FQ_E_UNSUPPORTED, "cast produced nulls (nulls are not supported on the device path)");
        return value_to_array(v, 1, ctx);
    }
    fq_col lc{}, rc{};
    fq_value ls{}, rs{};
    bool lcol, rcol;
    side(l, lc, ls, lcol);
    side(r, rc, rs, rcol);
    int32_t ct = 0;
    check_fq(fq_arith_result_type(op, lcol ? lc.dtype : ls.dtype, rcol ? rc.dtype : rs.dtype, &ct));
    const int64_t n = lcol ? lc.len : rc.len;
    Column out = Column::device(ct, n, ctx.stream());
    fq_col oc = out.abi();
    auto flag = DeviceBuffer::alloc(4, ctx.stream());
    check_fq(fq_arith(op, lcol ? &lc : nullptr, lcol ? nullptr : &ls, rcol ? &rc : nullptr, rcol ? nullptr : &rs,
                      &oc, (uint32_t *)flag->ptr, ctx.stream()));
    return out;
}

static Column device_compare(int32_t cmp, const ColumnarValue &l, const ColumnarValue &r, ExecCtx &ctx) {
    if (!l.is_array && !r.is_array)  // data_array_comparison.rs:90-95
        throw_internal(std::string("Cannot do data_array ") + fqc::cmp_op_str(cmp) + ", left:" +
                       dtype_name(l.data_type()) + ", right:" + dtype_name(r.data_type()));
    none_check(l);
    none_check(r);
    fq_col lc{}, rc{};
    fq_value ls{}, rs{};
    bool lcol, rcol;
    side(l, lc, ls, lcol);
    side(r, rc, rs, rcol);
    const int64_t n = lcol ? lc.len : rc.len;
    Column out = Column::device(FQ_DT_BOOLEAN, n, ctx.stream());
    auto flag = DeviceBuffer::alloc(4, ctx.stream());
    check_fq(fq_compare(cmp, lcol ? &lc : nullptr, lcol ? nullptr : &ls, rcol ? &rc : nullptr,
                        rcol ? nullptr : &rs, (uint64_t *)out.dptr(), n, (uint32_t *)flag->ptr, ctx.stream()));
    return out;
}

// ---------------------------------------------------------------------------
// FieldFunction
// ---------------------------------------------------------------------------
DataType FieldFunction::return_type(const DataSchema &s) const { return s.field_with_name(name_).dtype; }
bool FieldFunction::nullable(const DataSchema &s) const { return s.field_with_name(name_).nullable; }

ColumnarValue FieldFunction::eval(const DataBlock &b, ExecCtx &) {
    ColumnarValue v;
    v.is_array = true;
    v.array = b.column_by_name(name_);
    return v;
}

void FieldFunction::accumulate(const DataBlock &b, ExecCtx &ctx) {
    try {
        (void)b.column_by_name(name_);  // `saved = Some(column_by_name(..)?)`
    } catch (const FQException &e) {
        if (ctx.fusion) ctx.fusion->add_error(e);
        else throw;
    }
}

std::vector<DataValue> FieldFunction::accumulate_result() const {
    throw_internal("Unsupported aggregate operation for function field");
}
void FieldFunction::merge_state(const std::vector<DataValue> &) {
    throw_internal("Unsupported aggregate operation for function field");
}
DataValue FieldFunction::merge_result() const { throw_internal("Unsupported aggregate operation for function field"); }

bool FieldFunction::to_chain(const DataSchema &s, FusedChain &c) const {
    int idx;
    try {
        idx = s.index_of(name_);
    } catch (const FQException &) {
        return false;
    }
    const DataType dt = s.fields[(size_t)idx].dtype;
    if (!dtype_is_numeric(dt)) return false;
    c = FusedChain{};
    c.column = name_;
    c.col_dtype = dt;
    c.expr.n_steps = 0;
    c.expr.out_dtype = dt;
    c.out_dtype = dt;
    return true;
}

// ---------------------------------------------------------------------------
// ConstantFunction
// ---------------------------------------------------------------------------
ColumnarValue ConstantFunction::eval(const DataBlock &, ExecCtx &) {
    ColumnarValue v;
    v.is_array = false;
    v.scalar = value_;
    return v;
}

// ---------------------------------------------------------------------------
// ArithmeticFunction
// ---------------------------------------------------------------------------
std::string ArithmeticFunction::display() const {
    return left_->display() + " " + fqc::arith_op_str(op_) + " " + right_->display();
}

DataType ArithmeticFunction::return_type(const DataSchema &s) const {
    int32_t ct = 0;
    check_fq(fq_arith_result_type(op_, left_->return_type(s), right_->return_type(s), &ct));
    return ct;
}

ColumnarValue ArithmeticFunction::eval(const DataBlock &b, ExecCtx &ctx) {
    ColumnarValue l = left_->eval(b, ctx);
    ColumnarValue r = right_->eval(b, ctx);
    ColumnarValue out;
    out.is_array = true;
    out.array = device_arith(op_, l, r, ctx);
    return out;
}

std::vector<DataValue> ArithmeticFunction::accumulate_result() const {
    std::vector<DataValue> a = left_->accumulate_result();
    std::vector<DataValue> b = right_->accumulate_result();
    a.insert(a.end(), b.begin(), b.end());
    return a;
}

DataValue ArithmeticFunction::merge_result() const {
    return data_value_arithmetic_op(op_, left_->merge_result(), right_->merge_result());
}

// Expression trees run on the hipRTC kernels only: fuse them while the JIT is
// on (FQ_JIT / fq_jit_config) and hipRTC has not been found missing.
static bool tree_fusion_enabled() {
    fq_jit_stats js{};
    return fq_jit_get_stats(&js) == FQ_OK && js.mode != FQ_JIT_OFF && js.available != 0;
}

// Append one step `acc OP operand` (or `operand OP acc`) to a chain.
static bool push_step(FusedChain &c, int32_t op, bool column_operand, const DataValue *k, bool reversed) {
    if (c.expr.n_steps >= FQ_MAX_STEPS) return false;
    if (!is_chain_dtype(c.col_dtype)) return false;
    const DataType odt = column_operand ? c.col_dtype : k->dtype;
    int32_t ct = 0;
    const int32_t l = reversed ? odt : c.out_dtype, r = reversed ? c.out_dtype : odt;
    if (fqc::numerical_coercion(fqc::arith_op_str(op), l, r, &ct) != FQ_OK) return false;
    if (!is_chain_dtype(ct)) return false;
    fq_step &st = c.expr.steps[c.expr.n_steps];
    st.op = op;
    st.operand = column_operand ? FQ_OPERAND_COLUMN : FQ_OPERAND_CONST;
    st.reversed = reversed ? 1 : 0;
    st.dtype = ct;
    st.bits = 0;
    if (!column_operand && !fqc::cast_scalar(k->bits, k->dtype, ct, &st.bits)) return false;
    c.expr.n_steps++;
    c.expr.out_dtype = ct;
    c.out_dtype = ct;
    return true;
}

static bool numeric_constant(const Function &f, const DataValue *&v) {
    v = f.as_constant();
    return v && v->kind == DataValue::kSome && dtype_is_numeric(v->dtype);
}

bool ArithmeticFunction::to_chain(const DataSchema &s, FusedChain &c) const {
    const DataValue *k = nullptr;
    const std::string *fld = nullptr;
    FusedChain l, r;  // each child lowered once
    const bool lok = left_->to_chain(s, l), rok = right_->to_chain(s, r);
    if (numeric_constant(*right_, k) && lok) {
        c = l;
        return push_step(c, op_, false, k, false);
    }
    if (numeric_constant(*left_, k) && rok) {
        c = r;
        return push_step(c, op_, false, k, true);
    }
    if ((fld = right_->as_field()) && lok && *fld == l.column) {
        c = l;
        return push_step(c, op_, true, nullptr, false);
    }
    if ((fld = left_->as_field()) && rok && *fld == r.column) {
        c = r;
        return push_step(c, op_, true, nullptr, true);
    }
    // both children are expressions over the same column: an expression tree
    // (left subtree, FQ_OP_PUSH, right subtree, then this node with the
    // popped left value as its operand) -- hipRTC kernels only
    if (!lok || !rok || l.column != r.column || !tree_fusion_enabled()) return false;
    if (l.expr.n_steps + r.expr.n_steps + 2 > FQ_MAX_STEPS) return false;
    const int depth = std::max(l.depth, 1 + r.depth);
    if (depth > FQ_MAX_STACK || !is_chain_dtype(l.col_dtype)) return false;
    int32_t ct = 0;
    if (fqc::numerical_coercion(fqc::arith_op_str(op_), l.out_dtype, r.out_dtype, &ct) != FQ_OK || !is_chain_dtype(ct))
        return false;
    c = l;
    fq_step &push = c.expr.steps[c.expr.n_steps++];
    push = fq_step{};
    push.op = FQ_OP_PUSH;
    push.dtype = l.col_dtype;
    for (int i = 0; i < r.expr.n_steps; ++i) c.expr.steps[c.expr.n_steps++] = r.expr.steps[i];
    fq_step &node = c.expr.steps[c.expr.n_steps++];
    node = fq_step{};
    node.op = op_;
    node.operand = FQ_OPERAND_STACK;
    node.reversed = 1;  // left OP right
    node.dtype = ct;
    c.expr.out_dtype = ct;
    c.out_dtype = ct;
    c.depth = depth;
    return true;
}

// ---------------------------------------------------------------------------
// ComparisonFunction
// ---------------------------------------------------------------------------
std::string ComparisonFunction::display() const {
    return left_->display() + " " + fqc::cmp_op_str(cmp_) + " " + right_->display();
}

ColumnarValue ComparisonFunction::eval(const DataBlock &b, ExecCtx &ctx) {
    ColumnarValue l = left_->eval(b, ctx);
    ColumnarValue r = right_->eval(b, ctx);
    ColumnarValue out;
    out.is_array = true;
    out.array = device_compare(cmp_, l, r, ctx);
    return out;
}

std::vector<DataValue> ComparisonFunction::accumulate_result() const {
    throw_internal(std::string("Unsupported aggregate operation for function ") + fqc::cmp_op_str(cmp_));
}
void ComparisonFunction::merge_state(const std::vector<DataValue> &) {
    throw_internal(std::string("Unsupported aggregate operation for function ") + fqc::cmp_op_str(cmp_));
}
DataValue ComparisonFunction::merge_result() const {
    throw_internal(std::string("Unsupported aggregate operation for function ") + fqc::cmp_op_str(cmp_));
}

static int32_t flip(int32_t cmp) {
    switch (cmp) {
        case FQ_CMP_LT: return FQ_CMP_GT;
        case FQ_CMP_LTEQ: return FQ_CMP_GTEQ;
        case FQ_CMP_GT: return FQ_CMP_LT;
        case FQ_CMP_GTEQ: return FQ_CMP_LTEQ;
        default: return cmp;
    }
}

static bool make_pred(const FusedChain &lhs, int32_t cmp, bool column_rhs, const DataValue *k, FusedPred &p) {
    if (!is_chain_dtype(lhs.col_dtype)) return false;
    const DataType rdt = column_rhs ? lhs.col_dtype : k->dtype;
    int32_t ct = 0;
    if (fqc::equal_coercion(fqc::cmp_op_str(cmp), lhs.out_dtype, rdt, &ct) != FQ_OK) return false;
    if (!is_chain_dtype(ct)) return false;
    p = FusedPred{};
    p.column = lhs.column;
    p.col_dtype = lhs.col_dtype;
    p.pred.kind = FQ_PRED_EXPR;
    p.pred.cmp = cmp;
    p.pred.cmp_dtype = ct;
    p.pred.rhs_operand = column_rhs ? FQ_OPERAND_COLUMN : FQ_OPERAND_CONST;
    p.pred.lhs = lhs.expr;
    if (!column_rhs && !fqc::cast_scalar(k->bits, k->dtype, ct, &p.pred.rhs_bits)) return false;
    return true;
}

bool ComparisonFunction::to_pred(const DataSchema &s, FusedPred &p) const {
    const DataValue *k = nullptr;
    const std::string *fld = nullptr;
    FusedChain c;
    if (numeric_constant(*right_, k) && left_->to_chain(s, c)) return make_pred(c, cmp_, false, k, p);
    // scalar-array form: the reference flips the operator (data_array_comparison.rs:76-84)
    if (numeric_constant(*left_, k) && right_->to_chain(s, c)) return make_pred(c, flip(cmp_), false, k, p);
    if ((fld = right_->as_field()) && left_->to_chain(s, c) && *fld == c.column) return make_pred(c, cmp_, true, nullptr, p);
    if ((fld = left_->as_field()) && right_->to_chain(s, c) && *fld == c.column)
        return make_pred(c, flip(cmp_), true, nullptr, p);
    return false;
}

// ---------------------------------------------------------------------------
// AggregatorFunction
// ---------------------------------------------------------------------------
std::string AggregatorFunction::display() const {
    return std::string(agg_op_debug_name(op_)) + "(" + arg_->display() + ")";
}

DataType AggregatorFunction::return_type(const DataSchema &s) const {
    return op_ == FQ_AGG_COUNT ? FQ_DT_UINT64 : arg_->return_type(s);
}

void AggregatorFunction::merge_state(const std::vector<DataValue> &states) {
    if (depth_ >= states.size())
        throw_internal("index out of bounds: the len is " + std::to_string(states.size()) + " but the index is " +
                       std::to_string(depth_));
    const DataValue &val = states[depth_];
    if (op_ == FQ_AGG_COUNT || op_ == FQ_AGG_SUM) state_ = data_value_arithmetic_op(FQ_OP_ADD, state_, val);
    else state_ = data_value_aggregate_op(op_, state_, val);
}

void AggregatorFunction::accumulate(const DataBlock &b, ExecCtx &ctx) {
    if (ctx.fusion) {
        ctx.fusion->add(this, b);
        return;
    }
    accumulate_summary(summarize(b, ctx));
}

// One device block = `st.blocks` reference blocks.  For each block the
// reference does (function_aggregator.rs:57-100):
//   Count:   state = state + UInt64(rows)
//   Min/Max: state = min/max(state, arrow min/max(block))   (None when empty)
//   Sum:     state = state + arrow sum(block)               (None when empty;
//            any later None / None state -> to_array error)
void AggregatorFunction::accumulate_summary(const fq_agg_state &st) {
    if (st.blocks == 0) return;
    if (st.flags & FQ_STATE_DIV_ZERO) throw_status(FQ_E_DIVIDE_BY_ZERO, "Internal Error: Divide by zero error");
    if (st.flags & FQ_STATE_CAST_NULL)
        throw_status(FQ_E_UNSUPPORTED, "cast produced nulls (nulls are not supported on the device path)");
    switch (op_) {
        case FQ_AGG_COUNT:
            state_ = data_value_arithmetic_op(FQ_OP_ADD, state_, DataValue::u64(st.count));
            return;
        case FQ_AGG_MIN:
        case FQ_AGG_MAX: {
            const DataValue d = st.count ? DataValue::some(st.dtype, op_ == FQ_AGG_MAX ? st.max : st.min)
                                         : DataValue::none(st.dtype);
            state_ = data_value_aggregate_op(op_, state_, d);
            return;
        }
        default: {
            if (st.blocks == 1) {
                const DataValue d = st.count ? DataValue::some(st.dtype, st.sum) : DataValue::none(st.dtype);
                state_ = data_value_arithmetic_op(FQ_OP_ADD, state_, d);
                return;
            }
            if (st.flags & FQ_STATE_ANY_EMPTY) {
                // some block's sum is None and there are >= 2 blocks: the add
                // that meets it fails in to_array (data_value.rs:104-109)
                throw_internal("DataValue to array cannot be NONE NULL");
            }
            state_ = data_value_arithmetic_op(FQ_OP_ADD, state_, DataValue::some(st.dtype, st.sum));
            return;
        }
    }
}

static uint32_t scan_mask(uint32_t op) { return op | FQ_AGG_COUNT; }

static fq_agg_state run_scan(const Column &col, int64_t block_rows, const fq_pred *pred, const fq_expr *value,
                             uint32_t mask, ExecCtx &ctx) {
    auto out = DeviceBuffer::alloc(sizeof(fq_agg_state), ctx.stream());
    fq_col c = col.abi();
    check_fq(fq_aggregate(&c, block_rows, pred, value, mask, (fq_agg_state *)out->ptr, ctx.res->ws,
                          ctx.res->ws_bytes, ctx.stream()));
    fq_agg_state st{};
    check_hip(hipMemcpyAsync(&st, out->ptr, sizeof st, hipMemcpyDeviceToHost, ctx.stream()), "hipMemcpyAsync");
    ctx.sync();
    ctx.rt->stats.scan_launches++;
    ctx.rt->stats.scan_rows += (uint64_t)col.len;
    ctx.rt->stats.scan_bytes += (uint64_t)col.len * (uint64_t)dtype_size(col.dtype);
    return st;
}

static DataBlock compact_block(const DataBlock &b, const Column &bitmap, ExecCtx &ctx);

fq_agg_state AggregatorFunction::summarize(const DataBlock &b, ExecCtx &ctx) {
    const DataSchema &s = *b.schema;
    const uint64_t k = b.sub_blocks();
    const int64_t rows = b.columns.empty() ? 0 : b.columns[0].len;
    const int64_t R = b.sub_block_rows > 0 ? b.sub_block_rows : (rows > 0 ? rows : 1);
    FusedChain fc;
    FusedPred fp;
    const bool chain = arg_->to_chain(s, fc);
    const bool pred_ok = !b.filter || (b.filter->to_pred(s, fp) && chain && fp.column == fc.column);
    if (chain && pred_ok) {
        fq_agg_state st = run_scan(b.column_by_name(fc.column), R, b.filter ? fp.get() : nullptr,
                                   fc.expr.n_steps ? &fc.expr : nullptr, scan_mask(op_), ctx);
        st.blocks = k;
        return st;
    }
    // general path: materialise what the reference would evaluate
    DataBlock fb = b;
    fq_agg_state info{};
    if (b.filter) {
        DataBlock nb = b;
        nb.filter = nullptr;
        Column bm = eval_predicate(*b.filter, nb, ctx);
        fq_pred bp{};
        bp.kind = FQ_PRED_BITMAP;
        bp.bitmap = (const uint64_t *)bm.dptr();
        Column probe;
        for (const Column &c : nb.columns)
            if (c.on_device() && dtype_is_numeric(c.dtype)) {
                probe = c;
                break;
            }
        if (!probe.on_device()) throw_status(FQ_E_UNSUPPORTED, "filtered aggregate needs a numeric device column");
        info = run_scan(probe, R, &bp, nullptr, FQ_AGG_SUM | FQ_AGG_COUNT, ctx);
        fb = compact_block(nb, bm, ctx);
    }
    const ColumnarValue v = arg_->eval(fb, ctx);
    const int64_t frows = fb.num_rows();
    const DataType vdt = v.data_type();
    fq_agg_state st{};
    if (!dtype_is_numeric(vdt)) {
        if (op_ != FQ_AGG_COUNT)  // data_array_aggregate.rs:155-160
            throw_internal(std::string("Unsupported data_array_") + agg_op_name(op_) + " for data type: " +
                           dtype_name(vdt));
        if (!v.is_array) none_check(v);
        st.count = (uint64_t)frows;
        st.dtype = vdt;
    } else {
        const Column vc = v.to_array(frows, ctx);
        st = run_scan(vc, vc.len > 0 ? vc.len : 1, nullptr, nullptr, scan_mask(op_), ctx);
    }
    st.blocks = k;
    if (b.filter) st.flags |= info.flags & FQ_STATE_ANY_EMPTY;
    return st;
}

// ---------------------------------------------------------------------------
// LogicFunction (function_logic.rs:47-94, data_array_logic.rs:10-31)
// ---------------------------------------------------------------------------
static const char *logic_op_str(int32_t op) { return op == FQ_LOGIC_AND ? "and" : "or"; }

std::string LogicFunction::display() const {
    return left_->display() + " " + logic_op_str(op_) + " " + right_->display();
}

ColumnarValue LogicFunction::eval(const DataBlock &b, ExecCtx &ctx) {
    ColumnarValue l = left_->eval(b, ctx);
    ColumnarValue r = right_->eval(b, ctx);
    if (!l.is_array || !r.is_array)
        throw_internal(std::string("Cannot do data_array ") + logic_op_str(op_) + ", left:" +
                       dtype_name(l.data_type()) + ", right:" + dtype_name(r.data_type()));
    for (const ColumnarValue *v : {&l, &r})  // downcast_array! (macros.rs:5-16)
        if (v->array.dtype != FQ_DT_BOOLEAN)
            throw_internal(std::string("Cannot downcast_array from datatype:") + dtype_name(v->array.dtype) +
                           " item to:BooleanArray");
    if (l.array.len != r.array.len) throw_internal("Cannot perform bitwise operation on arrays of different length");
    Column out = Column::device(FQ_DT_BOOLEAN, l.array.len, ctx.stream());
    check_fq(fq_logic(op_, (const uint64_t *)l.array.dptr(), (const uint64_t *)r.array.dptr(), (uint64_t *)out.dptr(),
                      l.array.len, ctx.stream()));
    ColumnarValue v;
    v.is_array = true;
    v.array = out;
    return v;
}

std::vector<DataValue> LogicFunction::accumulate_result() const {
    throw_internal(std::string("Unsupported aggregate operation for function ") + logic_op_str(op_));
}
void LogicFunction::merge_state(const std::vector<DataValue> &) {
    throw_internal(std::string("Unsupported aggregate operation for function ") + logic_op_str(op_));
}
DataValue LogicFunction::merge_result() const {
    throw_internal(std::string("Unsupported aggregate operation for function ") + logic_op_str(op_));
}

// An and/or tree of fusable comparisons over one column -> FQ_PRED_TREE
// (postfix program over at most FQ_MAX_PRED_LEAVES leaves).
static bool flatten_logic(const Function &f, const DataSchema &s, FusedPred &out, std::vector<FusedPred> &leaves,
                          std::vector<int32_t> &prog) {
    if (const auto *lf = dynamic_cast<const LogicFunction *>(&f)) {
        if (!flatten_logic(lf->left(), s, out, leaves, prog) || !flatten_logic(lf->right(), s, out, leaves, prog))
            return false;
        prog.push_back(lf->op() == FQ_LOGIC_AND ? FQ_PRED_AND : FQ_PRED_OR);
        return true;
    }
    FusedPred p;
    if (!f.to_pred(s, p) || p.pred.kind != FQ_PRED_EXPR) return false;
    if (leaves.size() >= FQ_MAX_PRED_LEAVES) return false;
    if (!leaves.empty() && p.column != leaves[0].column) return false;
    prog.push_back((int32_t)leaves.size());
    leaves.push_back(p);
    return true;
}

bool LogicFunction::to_pred(const DataSchema &s, FusedPred &p) const {
    std::vector<FusedPred> leaves;
    std::vector<int32_t> prog;
    if (!flatten_logic(*this, s, p, leaves, prog) || leaves.empty()) return false;
    p = FusedPred{};
    p.column = leaves[0].column;
    p.col_dtype = leaves[0].col_dtype;
    p.pred.kind = FQ_PRED_TREE;
    p.tree.n_leaves = (int32_t)leaves.size();
    p.tree.n_prog = (int32_t)prog.size();
    for (size_t i = 0; i < prog.size(); ++i) p.tree.prog[i] = prog[i];
    for (size_t i = 0; i < leaves.size(); ++i) {
        const fq_pred &q = leaves[i].pred;
        fq_pred_leaf &l = p.tree.leaves[i];
        l.cmp = q.cmp;
        l.cmp_dtype = q.cmp_dtype;
        l.rhs_operand = q.rhs_operand;
        l.rhs_bits = q.rhs_bits;
        l.lhs = q.lhs;
    }
    return true;
}

// ---------------------------------------------------------------------------
// factory (function_factory.rs:14-40)
// ---------------------------------------------------------------------------
FunctionRef function_factory(const std::string &name, std::vector<FunctionRef> args, const FactoryOptions &o) {
    std::string n = name;
    std::transform(n.begin(), n.end(), n.begin(), [](unsigned char c) { return (char)tolower(c); });
    auto need = [&](size_t k) {
        if (args.size() < k)
            throw_internal("index out of bounds: the len is " + std::to_string(args.size()) + " but the index is " +
                           std::to_string(k - 1));
    };
    int32_t op = -1, cmp = -1;
    uint32_t agg = 0;
    if (n == "+") op = FQ_OP_ADD;
    else if (n == "-") op = FQ_OP_SUB;
    else if (n == "*") op = FQ_OP_MUL;
    else if (n == "/") op = FQ_OP_DIV;
    else if (n == "%" && o.modulo) op = FQ_OP_MOD;
    else if (n == "=") cmp = FQ_CMP_EQ;
    else if (n == "<") cmp = FQ_CMP_LT;
    else if (n == ">") cmp = FQ_CMP_GT;
    else if (n == "<=") cmp = FQ_CMP_LTEQ;
    else if (n == ">=") cmp = FQ_CMP_GTEQ;
    else if (n == "count") agg = FQ_AGG_COUNT;
    else if (n == "min") agg = FQ_AGG_MIN;
    else if (n == "max") agg = FQ_AGG_MAX;
    else if (n == "sum") agg = FQ_AGG_SUM;
    else if (n == "and" || n == "or") {
        need(2);
        return std::make_shared<LogicFunction>(n == "and" ? FQ_LOGIC_AND : FQ_LOGIC_OR, args[0], args[1]);
    } else throw_internal("Unsupported Function: " + name);
    if (op >= 0) {
        need(2);
        return std::make_shared<ArithmeticFunction>(op, args[0], args[1]);
    }
    if (cmp >= 0) {
        need(2);
        return std::make_shared<ComparisonFunction>(cmp, args[0], args[1]);
    }
    need(1);
    return std::make_shared<AggregatorFunction>(agg, args[0]);
}

// ---------------------------------------------------------------------------
// predicate evaluation + compaction (FilterTransform::expression_executor)
// ---------------------------------------------------------------------------
// A predicate over one 64-bit device column as ONE hipRTC kernel
// (fq_predicate_bitmap) instead of a kernel per Function node; false when the
// shape is not fusable or the JIT is off/unavailable (the caller evaluates
// the Function tree).
static bool fused_predicate_bitmap(Function &pred, const DataBlock &b, ExecCtx &ctx, Column &out) {
    FusedPred fp;
    if (!b.schema || !pred.to_pred(*b.schema, fp)) return false;
    const Column &c = b.column_by_name(fp.column);
    if (!c.on_device() || dtype_size(c.dtype) != 8) return false;
    Column bm = Column::device(FQ_DT_BOOLEAN, c.len, ctx.stream());
    auto flag = DeviceBuffer::alloc(sizeof(uint32_t), ctx.stream());
    fq_col ic = c.abi();
    const fq_status st = fq_predicate_bitmap(&ic, fp.get(), (uint64_t *)bm.dptr(), (uint32_t *)flag->ptr, ctx.stream());
    if (st == FQ_E_UNSUPPORTED) return false;  // no hipRTC / JIT off / shape outside it: per node (same errors)
    check_fq(st);
    out = bm;
    return true;
}

Column eval_predicate(Function &pred, const DataBlock &b, ExecCtx &ctx) {
    Column fused;
    if (fused_predicate_bitmap(pred, b, ctx, fused)) return fused;
    const ColumnarValue v = pred.eval(b, ctx);
    const int64_t rows = b.num_rows();
    if (!v.is_array) {
        if (v.scalar.kind == DataValue::kSome && v.scalar.dtype == FQ_DT_BOOLEAN) return value_to_array(v.scalar, rows, ctx);
        throw_internal("cannot downcast to boolean array");
    }
    if (v.array.dtype != FQ_DT_BOOLEAN) throw_internal("cannot downcast to boolean array");
    return v.array;
}

static DataBlock compact_block(const DataBlock &b, const Column &bitmap, ExecCtx &ctx) {
    DataBlock out;
    out.schema = b.schema;
    out.sub_block_rows = 0;
    const int64_t n = b.num_rows();
    const size_t wsb = fq_filter_workspace_bytes(n);
    auto ws = DeviceBuffer::alloc(wsb, ctx.stream());
    std::vector<uint8_t> hbits;
    for (const Column &c : b.columns) {
        if (c.on_device() && c.dtype != FQ_DT_BOOLEAN) {
            Column o = Column::device(c.dtype, n, ctx.stream());
            fq_col ic = c.abi();
            int64_t kept = 0;
            check_fq(fq_filter_compact(&ic, (const uint64_t *)bitmap.dptr(), o.dptr(), &kept, ws->ptr, wsb, ctx.stream()));
            o.len = kept;
            out.columns.push_back(o);
            continue;
        }
        // host / Boolean / Null columns: select on the host
        if (hbits.empty()) {
            std::vector<DataValue> bv = bitmap.to_host(ctx.stream());
            hbits.resize(bv.size());
            for (size_t i = 0; i < bv.size(); ++i) hbits[i] = (uint8_t)bv[i].bits;
        }
        std::vector<DataValue> rows = c.to_host(ctx.stream());
        std::vector<DataValue> kept;
        for (size_t i = 0; i < rows.size() && i < hbits.size(); ++i)
            if (hbits[i]) kept.push_back(rows[i]);
        if (c.dtype == FQ_DT_NULL) {
            Column nc;
            nc.dtype = FQ_DT_NULL;
            int64_t cnt = 0;
            for (auto h : hbits) cnt += h;
            nc.len = cnt;
            out.columns.push_back(nc);
        } else {
            out.columns.push_back(Column::host_values(c.dtype, std::move(kept)));
        }
    }
    return out;
}

// A block stream's valid rows into plain columns (fq_blocks_compact).
static DataBlock compact_layout(const DataBlock &b, ExecCtx &ctx) {
    const BlockLayout &L = *b.layout;
    DataBlock nb = b;
    nb.layout = nullptr;
    nb.ready = false;  // the compaction below is new device work
    std::vector<const void *> in;
    std::vector<void *> out;
    for (auto &c : nb.columns) {
        if (dtype_size(c.dtype) != 8 || c.dtype == FQ_DT_BOOLEAN || !c.on_device())
            throw_internal("block-stream layout over a column that is not 64-bit device data");
        in.push_back(c.dptr());
        Column o = Column::device(c.dtype, L.rows, ctx.stream());
        out.push_back(o.dptr());
        c = o;
    }
    const int64_t len = b.columns.empty() ? 0 : b.columns[0].len;
    const size_t wsb = fq_blocks_compact_workspace_bytes(L.n_blocks);
    auto ws = DeviceBuffer::alloc(wsb, ctx.stream());
    check_fq(fq_blocks_compact((int32_t)in.size(), in.data(), len, L.block_rows, (const int64_t *)L.counts->ptr,
                               out.data(), nullptr, ws->ptr, wsb, ctx.stream()));
    return nb;
}

DataBlock materialize(const DataBlock &b, ExecCtx &ctx) {
    if (b.layout) return compact_layout(b, ctx);
    if (!b.filter) return b;
    DataBlock nb = b;
    nb.filter = nullptr;
    nb.ready = false;
    Column bm = eval_predicate(*b.filter, nb, ctx);
    return compact_block(nb, bm, ctx);
}

// FilterTransform -> ProjectionTransform over a block that stands for a run of
// reference blocks (sub_block_rows, numbers_stream.rs:29-48): the reference
// filters and projects each 10,000-row block on its own
// (stream_expression.rs:38-50), so the output keeps that geometry -- block b's
// kept rows at rows [b * B, b * B + count[b]) -- and no block waits on another's
// count (fqk::filter_project_blocks_enqueue).  The launch is enqueued with the
// queue's other pipes (launch_mu) and this pipe waits for its own launch, not
// for the queue.
//
// Around each projection kernel the queue carries only a one-thread hand-off
// kernel: it moves {kept rows, flag words} into the worker's pinned, mapped
// result words and re-zeroes the worker's resident workspace (no memset before,
// no copy after), then the pipe's completion event.  In one process, 4 rounds x
// 8 queries of p1 (profiles/r06_a_p1_queue_ab.json, r06_d_p1_queue_ab_span.json):
// memset + copy 24.36 / 23.52 ms per query, this 23.94 / 23.33, the hand-off
// alone with the pipe polling the words 24.03 / 23.52 -- the first pair with an
// event pair around every launch, the second with one span per query.
static bool project_blocks(const DataBlock &b, const Column &c, const fq_pred *pred, std::vector<fq_expr> &exprs,
                           std::vector<Column> &outs, std::vector<void *> &ptrs, const SchemaRef &schema, ExecCtx &ctx,
                           DataBlock &out, LaunchSpan *span) {
    const int64_t n = c.len, B = b.sub_block_rows;
    const int64_t nb = n <= B ? 1 : (n + B - 1) / B;
    auto layout = std::make_shared<BlockLayout>();
    layout->block_rows = B;
    layout->n_blocks = n == 0 ? 0 : nb;
    layout->counts = DeviceBuffer::alloc((size_t)std::max<int64_t>(nb, 1) * 8, ctx.stream());
    // the map kernel (no predicate) has its words written by the host and no
    // hand-off: a workspace of its own, zeroed before it, the flags copied after
    const bool resident = pred && pred->kind != FQ_PRED_NONE;
    ctx.res->project_resident(ctx.stream());
    uint64_t *res = ctx.res->project_res;
    std::shared_ptr<DeviceBuffer> ws;
    if (!resident) ws = DeviceBuffer::alloc(fq_filter_project_blocks_workspace_bytes(), ctx.stream());
    // FQ_OPT_PROFILE 1: an event pair around each kernel; 2 with a span: none
    // here (LaunchSpan times the query's launches together)
    const int profile = ctx.rt->profile.load();
    const bool prof = profile == 1 || (profile == 2 && !span);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (prof) {
        e0 = ctx.res->take_event();
        e1 = ctx.res->take_event();
    }
    fq_col ic = c.abi();
    // the shape's kernel compiled (first use: hipRTC, ~0.2 s) before the
    // queue's launch lock is taken: a zero-length call only prepares it
    fq_col none = ic;
    none.len = 0;
    fq_status st = fqk::filter_project_blocks_enqueue(&none, B, pred, exprs.data(), (int32_t)exprs.size(), ptrs.data(),
                                                      nullptr, res, nullptr, nullptr, 0, nullptr, nullptr, ctx.stream());
    if (st == FQ_E_UNSUPPORTED) return false;
    check_fq(st);
    hipEvent_t done = ctx.res->take_sync_event();
    {
        std::lock_guard<std::mutex> lk(*ctx.launch_mu());
        if (span) span->before_launch(ctx);
        // this worker's last hand-off has landed (the pipe waited for it); an
        // empty block launches nothing, so its words must read 0 kept rows
        res[0] = res[1] = 0;
        st = fqk::filter_project_blocks_enqueue(&ic, B, pred, exprs.data(), (int32_t)exprs.size(), ptrs.data(),
                                                (int64_t *)layout->counts->ptr, res,
                                                resident ? ctx.res->project_dres : nullptr,
                                                resident ? ctx.res->project_ws : ws->ptr,
                                                fq_filter_project_blocks_workspace_bytes(), e0, e1, ctx.stream());
        if (st == FQ_OK) check_hip(hipEventRecord(done, ctx.stream()), "hipEventRecord");  // after the result words
    }
    if (st == FQ_OK) {
        const hipError_t he = hipEventSynchronize(done);
        if (he == hipSuccess && prof) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess) ctx.rt->stats.project_ns += (uint64_t)((double)ms * 1e6);
        }
        check_hip(he, "hipEventSynchronize");
    }
    if (e0) ctx.res->give_event(e0);
    if (e1) ctx.res->give_event(e1);
    ctx.res->give_sync_event(done);
    if (st == FQ_E_UNSUPPORTED) return false;  // the unfused path evaluates it (and raises what the reference does)
    check_fq(st);
    int64_t kept = 0;
    check_fq(fqk::filter_project_blocks_result(res, &kept));
    layout->rows = kept;
    auto &S = ctx.rt->stats;
    S.project_launches++;
    S.project_rows += (uint64_t)n;
    S.project_kept += (uint64_t)kept;
    S.project_bytes += (uint64_t)n * (uint64_t)dtype_size(c.dtype) + (uint64_t)kept * 8 * (uint64_t)outs.size();
    out = DataBlock{};
    out.schema = schema;
    out.sub_block_rows = B;
    out.layout = layout;
    out.ready = true;  // this pipe waited for the launch above
    for (auto &o : outs) out.columns.push_back(o);
    return true;
}

// ProjectionTransform over a block with a pending filter (or none): when every
// projected expression is a chain over the same 64-bit device column, one
// fq_filter_project call compacts and evaluates them together (the predicate
// fused too when it is over that column, else its bitmap is evaluated
// first).  false: not fusable, the caller materialises + evaluates.
bool project_fused(const DataBlock &b, const std::vector<FunctionRef> &funcs, const SchemaRef &schema, ExecCtx &ctx,
                   DataBlock &out, bool block_stream, LaunchSpan *span) {
    if (funcs.empty() || funcs.size() > FQ_MAX_PROJECT || !b.schema || b.columns.empty()) return false;
    std::vector<FusedChain> chains(funcs.size());
    bool computes = false;
    for (size_t j = 0; j < funcs.size(); ++j) {
        if (!funcs[j]->to_chain(*b.schema, chains[j])) return false;
        if (chains[j].column != chains[0].column || dtype_size(chains[j].out_dtype) != 8) return false;
        computes |= chains[j].expr.n_steps > 0;
    }
    if (!b.filter && !computes) return false;  // plain column references: zero-copy in the unfused path
    const Column &c = b.column_by_name(chains[0].column);
    if (!c.on_device() || dtype_size(c.dtype) != 8 || c.dtype == FQ_DT_BOOLEAN) return false;
    fq_jit_stats js{};
    if (fq_jit_get_stats(&js) != FQ_OK || js.mode == FQ_JIT_OFF || js.available == 0) return false;
    FusedPred fp;
    fq_pred bp{};
    const fq_pred *pred = nullptr;
    Column bm;
    if (b.filter) {
        if (b.filter->to_pred(*b.schema, fp) && fp.column == chains[0].column) {
            pred = fp.get();
        } else {
            DataBlock nb = b;
            nb.filter = nullptr;
            bm = eval_predicate(*b.filter, nb, ctx);
            bp.kind = FQ_PRED_BITMAP;
            bp.bitmap = (const uint64_t *)bm.dptr();
            pred = &bp;
        }
    }
    const int64_t n = c.len;
    std::vector<Column> outs;
    std::vector<void *> ptrs;
    std::vector<fq_expr> exprs;
    for (auto &fc : chains) {
        outs.push_back(Column::device(fc.out_dtype, n, ctx.stream()));
        ptrs.push_back(outs.back().dptr());
        exprs.push_back(fc.expr);
    }
    if (block_stream && pred && b.sub_block_rows >= FQ_PROJECT_MIN_BLOCK_ROWS)
        return project_blocks(b, c, pred, exprs, outs, ptrs, schema, ctx, out, span);
    const size_t wsb = fq_filter_project_workspace_bytes(n);
    auto ws = DeviceBuffer::alloc(wsb, ctx.stream());
    fq_col ic = c.abi();
    int64_t kept = 0;
    const fq_status st = fq_filter_project(&ic, pred, exprs.data(), (int32_t)exprs.size(), ptrs.data(), &kept, ws->ptr,
                                           wsb, ctx.stream());
    if (st == FQ_E_UNSUPPORTED) return false;  // the unfused path evaluates it (and raises what the reference does)
    check_fq(st);
    out = DataBlock{};
    out.schema = schema;
    out.sub_block_rows = 0;
    for (auto &o : outs) {
        o.len = kept;
        out.columns.push_back(o);
    }
    return true;
}

// ---------------------------------------------------------------------------
// LaunchSpan
// ---------------------------------------------------------------------------
LaunchSpan::~LaunchSpan() {
    for (auto &s : queues_) rt_->give_event(s.start);
}

void LaunchSpan::before_launch(ExecCtx &ctx) {
    if (rt_->profile.load(std::memory_order_relaxed) != 2) return;
    std::lock_guard<std::mutex> lk(mu_);
    for (const QueueSpan &s : queues_)
        if (s.q == ctx.stream()) return;
    QueueSpan s;
    s.q = ctx.stream();
    s.launch_mu = ctx.launch_mu();
    s.start = rt_->take_event();
    check_hip(hipEventRecord(s.start, s.q), "hipEventRecord");
    queues_.push_back(s);
}

void LaunchSpan::arrive() noexcept {
    std::vector<QueueSpan> qs;
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (--left_ != 0) return;
        qs = queues_;
    }
    // the last pipe: every launch of the query has completed (each pipe waited
    // for its own); one end event per queue closes its span.  The query's
    // span is the union over its queues (the row queues' launches overlap):
    // earliest start to latest end, both measured from the first queue's start.
    if (qs.empty()) return;
    float lo = 0, hi = 0;
    bool ok = true;
    for (QueueSpan &s : qs) {
        hipEvent_t end = nullptr;
        try {
            end = rt_->take_event();
            {
                std::lock_guard<std::mutex> ql(*s.launch_mu);
                ok = ok && hipEventRecord(end, s.q) == hipSuccess;
            }
            float a = 0, b = 0;
            ok = ok && hipEventSynchronize(end) == hipSuccess &&
                 hipEventElapsedTime(&a, qs[0].start, s.start) == hipSuccess &&
                 hipEventElapsedTime(&b, qs[0].start, end) == hipSuccess;
            lo = std::min(lo, a);
            hi = std::max(hi, b);
        } catch (...) {  // timing only: never fail the query for it
            ok = false;
        }
        if (end) rt_->give_event(end);
    }
    (void)hipGetLastError();
    if (ok) rt_->stats.project_ns += (uint64_t)((double)(hi - lo) * 1e6);
}

// ---------------------------------------------------------------------------
// ScanGroup
// ---------------------------------------------------------------------------
ScanGroup::~ScanGroup() {
    for (auto &s : queues_) {
        rt_->give_event(s.start);
        rt_->give_event(s.end);
    }
}

void ScanGroup::before_launch(ExecCtx &ctx) {
    std::lock_guard<std::mutex> lk(mu_);
    for (const QueueSpan &s : queues_)
        if (s.q == ctx.stream()) return;
    QueueSpan s;
    s.q = ctx.stream();
    s.launch_mu = ctx.launch_mu();
    if (rt_->profile.load() == 2) {  // the span opens right before this queue's first scan
        s.start = rt_->take_event();
        check_hip(hipEventRecord(s.start, s.q), "hipEventRecord");
    }
    queues_.push_back(s);
}

void ScanGroup::arrive(bool wait) noexcept {
    std::unique_lock<std::mutex> lk(mu_);
    if (--left_ > 0) {
        if (wait) cv_.wait(lk, [&] { return closed_; });
        return;
    }
    // the last pipe: every pipe has enqueued its scans, so queues_ no longer
    // changes; the end events are recorded without mu_ held (before_launch
    // takes mu_ under a queue's launch lock)
    std::vector<QueueSpan> qs = queues_;
    lk.unlock();
    std::string err;
    for (QueueSpan &s : qs) {
        try {
            std::lock_guard<std::mutex> ql(*s.launch_mu);
            s.end = rt_->take_event();
            check_hip(hipEventRecord(s.end, s.q), "hipEventRecord");
        } catch (const std::exception &e) {
            // this queue's end is unknown: wait_end synchronises the queue itself
            if (err.empty()) err = e.what();
            if (s.end) rt_->give_event(s.end);
            s.end = nullptr;
        } catch (...) {
            if (err.empty()) err = "Internal Error: unknown exception recording a scan group's end";
            s.end = nullptr;
        }
    }
    lk.lock();
    queues_ = qs;
    arrive_error_ = err;
    closed_ = true;
    cv_.notify_all();
}

// ONE pipe waits on the end events; the others sleep on the group's condition
// and are woken together.  Eight threads in hipEventSynchronize on one event
// were released one by one, ~15 us apart: ~100 us at the end of every C3
// query (profiles/r05_c_c3_query_timeline.txt).
void ScanGroup::wait_end() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return closed_; });  // every pipe has arrived: the end events exist
    if (waiter_) {
        cv_.wait(lk, [&] { return ended_; });
        if (end_error_ != hipSuccess) check_hip(end_error_, "hipEventSynchronize");
        if (!arrive_error_.empty()) throw FQException(FQ_E_HIP, arrive_error_);
        return;
    }
    waiter_ = true;
    std::vector<QueueSpan> qs = queues_;
    lk.unlock();
    hipError_t err = hipSuccess;
    for (const QueueSpan &s : qs)
        if (err == hipSuccess) err = s.end ? hipEventSynchronize(s.end) : hipStreamSynchronize(s.q);
    if (rt_->profile.load(std::memory_order_relaxed) == 2) rt_->stats.scan_end_seen = now_ns();
    lk.lock();
    ended_ = true;
    end_error_ = err;
    cv_.notify_all();
    const std::string arrive_error = arrive_error_;
    lk.unlock();
    check_hip(err, "hipEventSynchronize");
    if (!arrive_error.empty()) throw FQException(FQ_E_HIP, arrive_error);
}

void ScanGroup::account() {
    std::lock_guard<std::mutex> lk(mu_);
    if (accounted_) return;
    accounted_ = true;
    for (const QueueSpan &s : queues_) {
        float ms = 0;
        if (s.start && s.end && hipEventElapsedTime(&ms, s.start, s.end) == hipSuccess)
            rt_->stats.scan_ns += (uint64_t)((double)ms * 1e6);
    }
}

// ---------------------------------------------------------------------------
// AggFusion
// ---------------------------------------------------------------------------
AggFusion::AggFusion(ExecCtx &ctx, ScanTicket *ticket)
    : ctx_(ctx), rt_(ctx.rt), res_(ctx.res), stream_(ctx.stream()), launch_mu_(ctx.launch_mu()), ticket_(ticket) {}

AggFusion::~AggFusion() {
    // an exception left scans in flight: they write into this worker's pinned
    // slots, which the next query reuses -- let them land first
    if (launched_ && !finished_) {
        try {
            wait_launched();
        } catch (...) {
        }
    }
    for (auto &p : events_) {
        res_->give_event(p.first);
        res_->give_event(p.second);
    }
}

fq_agg_state *AggFusion::slot_host(size_t k) const {
    return res_->slot_chunks[k / WorkerRes::kSlotChunk] + k % WorkerRes::kSlotChunk;
}

size_t AggFusion::alloc_slot() {
    const size_t k = nslots_++;
    auto &chunks = ctx_.res->slot_chunks;
    while (chunks.size() * WorkerRes::kSlotChunk <= k) {
        void *p = nullptr;
        check_hip(hipHostMalloc(&p, WorkerRes::kSlotChunk * sizeof(fq_agg_state),
                                hipHostMallocMapped | hipHostMallocCoherent),
                  "hipHostMalloc(result slots)");
        chunks.push_back((fq_agg_state *)p);
    }
    return k;
}

void AggFusion::wait_launched() {
    hipEvent_t done = res_->take_sync_event();
    {
        std::lock_guard<std::mutex> lk(*launch_mu_);
        check_hip(hipEventRecord(done, stream_), "hipEventRecord");
    }
    hipError_t e = hipEventSynchronize(done);
    res_->give_sync_event(done);
    check_hip(e, "hipEventSynchronize");
}

void AggFusion::add_error(const FQException &e) {
    Entry en;
    en.has_error = true;
    en.err = e;
    log_.push_back(en);
}

void AggFusion::add(AggregatorFunction *agg, const DataBlock &b) {
    const DataSchema &s = *b.schema;
    FusedChain fc;
    FusedPred fp;
    bool ok = agg->arg().to_chain(s, fc);
    if (ok && b.filter) ok = b.filter->to_pred(s, fp) && fp.column == fc.column;
    if (!ok) {
        Entry en;
        en.agg = agg;
        try {
            en.st = agg->summarize(b, ctx_);
        } catch (const FQException &e) {
            en.has_error = true;
            en.err = e;
        }
        log_.push_back(en);
        return;
    }
    const std::string key = fc.key() + "|" + (b.filter ? fp.key() : std::string());
    Group *g = nullptr;
    for (auto &x : cur_)
        if (x.key == key) g = &x;
    if (!g) {
        cur_.emplace_back();
        g = &cur_.back();
        g->key = key;
        g->col = b.column_by_name(fc.column);
        g->value = fc;
        g->has_pred = (bool)b.filter;
        if (g->has_pred) g->pred = fp;
        g->filter_keepalive = b.filter;
        const int64_t rows = g->col.len;
        g->block_rows = b.sub_block_rows > 0 ? b.sub_block_rows : (rows > 0 ? rows : 1);
        g->blocks = b.sub_blocks();
        g->slot = alloc_slot();
    }
    g->mask |= scan_mask(agg->op());
    Entry en;
    en.agg = agg;
    en.slot = g->slot;
    en.st.blocks = g->blocks;
    log_.push_back(en);
}

void AggFusion::end_block() {
    const int prof = ctx_.rt->profile.load();
    // an event pair per scan; 2: one span per query when the query's pipes
    // form a ScanGroup (a Function-handle call has none: pairs)
    const bool pairs = prof == 1 || (prof == 2 && !(ticket_ && ticket_->group()));
    for (Group &g : cur_) {
        fq_col c = g.col.abi();
        void *dst = nullptr;
        check_hip(hipHostGetDevicePointer(&dst, slot_host(g.slot), 0), "hipHostGetDevicePointer");
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (pairs) {
            e0 = ctx_.res->take_event();
            e1 = ctx_.res->take_event();
        }
        if (prof && (g.has_pred || g.value.expr.n_steps)) {
            // compile a specialised scan (first use of this expression shape)
            // outside the timed region (identity scans are precompiled)
            fq_jit_stats js;
            if (fq_jit_get_stats(&js) == FQ_OK &&
                (js.mode == FQ_JIT_ALWAYS || (js.mode == FQ_JIT_AUTO && c.len >= js.min_rows)))
                check_fq(fq_jit_prepare(&c, g.block_rows, g.has_pred ? g.pred.get() : nullptr,
                                        g.value.expr.n_steps ? &g.value.expr : nullptr, g.mask, nullptr));
        }
        {
            // events and the scan enqueue back to back even when other pipes
            // share this queue, so an event pair brackets this scan
            std::lock_guard<std::mutex> lk(*ctx_.launch_mu());
            const fq_pred *pred = g.has_pred ? g.pred.get() : nullptr;
            const fq_expr *val = g.value.expr.n_steps ? &g.value.expr : nullptr;
            if (ticket_ && ticket_->group()) ticket_->group()->before_launch(ctx_);
            if (pairs) check_hip(hipEventRecord(e0, stream_), "hipEventRecord");
            check_fq(fq_aggregate(&c, g.block_rows, pred, val, g.mask, (fq_agg_state *)dst, res_->ws, res_->ws_bytes,
                                  stream_));
            if (pairs) check_hip(hipEventRecord(e1, stream_), "hipEventRecord");
        }
        launched_ = true;
        if (const int64_t q0 = ctx_.rt->stats.query_t0.exchange(0))
            ctx_.rt->stats.first_launch_ns += (uint64_t)(now_ns() - q0);
        if (pairs) events_.push_back({e0, e1});
        ctx_.rt->stats.scan_launches++;
        ctx_.rt->stats.scan_rows += (uint64_t)g.col.len;
        ctx_.rt->stats.scan_bytes += (uint64_t)g.col.len * (uint64_t)dtype_size(g.col.dtype);
        // a stream-ordered column (hipFreeAsync on the queue the scan was just
        // enqueued on) may be dropped now: its memory returns to the pool only
        // after the scan -- so a query over generated chunks holds one chunk per
        // pipe, not all of them; a synchronously allocated one is kept to finish()
        if (g.col.dev && !g.col.dev->async) keepalive_.push_back(g.col);
    }
    cur_.clear();
}

void AggFusion::finish() {
    end_block();
    if (ticket_ && ticket_->group()) {
        // the query's pipes wait together on one event behind the last scan
        ticket_->arrive(launched_);
    } else if (launched_) {
        // only this pipe's scans, not the whole queue: with profiling the last
        // scan's closing timing event already marks that point (no extra marker)
        if (!events_.empty()) check_hip(hipEventSynchronize(events_.back().second), "hipEventSynchronize");
        else wait_launched();
    }
    replay();
}

bool AggFusion::finish_deferred() {
    end_block();
    if (!launched_ || !ticket_ || !ticket_->group()) return false;
    ticket_->arrive_only();
    ticket_ = nullptr;  // the ticket lives on the pipe's stack
    return true;
}

void AggFusion::replay() {
    finished_ = true;
    for (auto &p : events_) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess)
            rt_->stats.scan_ns += (uint64_t)((double)ms * 1e6);
    }
    keepalive_.clear();
    // each device slot (pinned host memory the scans' folds wrote) read once:
    // the aggregators of one fused scan share it
    std::vector<fq_agg_state> slots(nslots_);
    std::vector<char> have(nslots_, 0);
    for (Entry &en : log_) {
        if (en.has_error) throw en.err;
        fq_agg_state st = en.st;
        if (en.slot != (size_t)-1) {
            if (!have[en.slot]) {
                memcpy(&slots[en.slot], slot_host(en.slot), sizeof(fq_agg_state));
                have[en.slot] = 1;
            }
            st = slots[en.slot];
            st.blocks = en.st.blocks;
        }
        en.agg->accumulate_summary(st);
    }
}

}  // namespace fq
