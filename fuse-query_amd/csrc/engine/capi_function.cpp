// C ABI of the Function surface (include/fq_engine.h, "Function handles"):
// the engine's C++ Function objects (functions.h) behind opaque handles, so a
// host binds the reference's Function protocol (src/functions/function.rs:28-131)
// directly -- and so the reference's own protocol tests
// (function_aggregator_test.rs, data_value_*_test.rs) replay on the product.
#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "../fq_common.h"
#include "core.h"
#include "fq_engine.h"
#include "functions.h"

struct fq_function {
    fq::FunctionRef f;
};

// fq_engine is defined in capi_engine.cpp; the device calls here need its Runtime
fq::Runtime *fq_engine_runtime(fq_engine *e);

namespace {

template <typename F>
fq_status guard(F &&f) {
    try {
        f();
        return FQ_OK;
    } catch (const fq::FQException &e) {
        return fqc::fail(e.status, e.msg);
    } catch (const std::exception &e) {
        return fqc::internal(e.what());
    } catch (...) {
        return fqc::internal("unknown exception");
    }
}

fq::DataValue from_scalar(const fq_scalar &s) {
    switch (s.kind) {
        case FQ_SCALAR_NULL: return fq::DataValue::null();
        case FQ_SCALAR_NONE: return fq::DataValue::none(s.dtype);
        case FQ_SCALAR_SOME:
            if (s.dtype == FQ_DT_UTF8) return fq::DataValue::string(std::string(s.str ? s.str : "", s.str ? s.str_len : 0));
            if (s.dtype == FQ_DT_NULL || s.dtype > FQ_DT_UTF8 || s.dtype < 0)
                throw fq::FQException(FQ_E_INVALID, "fq_scalar: bad dtype");
            return fq::DataValue::some(s.dtype, s.bits);
        default: throw fq::FQException(FQ_E_INVALID, "fq_scalar: bad kind");
    }
}

// Returned Utf8 payloads live here until the thread's next returning call.
thread_local std::vector<std::string> t_strings;

fq_scalar to_scalar(const fq::DataValue &v) {
    fq_scalar s{};
    switch (v.kind) {
        case fq::DataValue::kNull: s.kind = FQ_SCALAR_NULL; return s;
        case fq::DataValue::kNone:
            s.kind = FQ_SCALAR_NONE;
            s.dtype = v.dtype;
            return s;
        case fq::DataValue::kSome:
            s.kind = FQ_SCALAR_SOME;
            s.dtype = v.dtype;
            if (v.dtype == FQ_DT_UTF8) {
                t_strings.push_back(v.str);
                s.str = t_strings.back().c_str();
                s.str_len = t_strings.back().size();
            } else {
                s.bits = v.bits;
            }
            return s;
        default: throw fq::FQException(FQ_E_UNSUPPORTED, "a Struct DataValue has no fq_scalar form");
    }
}

fq::SchemaRef block_schema(const fq_block &b) {
    if (b.n_columns < 0 || (b.n_columns > 0 && (!b.names || !b.columns)))
        throw fq::FQException(FQ_E_INVALID, "fq_block: bad columns");
    auto s = std::make_shared<fq::DataSchema>();
    for (int32_t i = 0; i < b.n_columns; ++i) {
        if (!b.names[i]) throw fq::FQException(FQ_E_INVALID, "fq_block: null column name");
        s->fields.push_back(fq::DataField{b.names[i], b.columns[i].dtype, false});
    }
    return s;
}

// The caller's columns, borrowed: the buffers are never freed or cached here.
// block_rows / filter become the DataBlock's reference-block geometry and its
// pending filter, exactly what a numbers_mt pipe hands AggregatePartial.
fq::DataBlock borrow_block(const fq_block &b) {
    fq::DataBlock blk;
    blk.schema = block_schema(b);
    if (b.block_rows < 0) throw fq::FQException(FQ_E_INVALID, "fq_block: negative block_rows");
    blk.sub_block_rows = b.block_rows;
    if (b.filter) blk.filter = b.filter->f->clone();
    for (int32_t i = 0; i < b.n_columns; ++i) {
        const fq_col &c = b.columns[i];
        if (c.len < 0 || (c.len > 0 && !c.data)) throw fq::FQException(FQ_E_INVALID, "fq_block: bad column");
        if (i > 0 && c.len != b.columns[0].len)
            throw fq::FQException(FQ_E_INVALID, "fq_block: columns of unequal length");
        if (!fq::dtype_is_numeric(c.dtype) && c.dtype != FQ_DT_BOOLEAN)
            throw fq::FQException(FQ_E_UNSUPPORTED, std::string("fq_block: device columns of ") +
                                                        fq::dtype_name(c.dtype) + " are not supported");
        fq::Column col;
        col.dtype = c.dtype;
        col.len = c.len;
        auto *db = new fq::DeviceBuffer();
        db->ptr = c.data;
        db->async = false;
        col.dev = std::shared_ptr<fq::DeviceBuffer>(db, [](fq::DeviceBuffer *p) {
            p->ptr = nullptr;  // borrowed
            delete p;
        });
        blk.columns.push_back(col);
    }
    return blk;
}

fq::Runtime *device_runtime(fq_engine *e) {
    fq::Runtime *rt = fq_engine_runtime(e);
    if (!rt->has_device())
        throw fq::FQException(FQ_E_HIP, "fq_engine: this engine has no device (created with device -1); "
                                        "the hot path has no CPU fallback");
    return rt;
}

}  // namespace

extern "C" {

fq_status fq_function_field(const char *name, fq_function **out) {
    if (!name || !out) return fqc::fail(FQ_E_INVALID, "fq_function_field: bad argument");
    *out = nullptr;
    return guard([&] { *out = new fq_function{std::make_shared<fq::FieldFunction>(name)}; });
}

fq_status fq_function_constant(const fq_scalar *value, fq_function **out) {
    if (!value || !out) return fqc::fail(FQ_E_INVALID, "fq_function_constant: bad argument");
    *out = nullptr;
    return guard([&] { *out = new fq_function{std::make_shared<fq::ConstantFunction>(from_scalar(*value))}; });
}

fq_status fq_function_create(const char *name, fq_function *const *args, int32_t n_args, fq_function **out) {
    if (!name || !out || n_args < 0 || (n_args > 0 && !args))
        return fqc::fail(FQ_E_INVALID, "fq_function_create: bad argument");
    *out = nullptr;
    return guard([&] {
        std::vector<fq::FunctionRef> fs;
        for (int32_t i = 0; i < n_args; ++i) {
            if (!args[i]) throw fq::FQException(FQ_E_INVALID, "fq_function_create: null argument");
            fs.push_back(args[i]->f->clone());  // try_create clones its args (function_arithmetic.rs:30-31)
        }
        *out = new fq_function{fq::function_factory(name, std::move(fs), fq::FactoryOptions{})};
    });
}

fq_status fq_function_clone(const fq_function *f, fq_function **out) {
    if (!f || !out) return fqc::fail(FQ_E_INVALID, "fq_function_clone: bad argument");
    *out = nullptr;
    return guard([&] { *out = new fq_function{f->f->clone()}; });
}

void fq_function_free(fq_function *f) { delete f; }

fq_status fq_function_display(const fq_function *f, char *buf, size_t cap, size_t *len) {
    if (!f || !len || (cap > 0 && !buf)) return fqc::fail(FQ_E_INVALID, "fq_function_display: bad argument");
    return guard([&] {
        const std::string s = f->f->display();
        *len = s.size();
        if (cap < s.size() + 1) throw fq::FQException(FQ_E_INVALID, "fq_function_display: buffer too small");
        memcpy(buf, s.c_str(), s.size() + 1);
    });
}

fq_status fq_function_set_depth(fq_function *f, uint64_t depth) {
    if (!f) return fqc::fail(FQ_E_INVALID, "fq_function_set_depth: bad argument");
    return guard([&] { f->f->set_depth((size_t)depth); });
}

fq_status fq_function_return_type(const fq_function *f, const fq_block *schema, int32_t *out) {
    if (!f || !schema || !out) return fqc::fail(FQ_E_INVALID, "fq_function_return_type: bad argument");
    return guard([&] { *out = f->f->return_type(*block_schema(*schema)); });
}

fq_status fq_function_nullable(const fq_function *f, const fq_block *schema, int32_t *out) {
    if (!f || !schema || !out) return fqc::fail(FQ_E_INVALID, "fq_function_nullable: bad argument");
    return guard([&] { *out = f->f->nullable(*block_schema(*schema)) ? 1 : 0; });
}

fq_status fq_function_eval(fq_engine *e, fq_function *f, const fq_block *b, void *d_out, size_t cap,
                           size_t *out_bytes, int32_t *out_dtype, int64_t *out_len, int32_t *is_array,
                           fq_scalar *scalar) {
    if (!e || !f || !b || !out_bytes || !out_dtype || !out_len || !is_array || !scalar)
        return fqc::fail(FQ_E_INVALID, "fq_function_eval: bad argument");
    return guard([&] {
        fq::ExecCtx ctx(device_runtime(e));
        fq::DataBlock blk = borrow_block(*b);
        // a filtered block evaluates its kept rows (per reference block, in
        // order: their concatenation is the compacted column)
        if (fq::needs_materialize(blk)) blk = fq::materialize(blk, ctx);
        const fq::ColumnarValue v = f->f->eval(blk, ctx);
        *out_bytes = 0;
        *out_len = 0;
        *out_dtype = v.data_type();
        if (!v.is_array) {
            *is_array = 0;
            t_strings.clear();
            t_strings.reserve(1);
            *scalar = to_scalar(v.scalar);
            ctx.sync();
            return;
        }
        *is_array = 1;
        const fq::Column &c = v.array;
        const size_t bytes = c.dtype == FQ_DT_BOOLEAN ? (size_t)((c.len + 63) / 64) * 8
                                                      : (size_t)c.len * (size_t)fq::dtype_size(c.dtype);
        *out_bytes = bytes;
        *out_len = c.len;
        if (bytes > cap || (bytes > 0 && !d_out))
            throw fq::FQException(FQ_E_INVALID, "fq_function_eval: output buffer too small");
        if (bytes > 0) {
            if (!c.on_device()) throw fq::FQException(FQ_E_UNSUPPORTED, "fq_function_eval: host column result");
            fq::check_hip(hipMemcpyAsync(d_out, c.dptr(), bytes, hipMemcpyDeviceToDevice, ctx.stream()),
                          "hipMemcpyAsync");
        }
        ctx.sync();
    });
}

fq_status fq_function_accumulate(fq_engine *e, fq_function *f, const fq_block *b) {
    if (!e || !f || !b) return fqc::fail(FQ_E_INVALID, "fq_function_accumulate: bad argument");
    return guard([&] {
        fq::ExecCtx ctx(device_runtime(e));
        const fq::DataBlock blk = borrow_block(*b);
        f->f->accumulate(blk, ctx);
        ctx.sync();
    });
}

fq_status fq_functions_accumulate(fq_engine *e, fq_function *const *fs, int32_t n, const fq_block *b) {
    if (!e || !b || n < 0 || (n > 0 && !fs)) return fqc::fail(FQ_E_INVALID, "fq_functions_accumulate: bad argument");
    for (int32_t i = 0; i < n; ++i)
        if (!fs[i]) return fqc::fail(FQ_E_INVALID, "fq_functions_accumulate: NULL function");
    return guard([&] {
        fq::ExecCtx ctx(device_runtime(e));
        const fq::DataBlock blk = borrow_block(*b);
        // AggregatePartialTransform::execute's loop for this one block: the
        // aggregators defer to the fusion, which launches one scan per distinct
        // (argument, filter) and replays the states in (function) order
        fq::AggFusion fusion(ctx);
        fq::AggFusion *prev = ctx.fusion;
        ctx.fusion = &fusion;
        try {
            for (int32_t i = 0; i < n; ++i) fs[i]->f->accumulate(blk, ctx);
        } catch (...) {
            ctx.fusion = prev;
            throw;
        }
        ctx.fusion = prev;
        fusion.finish();
    });
}

fq_status fq_function_accumulate_result(const fq_function *f, fq_scalar *states, size_t cap, size_t *n) {
    if (!f || !n || (cap > 0 && !states)) return fqc::fail(FQ_E_INVALID, "fq_function_accumulate_result: bad argument");
    return guard([&] {
        const std::vector<fq::DataValue> st = f->f->accumulate_result();
        *n = st.size();
        if (st.size() > cap) throw fq::FQException(FQ_E_INVALID, "fq_function_accumulate_result: buffer too small");
        t_strings.clear();
        t_strings.reserve(st.size());  // no reallocation: the c_str() pointers stay valid
        for (size_t i = 0; i < st.size(); ++i) states[i] = to_scalar(st[i]);
    });
}

fq_status fq_function_merge_state(fq_function *f, const fq_scalar *states, size_t n) {
    if (!f || (n > 0 && !states)) return fqc::fail(FQ_E_INVALID, "fq_function_merge_state: bad argument");
    return guard([&] {
        std::vector<fq::DataValue> st;
        st.reserve(n);
        for (size_t i = 0; i < n; ++i) st.push_back(from_scalar(states[i]));
        f->f->merge_state(st);
    });
}

fq_status fq_function_merge_result(const fq_function *f, fq_scalar *out) {
    if (!f || !out) return fqc::fail(FQ_E_INVALID, "fq_function_merge_result: bad argument");
    return guard([&] {
        const fq::DataValue v = f->f->merge_result();
        t_strings.clear();
        t_strings.reserve(1);
        *out = to_scalar(v);
    });
}

fq_status fq_data_value_arithmetic_op(int32_t op, const fq_scalar *l, const fq_scalar *r, fq_scalar *out) {
    if (!l || !r || !out) return fqc::fail(FQ_E_INVALID, "fq_data_value_arithmetic_op: bad argument");
    return guard([&] {
        const fq::DataValue v = fq::data_value_arithmetic_op(op, from_scalar(*l), from_scalar(*r));
        t_strings.clear();
        t_strings.reserve(1);
        *out = to_scalar(v);
    });
}

fq_status fq_data_value_aggregate_op(uint32_t agg, const fq_scalar *l, const fq_scalar *r, fq_scalar *out) {
    if (!l || !r || !out) return fqc::fail(FQ_E_INVALID, "fq_data_value_aggregate_op: bad argument");
    return guard([&] {
        const fq::DataValue v = fq::data_value_aggregate_op(agg, from_scalar(*l), from_scalar(*r));
        t_strings.clear();
        t_strings.reserve(1);
        *out = to_scalar(v);
    });
}

}  // extern "C"
