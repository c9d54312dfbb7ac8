// Error plumbing, dtype table and the host-side state merge of the C ABI.
#include "fq_common.h"

#include <stdio.h>

#include <mutex>
#include <vector>

namespace fqc {

static thread_local std::string g_last_error;

fq_status fail(fq_status st, const std::string &msg) {
    g_last_error = msg;
    return st;
}

fq_status internal(const std::string &msg) { return fail(FQ_E_INTERNAL, "Internal Error: " + msg); }

fq_status hip_fail(hipError_t e, const char *what) {
    std::string m = "HIP error ";
    m += hipGetErrorName(e);
    m += " (";
    m += hipGetErrorString(e);
    m += ") in ";
    m += what;
    (void)hipGetLastError();  // clear sticky non-fatal errors
    return fail(FQ_E_HIP, m);
}

int device_cu_count() {
    static std::mutex mu;
    static std::vector<int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    std::lock_guard<std::mutex> lk(mu);
    if ((int)cache.size() <= dev) cache.resize(dev + 1, 0);
    if (cache[dev] == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 256;
        cache[dev] = cus;
    }
    return cache[dev];
}

const char *dtype_name(int32_t dt) {
    switch (dt) {
        case FQ_DT_NULL: return "Null";
        case FQ_DT_BOOLEAN: return "Boolean";
        case FQ_DT_INT8: return "Int8";
        case FQ_DT_INT16: return "Int16";
        case FQ_DT_INT32: return "Int32";
        case FQ_DT_INT64: return "Int64";
        case FQ_DT_UINT8: return "UInt8";
        case FQ_DT_UINT16: return "UInt16";
        case FQ_DT_UINT32: return "UInt32";
        case FQ_DT_UINT64: return "UInt64";
        case FQ_DT_FLOAT32: return "Float32";
        case FQ_DT_FLOAT64: return "Float64";
        case FQ_DT_UTF8: return "Utf8";
        default: return "Unknown";
    }
}

int dtype_size(int32_t dt) {
    switch (dt) {
        case FQ_DT_INT8:
        case FQ_DT_UINT8: return 1;
        case FQ_DT_INT16:
        case FQ_DT_UINT16: return 2;
        case FQ_DT_INT32:
        case FQ_DT_UINT32:
        case FQ_DT_FLOAT32: return 4;
        case FQ_DT_INT64:
        case FQ_DT_UINT64:
        case FQ_DT_FLOAT64: return 8;
        default: return 0;
    }
}

bool dtype_is_signed_int(int32_t dt) { return dt >= FQ_DT_INT8 && dt <= FQ_DT_INT64; }
bool dtype_is_unsigned_int(int32_t dt) { return dt >= FQ_DT_UINT8 && dt <= FQ_DT_UINT64; }
bool dtype_is_float(int32_t dt) { return dt == FQ_DT_FLOAT32 || dt == FQ_DT_FLOAT64; }
bool dtype_is_numeric(int32_t dt) { return dt >= FQ_DT_INT8 && dt <= FQ_DT_FLOAT64; }

}  // namespace fqc

// ---------------------------------------------------------------------------
// C ABI: library-level entry points
// ---------------------------------------------------------------------------
extern "C" {

int32_t fq_abi_version(void) { return FQ_ABI_VERSION; }

const char *fq_last_error(void) { return fqc::g_last_error.c_str(); }

fq_status fq_device_count(int32_t *out) {
    if (!out) return fqc::fail(FQ_E_INVALID, "fq_device_count: out is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *out = 0;
        return fqc::hip_fail(e, "hipGetDeviceCount");
    }
    *out = n;
    return FQ_OK;
}

// AggregatorFunction::merge_state (function_aggregator.rs:106-139) for the
// device partial states: Sum -> wrapping add (integers) / binary64 add,
// Count/blocks -> add, Max/Min -> max/min over the states that hold a value.
fq_status fq_state_merge(const fq_agg_state *states, int32_t n, fq_agg_state *out) {
    if (!out || (n > 0 && !states)) return fqc::fail(FQ_E_INVALID, "fq_state_merge: NULL argument");
    if (n <= 0) return fqc::fail(FQ_E_INVALID, "fq_state_merge: n must be > 0");
    const int32_t dt = states[0].dtype;
    for (int32_t i = 1; i < n; ++i)
        if (states[i].dtype != dt)
            return fqc::internal(std::string("Unsupported data_value_sum for data type: left:") +
                                 fqc::dtype_name(dt) + ", right:" + fqc::dtype_name(states[i].dtype));
    fq_agg_state r = states[0];
    for (int32_t i = 1; i < n; ++i) {
        const fq_agg_state &s = states[i];
        r.flags |= s.flags;
        r.blocks += s.blocks;
        if (s.count == 0) continue;
        if (r.count == 0) {  // nothing accumulated yet: take s's values
            r.sum = s.sum;
            r.max = s.max;
            r.min = s.min;
            r.count = s.count;
            continue;
        }
        r.count += s.count;
        if (fqc::dtype_is_float(dt)) {
            double a, b, mx_a, mx_b, mn_a, mn_b;
            __builtin_memcpy(&a, &r.sum, 8);
            __builtin_memcpy(&b, &s.sum, 8);
            __builtin_memcpy(&mx_a, &r.max, 8);
            __builtin_memcpy(&mx_b, &s.max, 8);
            __builtin_memcpy(&mn_a, &r.min, 8);
            __builtin_memcpy(&mn_b, &s.min, 8);
            double sum = a + b;
            if (dt == FQ_DT_FLOAT32) sum = (double)((float)a + (float)b);
            const double mx = mx_b > mx_a ? mx_b : mx_a;
            const double mn = mn_b < mn_a ? mn_b : mn_a;
            __builtin_memcpy(&r.sum, &sum, 8);
            __builtin_memcpy(&r.max, &mx, 8);
            __builtin_memcpy(&r.min, &mn, 8);
        } else if (fqc::dtype_is_signed_int(dt)) {
            r.sum = r.sum + s.sum;
            const int bits = 8 * fqc::dtype_size(dt);
            if (bits < 64) {  // wrap in the value type, keep sign extension
                const uint64_t m = (1ull << bits) - 1;
                uint64_t v = r.sum & m;
                if (v >> (bits - 1)) v |= ~m;
                r.sum = v;
            }
            r.max = ((int64_t)s.max > (int64_t)r.max) ? s.max : r.max;
            r.min = ((int64_t)s.min < (int64_t)r.min) ? s.min : r.min;
        } else {
            r.sum = r.sum + s.sum;
            const int bits = 8 * fqc::dtype_size(dt);
            if (bits < 64) r.sum &= (1ull << bits) - 1;
            r.max = s.max > r.max ? s.max : r.max;
            r.min = s.min < r.min ? s.min : r.min;
        }
    }
    *out = r;
    return FQ_OK;
}

}  // extern "C"

namespace fqc {

const char *arith_op_str(int32_t op) {
    switch (op) {
        case FQ_OP_ADD: return "+";
        case FQ_OP_SUB: return "-";
        case FQ_OP_MUL: return "*";
        case FQ_OP_DIV: return "/";
        case FQ_OP_MOD: return "%";
        default: return "?";
    }
}

const char *cmp_op_str(int32_t cmp) {
    switch (cmp) {
        case FQ_CMP_EQ: return "=";
        case FQ_CMP_LT: return "<";
        case FQ_CMP_LTEQ: return "<=";
        case FQ_CMP_GT: return ">";
        case FQ_CMP_GTEQ: return ">=";
        default: return "?";
    }
}

fq_status numerical_coercion(const char *op, int32_t l, int32_t r, int32_t *out) {
    if (!dtype_is_numeric(l) || !dtype_is_numeric(r))
        return internal(std::string("Unsupported (") + dtype_name(l) + ") " + op + " (" + dtype_name(r) + ")");
    if (l == r) {
        *out = l;
        return FQ_OK;
    }
    // ordered from most to least informative (data_type.rs:50-84)
    static const int32_t order[] = {FQ_DT_FLOAT64, FQ_DT_FLOAT32, FQ_DT_INT64,  FQ_DT_INT32, FQ_DT_INT16,
                                    FQ_DT_INT8,    FQ_DT_UINT64,  FQ_DT_UINT32, FQ_DT_UINT16, FQ_DT_UINT8};
    for (int32_t t : order) {
        if (l == t || r == t) {
            *out = t;
            return FQ_OK;
        }
    }
    return internal(std::string("Unsupported (") + dtype_name(l) + ") " + op + " (" + dtype_name(r) + ")");
}

fq_status equal_coercion(const char *op, int32_t l, int32_t r, int32_t *out) {
    if (l == r) {
        *out = l;
        return FQ_OK;
    }
    return numerical_coercion(op, l, r, out);
}

static bool int_range(int32_t dt, int64_t &lo, uint64_t &hi) {
    switch (dt) {
        case FQ_DT_INT8: lo = INT8_MIN; hi = INT8_MAX; return true;
        case FQ_DT_INT16: lo = INT16_MIN; hi = INT16_MAX; return true;
        case FQ_DT_INT32: lo = INT32_MIN; hi = INT32_MAX; return true;
        case FQ_DT_INT64: lo = INT64_MIN; hi = INT64_MAX; return true;
        case FQ_DT_UINT8: lo = 0; hi = UINT8_MAX; return true;
        case FQ_DT_UINT16: lo = 0; hi = UINT16_MAX; return true;
        case FQ_DT_UINT32: lo = 0; hi = UINT32_MAX; return true;
        case FQ_DT_UINT64: lo = 0; hi = UINT64_MAX; return true;
        default: return false;
    }
}

bool cast_scalar(uint64_t bits, int32_t from, int32_t to, uint64_t *out) {
    if (from == to) {
        *out = bits;
        return true;
    }
    if (dtype_is_float(to)) {
        double d;
        if (dtype_is_float(from)) __builtin_memcpy(&d, &bits, 8);
        else if (dtype_is_signed_int(from)) d = (double)(int64_t)bits;
        else d = (double)bits;
        if (to == FQ_DT_FLOAT32) d = (double)(float)d;
        __builtin_memcpy(out, &d, 8);
        return true;
    }
    int64_t lo;
    uint64_t hi;
    if (!int_range(to, lo, hi)) return false;
    if (dtype_is_float(from)) {
        double d;
        __builtin_memcpy(&d, &bits, 8);
        const double t = __builtin_trunc(d);
        if (t != t) return false;
        if (!(t >= (double)lo && t < (double)hi + 1.0)) return false;
        *out = dtype_is_signed_int(to) ? (uint64_t)(int64_t)t : (uint64_t)t;
        return true;
    }
    if (dtype_is_signed_int(from)) {
        const int64_t v = (int64_t)bits;
        if (v < lo) return false;
        if (v >= 0 && (uint64_t)v > hi) return false;
        *out = (uint64_t)v;
        return true;
    }
    // unsigned source
    if (bits > hi) return false;
    *out = bits;
    return true;
}

}  // namespace fqc

namespace fqc {
namespace {
struct Staging {
    uint64_t *p = nullptr;
    bool tried = false;
    ~Staging() {
        if (p) (void)hipHostFree(p);
    }
};
thread_local Staging g_staging;
}  // namespace

uint64_t *host_staging() {
    if (!g_staging.tried) {
        g_staging.tried = true;
        void *p = nullptr;
        if (hipHostMalloc(&p, 8 * sizeof(uint64_t), hipHostMallocDefault) == hipSuccess) g_staging.p = (uint64_t *)p;
        else (void)hipGetLastError();
    }
    return g_staging.p;
}
}  // namespace fqc
