// Element-wise ArithmeticFunction / ComparisonFunction evaluation on gfx950.
//
//   fq_arith    data_array_arithmetic_op  src/datavalues/data_array_arithmetic.rs:14-55
//               (cast both sides to numerical_coercion, then arrow add/subtract/
//               multiply/divide; release-mode integer wrap; '/' on a zero divisor
//               -> ArrowError::DivideByZero)
//   fq_compare  data_array_comparison_op  src/datavalues/data_array_comparison.rs:14-94
//               (cast to equal_coercion, arrow eq/lt/lt_eq/gt/gt_eq[_scalar]);
//               the Boolean result is an LSB-first bitmap written one 64-bit
//               word per wave with __ballot.
//
// These materialise a column; the aggregate path fuses the same arithmetic
// into its scan (fq_aggregate.hip) and only falls back here for expression
// shapes the fused chain cannot express.
#include <hip/hip_runtime.h>

#include <string>

#include "fq_common.h"
#include "fq_device.h"

namespace fqk {

template <typename TC>
__device__ __forceinline__ TC conv_s(int64_t w, bool &ok) {
    if constexpr (__is_same(TC, float) || __is_same(TC, double)) {
        return (TC)w;
    } else if constexpr (TC(-1) < TC(0)) {
        if (w < (int64_t)Lim<TC>::lo() || w > (int64_t)Lim<TC>::hi()) ok = false;
        return (TC)w;
    } else {
        if (w < 0 || (uint64_t)w > (uint64_t)Lim<TC>::hi()) ok = false;
        return (TC)w;
    }
}

template <typename TC>
__device__ __forceinline__ TC conv_u(uint64_t w, bool &ok) {
    if constexpr (__is_same(TC, float) || __is_same(TC, double)) {
        return (TC)w;
    } else {
        if (w > (uint64_t)Lim<TC>::hi()) ok = false;
        return (TC)w;
    }
}

template <typename TC>
__device__ __forceinline__ TC conv_f(double w, bool &ok) {
    if constexpr (__is_same(TC, float) || __is_same(TC, double)) {
        return (TC)w;
    } else {
        const double t = trunc(w);
        if (!(t >= (double)Lim<TC>::lo() && t < (double)Lim<TC>::hi() + 1.0)) {
            ok = false;
            return TC(0);
        }
        if constexpr (TC(-1) < TC(0)) return (TC)(int64_t)t;
        else return (TC)(uint64_t)t;
    }
}

// arrow::compute::cast of one element of a column of runtime type `dt`
template <typename TC>
__device__ __forceinline__ TC load_as(const void *p, int32_t dt, int64_t i, bool &ok) {
    switch (dt) {
        case FQ_DT_INT8: return conv_s<TC>(((const int8_t *)p)[i], ok);
        case FQ_DT_INT16: return conv_s<TC>(((const int16_t *)p)[i], ok);
        case FQ_DT_INT32: return conv_s<TC>(((const int32_t *)p)[i], ok);
        case FQ_DT_INT64: return conv_s<TC>(((const int64_t *)p)[i], ok);
        case FQ_DT_UINT8: return conv_u<TC>(((const uint8_t *)p)[i], ok);
        case FQ_DT_UINT16: return conv_u<TC>(((const uint16_t *)p)[i], ok);
        case FQ_DT_UINT32: return conv_u<TC>(((const uint32_t *)p)[i], ok);
        case FQ_DT_UINT64: return conv_u<TC>(((const uint64_t *)p)[i], ok);
        case FQ_DT_FLOAT32: return conv_f<TC>(((const float *)p)[i], ok);
        case FQ_DT_FLOAT64: return conv_f<TC>(((const double *)p)[i], ok);
        default: ok = false; return TC(0);
    }
}

template <typename TC>
struct Unsigned {
    using T = TC;
};
template <> struct Unsigned<int8_t> { using T = uint8_t; };
template <> struct Unsigned<int16_t> { using T = uint16_t; };
template <> struct Unsigned<int32_t> { using T = uint32_t; };
template <> struct Unsigned<int64_t> { using T = uint64_t; };

template <typename TC>
__device__ __forceinline__ TC arith(int32_t op, TC a, TC b, uint32_t &flags) {
    if constexpr (__is_same(TC, float) || __is_same(TC, double)) {
        switch (op) {
            case FQ_OP_ADD: return a + b;
            case FQ_OP_SUB: return a - b;
            case FQ_OP_MUL: return a * b;
            case FQ_OP_DIV:
                if (b == TC(0)) flags |= FQ_STATE_DIV_ZERO;
                return a / b;
            default:
                if (b == TC(0)) flags |= FQ_STATE_DIV_ZERO;
                return (TC)fmod((double)a, (double)b);
        }
    } else {
        using U = typename Unsigned<TC>::T;
        switch (op) {
            case FQ_OP_ADD: return (TC)(U)((U)a + (U)b);
            case FQ_OP_SUB: return (TC)(U)((U)a - (U)b);
            case FQ_OP_MUL: return (TC)(U)((U)a * (U)b);
            default:
                if (b == TC(0)) {
                    flags |= FQ_STATE_DIV_ZERO;
                    return TC(0);
                }
                if constexpr (TC(-1) < TC(0)) {
                    if (b == TC(-1)) return op == FQ_OP_DIV ? (TC)(U)((U)0 - (U)a) : TC(0);
                }
                return op == FQ_OP_DIV ? (TC)(a / b) : (TC)(a % b);
        }
    }
}

template <typename TC>
__device__ __forceinline__ bool compare(int32_t cmp, TC a, TC b) {
    switch (cmp) {
        case FQ_CMP_EQ: return a == b;
        case FQ_CMP_LT: return a < b;
        case FQ_CMP_LTEQ: return a <= b;
        case FQ_CMP_GT: return a > b;
        default: return a >= b;
    }
}

__device__ __forceinline__ void flush_flags(uint32_t flags, uint32_t *flag) {
    // one atomic per wave that saw anything
    const uint64_t any = __ballot(flags != 0);
    if (any) {
        uint32_t f = flags;
#pragma unroll
        for (int off = kWave / 2; off > 0; off >>= 1) f |= (uint32_t)__shfl_xor((int)f, off, kWave);
        if ((threadIdx.x & (kWave - 1)) == 0 && flag) atomicOr(flag, f);
    }
}

template <typename TC>
__global__ void __launch_bounds__(256)
    arith_kernel(int32_t op, const void *__restrict__ l, int32_t ldt, uint64_t lc, int lsc,
                 const void *__restrict__ r, int32_t rdt, uint64_t rc, int rsc, TC *__restrict__ out,
                 int64_t n, uint32_t *flag) {
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    uint32_t flags = 0;
    const TC lconst = from_bits<TC>(lc), rconst = from_bits<TC>(rc);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += T) {
        bool ok = true;
        const TC a = lsc ? lconst : load_as<TC>(l, ldt, i, ok);
        const TC b = rsc ? rconst : load_as<TC>(r, rdt, i, ok);
        if (!ok) flags |= FQ_STATE_CAST_NULL;
        out[i] = arith<TC>(op, a, b, flags);
    }
    flush_flags(flags, flag);
}

// one wave = one 64-row bitmap word
template <typename TC>
__global__ void __launch_bounds__(256)
    compare_kernel(int32_t cmp, const void *__restrict__ l, int32_t ldt, uint64_t lc, int lsc,
                   const void *__restrict__ r, int32_t rdt, uint64_t rc, int rsc,
                   uint64_t *__restrict__ bitmap, int64_t n, uint32_t *flag) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nwords = (n + kWave - 1) / kWave;
    const int64_t W = ((int64_t)gridDim.x * blockDim.x) / kWave;
    uint32_t flags = 0;
    const TC lconst = from_bits<TC>(lc), rconst = from_bits<TC>(rc);
    for (int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave; w < nwords; w += W) {
        const int64_t i = w * kWave + lane;
        bool p = false;
        if (i < n) {
            bool ok = true;
            const TC a = lsc ? lconst : load_as<TC>(l, ldt, i, ok);
            const TC b = rsc ? rconst : load_as<TC>(r, rdt, i, ok);
            if (!ok) flags |= FQ_STATE_CAST_NULL;
            p = compare<TC>(cmp, a, b);
        }
        const uint64_t m = __ballot(p);
        if (lane == 0) bitmap[w] = m;
    }
    flush_flags(flags, flag);
}

struct EwArgs {
    int32_t op;
    const void *l;
    int32_t ldt;
    uint64_t lc;
    int lsc;
    const void *r;
    int32_t rdt;
    uint64_t rc;
    int rsc;
    void *out;
    int64_t n;
    uint32_t *flag;
    hipStream_t st;
    int grid;
};

template <typename TC, bool CMP>
static fq_status launch(const EwArgs &a) {
    if constexpr (CMP) {
        hipLaunchKernelGGL((compare_kernel<TC>), dim3(a.grid), dim3(256), 0, a.st, a.op, a.l, a.ldt, a.lc,
                           a.lsc, a.r, a.rdt, a.rc, a.rsc, (uint64_t *)a.out, a.n, a.flag);
    } else {
        hipLaunchKernelGGL((arith_kernel<TC>), dim3(a.grid), dim3(256), 0, a.st, a.op, a.l, a.ldt, a.lc,
                           a.lsc, a.r, a.rdt, a.rc, a.rsc, (TC *)a.out, a.n, a.flag);
    }
    FQ_HIP_TRY(hipGetLastError());
    return FQ_OK;
}

template <bool CMP>
static fq_status launch_typed(int32_t tc, const EwArgs &a) {
    switch (tc) {
        case FQ_DT_INT8: return launch<int8_t, CMP>(a);
        case FQ_DT_INT16: return launch<int16_t, CMP>(a);
        case FQ_DT_INT32: return launch<int32_t, CMP>(a);
        case FQ_DT_INT64: return launch<int64_t, CMP>(a);
        case FQ_DT_UINT8: return launch<uint8_t, CMP>(a);
        case FQ_DT_UINT16: return launch<uint16_t, CMP>(a);
        case FQ_DT_UINT32: return launch<uint32_t, CMP>(a);
        case FQ_DT_UINT64: return launch<uint64_t, CMP>(a);
        case FQ_DT_FLOAT32: return launch<float, CMP>(a);
        case FQ_DT_FLOAT64: return launch<double, CMP>(a);
        default: return fqc::fail(FQ_E_UNSUPPORTED, "element-wise kernel: unsupported type");
    }
}

// DataValue::to_array(size) error text for X(None) (data_value.rs:104-109)
static fq_status none_scalar_error(int32_t dt) {
    (void)dt;
    return fqc::internal("DataValue to array cannot be NONE NULL");
}

// Common validation + scalar conversion; returns the coercion type in *tc.
static fq_status prepare(bool cmp, int32_t op, const fq_col *lhs, const fq_value *ls, const fq_col *rhs,
                         const fq_value *rs, int64_t n, EwArgs &a, int32_t *tc) {
    if ((!lhs) == (!ls) || (!rhs) == (!rs))
        return fqc::fail(FQ_E_INVALID, "exactly one of column/scalar per side");
    const int32_t ldt = lhs ? lhs->dtype : ls->dtype;
    const int32_t rdt = rhs ? rhs->dtype : rs->dtype;
    // a Null scalar becomes a NullArray whose type is Null (to_array, data_value.rs:79)
    fq_status s = cmp ? fqc::equal_coercion(fqc::cmp_op_str(op), ldt, rdt, tc)
                      : fqc::numerical_coercion(fqc::arith_op_str(op), ldt, rdt, tc);
    if (s != FQ_OK) return s;
    if (!fqc::dtype_is_numeric(*tc)) {
        // equal_coercion of two identical non-numeric types
        if (*tc == FQ_DT_UTF8)
            return fqc::fail(FQ_E_UNSUPPORTED, "Utf8 comparison is not supported on the device path");
        // arrow_array_op! has no arm for the type (macros.rs:66-87)
        static const char *names[] = {"eq", "lt", "lt_eq", "gt", "gt_eq"};
        return fqc::internal(std::string("Unsupported arithmetic_compute::") + names[op] +
                             " for data type: " + fqc::dtype_name(*tc));
    }
    if (ls && !ls->is_some) return none_scalar_error(ldt);
    if (rs && !rs->is_some) return none_scalar_error(rdt);
    if (lhs && lhs->len != n) return fqc::fail(FQ_E_INVALID, "lhs length mismatch");
    if (rhs && rhs->len != n) return fqc::fail(FQ_E_INVALID, "rhs length mismatch");
    if ((lhs && n > 0 && !lhs->data) || (rhs && n > 0 && !rhs->data))
        return fqc::fail(FQ_E_INVALID, "NULL column data");
    a = EwArgs{};
    a.op = op;
    a.n = n;
    if (lhs) {
        a.l = lhs->data;
        a.ldt = lhs->dtype;
    } else {
        a.lsc = 1;
        if (!fqc::cast_scalar(ls->bits, ls->dtype, *tc, &a.lc))
            return fqc::fail(FQ_E_UNSUPPORTED, "scalar cast produced a null (nulls are not supported on the device path)");
    }
    if (rhs) {
        a.r = rhs->data;
        a.rdt = rhs->dtype;
    } else {
        a.rsc = 1;
        if (!fqc::cast_scalar(rs->bits, rs->dtype, *tc, &a.rc))
            return fqc::fail(FQ_E_UNSUPPORTED, "scalar cast produced a null (nulls are not supported on the device path)");
    }
    const int max_grid = fqc::device_cu_count() * 8;
    int64_t grid = (n + 255) / 256;
    if (grid < 1) grid = 1;
    a.grid = (int)(grid < max_grid ? grid : max_grid);
    return FQ_OK;
}

static fq_status check_flag(uint32_t *d_flag, hipStream_t st) {
    if (!d_flag) return FQ_OK;
    uint32_t h = 0;
    FQ_HIP_TRY(hipMemcpyAsync(&h, d_flag, sizeof(h), hipMemcpyDeviceToHost, st));
    FQ_HIP_TRY(hipStreamSynchronize(st));
    if (h & FQ_STATE_DIV_ZERO) return fqc::fail(FQ_E_DIVIDE_BY_ZERO, "Internal Error: Divide by zero error");
    if (h & FQ_STATE_CAST_NULL)
        return fqc::fail(FQ_E_UNSUPPORTED, "cast produced nulls (nulls are not supported on the device path)");
    return FQ_OK;
}

}  // namespace fqk

extern "C" {

fq_status fq_arith_result_type(int32_t op, int32_t lhs_dtype, int32_t rhs_dtype, int32_t *out) {
    if (!out) return fqc::fail(FQ_E_INVALID, "fq_arith_result_type: out is NULL");
    return fqc::numerical_coercion(fqc::arith_op_str(op), lhs_dtype, rhs_dtype, out);
}

fq_status fq_arith(int32_t op, const fq_col *lhs, const fq_value *lhs_scalar, const fq_col *rhs,
                   const fq_value *rhs_scalar, fq_col *out, uint32_t *d_flag, void *stream) {
    using namespace fqk;
    if (!out) return fqc::fail(FQ_E_INVALID, "fq_arith: out is NULL");
    if (op < FQ_OP_ADD || op > FQ_OP_MOD) return fqc::fail(FQ_E_INVALID, "fq_arith: bad op");
    const int64_t n = lhs ? lhs->len : (rhs ? rhs->len : 1);
    EwArgs a;
    int32_t tc = 0;
    fq_status s = prepare(false, op, lhs, lhs_scalar, rhs, rhs_scalar, n, a, &tc);
    if (s != FQ_OK) return s;
    if (out->dtype != tc) return fqc::fail(FQ_E_INVALID, "fq_arith: out dtype must be the coercion type");
    if (out->len != n) return fqc::fail(FQ_E_INVALID, "fq_arith: out length mismatch");
    if (n == 0) return FQ_OK;
    if (!out->data) return fqc::fail(FQ_E_INVALID, "fq_arith: NULL out data");
    a.out = out->data;
    a.flag = d_flag;
    a.st = (hipStream_t)stream;
    if (d_flag) FQ_HIP_TRY(hipMemsetAsync(d_flag, 0, sizeof(uint32_t), a.st));
    s = launch_typed<false>(tc, a);
    if (s != FQ_OK) return s;
    return check_flag(d_flag, a.st);
}

fq_status fq_compare(int32_t cmp, const fq_col *lhs, const fq_value *lhs_scalar, const fq_col *rhs,
                     const fq_value *rhs_scalar, uint64_t *d_bitmap, int64_t len, uint32_t *d_flag,
                     void *stream) {
    using namespace fqk;
    if (cmp < FQ_CMP_EQ || cmp > FQ_CMP_GTEQ) return fqc::fail(FQ_E_INVALID, "fq_compare: bad op");
    EwArgs a;
    int32_t tc = 0;
    fq_status s = prepare(true, cmp, lhs, lhs_scalar, rhs, rhs_scalar, len, a, &tc);
    if (s != FQ_OK) return s;
    if (len == 0) return FQ_OK;
    if (!d_bitmap) return fqc::fail(FQ_E_INVALID, "fq_compare: NULL bitmap");
    a.out = d_bitmap;
    a.flag = d_flag;
    a.st = (hipStream_t)stream;
    const int64_t nwords = (len + 63) / 64;
    const int max_grid = fqc::device_cu_count() * 8;
    int64_t grid = (nwords + 3) / 4;
    a.grid = (int)(grid < max_grid ? grid : max_grid);
    if (d_flag) FQ_HIP_TRY(hipMemsetAsync(d_flag, 0, sizeof(uint32_t), a.st));
    s = launch_typed<true>(tc, a);
    if (s != FQ_OK) return s;
    return check_flag(d_flag, a.st);
}

}  // extern "C"
