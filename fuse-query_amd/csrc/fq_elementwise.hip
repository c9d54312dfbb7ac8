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
#include <stdlib.h>

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

// ---------------------------------------------------------------------------
// 16-byte vector fast paths for the common case: every column operand already
// has the coercion type (no cast), the type is 64-bit, and every pointer is
// 16-byte aligned.  Same streaming structure as the scan (fq_aggregate.hip):
// tile-contiguous, non-temporal, 8 vectors per lane in flight, 2 workgroups
// per CU (tools/tune_scan.py --write: 5.6 TB/s for read+write streams vs 4.4
// for the element-granular grid stride).  The op is a template parameter, so
// the loop body is straight-line.  Rows past the last whole tile go to the
// generic kernels above.
// ---------------------------------------------------------------------------
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kEwU = 8;

template <typename TC, int OP, bool LSC, bool RSC>
__global__ void __launch_bounds__(256)
    arith_vec_kernel(const TC *__restrict__ l, uint64_t lc, const TC *__restrict__ r, uint64_t rc,
                     TC *__restrict__ out, int64_t ntiles, uint32_t *flag) {
    static_assert(sizeof(TC) == 8, "64-bit fast path");
    const u32x4 *__restrict__ lv = reinterpret_cast<const u32x4 *>(l);
    const u32x4 *__restrict__ rv = reinterpret_cast<const u32x4 *>(r);
    u32x4 *__restrict__ ov = reinterpret_cast<u32x4 *>(out);
    const TC lconst = from_bits<TC>(lc), rconst = from_bits<TC>(rc);
    uint32_t flags = 0;
    constexpr int64_t TV = (int64_t)kEwU * 256;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t base = t * TV + threadIdx.x;
        u32x4 a[kEwU], b[kEwU];
#pragma unroll
        for (int k = 0; k < kEwU; ++k) {
            if constexpr (!LSC) a[k] = __builtin_nontemporal_load(lv + base + (int64_t)k * 256);
            if constexpr (!RSC) b[k] = __builtin_nontemporal_load(rv + base + (int64_t)k * 256);
        }
#pragma unroll
        for (int k = 0; k < kEwU; ++k) {
            TC x[2], y[2], z[2];
            if constexpr (!LSC) __builtin_memcpy(x, &a[k], 16);
            else x[0] = x[1] = lconst;
            if constexpr (!RSC) __builtin_memcpy(y, &b[k], 16);
            else y[0] = y[1] = rconst;
            z[0] = arith<TC>(OP, x[0], y[0], flags);
            z[1] = arith<TC>(OP, x[1], y[1], flags);
            u32x4 o;
            __builtin_memcpy(&o, z, 16);
            __builtin_nontemporal_store(o, ov + base + (int64_t)k * 256);
        }
    }
    flush_flags(flags, flag);
}

// A wave compares 8 x 128 rows per iteration (lane l holds rows 2l and 2l+1
// of each 128-row segment in one 16-byte load; 8 loads in flight) and lanes
// 0..15 store the segments' 16 bitmap words (128 contiguous bytes).
// `ngroups` = whole 1024-row groups.  (4 segments: 5.2 TB/s; 8: 6.1 TB/s.)
// Bit r of a segment's words belongs to lane r >> 1: one ds_bpermute hands
// lane l the two results of lane l >> 1 (word 0) and of lane 32 + (l >> 1)
// (word 1), so each word is a single ballot; interleaving two 32-bit ballots
// on the scalar unit instead (spread32, 4 per segment) cost 1.68 vs 1.55 ms
// per 10 GB (tools/bench_kernels.py, round 1; removed in round 6).
template <typename TC, int CMP, bool LSC, bool RSC>
__global__ void __launch_bounds__(256)
    compare_vec_kernel(const TC *__restrict__ l, uint64_t lc, const TC *__restrict__ r, uint64_t rc,
                       uint64_t *__restrict__ bitmap, int64_t ngroups) {
    static_assert(sizeof(TC) == 8, "64-bit fast path");
    constexpr int SEG = 8;  // 128-row segments per group
    const int lane = threadIdx.x & (kWave - 1);
    const u32x4 *__restrict__ lv = reinterpret_cast<const u32x4 *>(l);
    const u32x4 *__restrict__ rv = reinterpret_cast<const u32x4 *>(r);
    const TC lconst = from_bits<TC>(lc), rconst = from_bits<TC>(rc);
    const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    const int64_t GW = ((int64_t)gridDim.x * blockDim.x) / kWave;
    for (int64_t g = gw; g < ngroups; g += GW) {
        const int64_t v0 = g * (SEG * kWave) + lane;  // vector index of this lane in segment 0
        u32x4 a[SEG], b[SEG];
#pragma unroll
        for (int k = 0; k < SEG; ++k) {
            if constexpr (!LSC) a[k] = __builtin_nontemporal_load(lv + v0 + k * kWave);
            if constexpr (!RSC) b[k] = __builtin_nontemporal_load(rv + v0 + k * kWave);
        }
        uint64_t mine = 0;
#pragma unroll
        for (int k = 0; k < SEG; ++k) {
            TC x[2], y[2];
            if constexpr (!LSC) __builtin_memcpy(x, &a[k], 16);
            else x[0] = x[1] = lconst;
            if constexpr (!RSC) __builtin_memcpy(y, &b[k], 16);
            else y[0] = y[1] = rconst;
            const int two = (compare<TC>(CMP, x[0], y[0]) ? 1 : 0) | (compare<TC>(CMP, x[1], y[1]) ? 2 : 0);
            const int lo = __builtin_amdgcn_ds_bpermute((lane >> 1) << 2, two);
            const int hi = __builtin_amdgcn_ds_bpermute((32 + (lane >> 1)) << 2, two);
            const uint64_t w0 = __ballot((lo >> (lane & 1)) & 1);
            const uint64_t w1 = __ballot((hi >> (lane & 1)) & 1);
            mine = lane == 2 * k ? w0 : mine;
            mine = lane == 2 * k + 1 ? w1 : mine;
        }
        if (lane < 2 * SEG) bitmap[g * (2 * SEG) + lane] = mine;
    }
}

template <typename TC, bool CMPK, int OP>
static void launch_vec_op(bool lsc, bool rsc, const void *l, uint64_t lc, const void *r, uint64_t rc, void *out,
                          int64_t units, uint32_t *flag, int grid, hipStream_t st) {
    const TC *L = (const TC *)l, *R = (const TC *)r;
    if constexpr (CMPK) {
        uint64_t *bm = (uint64_t *)out;
        if (lsc) hipLaunchKernelGGL((compare_vec_kernel<TC, OP, true, false>), dim3(grid), dim3(256), 0, st, L, lc, R, rc, bm, units);
        else if (rsc) hipLaunchKernelGGL((compare_vec_kernel<TC, OP, false, true>), dim3(grid), dim3(256), 0, st, L, lc, R, rc, bm, units);
        else hipLaunchKernelGGL((compare_vec_kernel<TC, OP, false, false>), dim3(grid), dim3(256), 0, st, L, lc, R, rc, bm, units);
        (void)flag;
    } else {
        TC *O = (TC *)out;
        if (lsc) hipLaunchKernelGGL((arith_vec_kernel<TC, OP, true, false>), dim3(grid), dim3(256), 0, st, L, lc, R, rc, O, units, flag);
        else if (rsc) hipLaunchKernelGGL((arith_vec_kernel<TC, OP, false, true>), dim3(grid), dim3(256), 0, st, L, lc, R, rc, O, units, flag);
        else hipLaunchKernelGGL((arith_vec_kernel<TC, OP, false, false>), dim3(grid), dim3(256), 0, st, L, lc, R, rc, O, units, flag);
    }
}

template <typename TC, bool CMPK>
static void launch_vec(int32_t op, bool lsc, bool rsc, const void *l, uint64_t lc, const void *r, uint64_t rc,
                       void *out, int64_t units, uint32_t *flag, int grid, hipStream_t st) {
    // FQ_OP_* and FQ_CMP_* are both 0..4
    switch (op) {
        case 0: return launch_vec_op<TC, CMPK, 0>(lsc, rsc, l, lc, r, rc, out, units, flag, grid, st);
        case 1: return launch_vec_op<TC, CMPK, 1>(lsc, rsc, l, lc, r, rc, out, units, flag, grid, st);
        case 2: return launch_vec_op<TC, CMPK, 2>(lsc, rsc, l, lc, r, rc, out, units, flag, grid, st);
        case 3: return launch_vec_op<TC, CMPK, 3>(lsc, rsc, l, lc, r, rc, out, units, flag, grid, st);
        default: return launch_vec_op<TC, CMPK, 4>(lsc, rsc, l, lc, r, rc, out, units, flag, grid, st);
    }
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

// Launches the vector fast path over the longest whole-tile prefix it covers
// and returns in `a` the (offset) arguments of the remaining rows for the
// generic kernel; a.n = 0 when nothing remains.
static fq_status launch_fast(bool cmp, int32_t tc, EwArgs &a) {
    auto aligned = [](const void *p) { return ((uintptr_t)p & 15u) == 0; };
    if (fqc::dtype_size(tc) != 8 || (a.lsc && a.rsc)) return FQ_OK;
    if (!a.lsc && (a.ldt != tc || !aligned(a.l))) return FQ_OK;
    if (!a.rsc && (a.rdt != tc || !aligned(a.r))) return FQ_OK;
    if (!aligned(a.out)) return FQ_OK;
    const int64_t rows_per_unit = cmp ? 1024 : (int64_t)kEwU * 256 * 2;
    const int64_t units = a.n / rows_per_unit;
    if (units == 0) return FQ_OK;
    // workgroups per CU: arith 8, compare 2 (tools/probes/ew_wg_sweep.sh, one box:
    // arith u64 + const 3.57/3.49/3.44/3.38 ms at 1/2/4/8, compare 1.68/1.71/1.75/1.73);
    // FQ_TUNE_EW_WG_PER_CU overrides both (tuning)
    const int wg_override = (int)fqc::knob(FQ_TUNE_EW_WG_PER_CU);
    const int64_t cap = (int64_t)fqc::device_cu_count() * (wg_override ? wg_override : (cmp ? 2 : 8));
    // arith: one tile per workgroup iteration; compare: one 1,024-row group per wave
    const int64_t want = cmp ? (units + 3) / 4 : units;
    const int grid = (int)(want < cap ? want : cap);
    switch (tc) {
        case FQ_DT_INT64:
            if (cmp) launch_vec<int64_t, true>(a.op, a.lsc, a.rsc, a.l, a.lc, a.r, a.rc, a.out, units, a.flag, grid, a.st);
            else launch_vec<int64_t, false>(a.op, a.lsc, a.rsc, a.l, a.lc, a.r, a.rc, a.out, units, a.flag, grid, a.st);
            break;
        case FQ_DT_UINT64:
            if (cmp) launch_vec<uint64_t, true>(a.op, a.lsc, a.rsc, a.l, a.lc, a.r, a.rc, a.out, units, a.flag, grid, a.st);
            else launch_vec<uint64_t, false>(a.op, a.lsc, a.rsc, a.l, a.lc, a.r, a.rc, a.out, units, a.flag, grid, a.st);
            break;
        case FQ_DT_FLOAT64:
            if (cmp) launch_vec<double, true>(a.op, a.lsc, a.rsc, a.l, a.lc, a.r, a.rc, a.out, units, a.flag, grid, a.st);
            else launch_vec<double, false>(a.op, a.lsc, a.rsc, a.l, a.lc, a.r, a.rc, a.out, units, a.flag, grid, a.st);
            break;
        default: return FQ_OK;
    }
    FQ_HIP_TRY(hipGetLastError());
    const int64_t done = units * rows_per_unit;
    if (!a.lsc) a.l = (const char *)a.l + done * 8;
    if (!a.rsc) a.r = (const char *)a.r + done * 8;
    a.out = cmp ? (void *)((uint64_t *)a.out + done / 64) : (void *)((char *)a.out + done * 8);
    a.n -= done;
    if (cmp) {
        const int64_t nwords = (a.n + 63) / 64;
        const int max_grid = fqc::device_cu_count() * 8;
        const int64_t g = (nwords + 3) / 4;
        a.grid = (int)(g < 1 ? 1 : (g < max_grid ? g : max_grid));
    } else {
        const int max_grid = fqc::device_cu_count() * 8;
        const int64_t g = (a.n + 255) / 256;
        a.grid = (int)(g < 1 ? 1 : (g < max_grid ? g : max_grid));
    }
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
    s = launch_fast(false, tc, a);
    if (s != FQ_OK) return s;
    if (a.n > 0) {
        s = launch_typed<false>(tc, a);
        if (s != FQ_OK) return s;
    }
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
    s = launch_fast(true, tc, a);
    if (s != FQ_OK) return s;
    if (a.n > 0) {
        s = launch_typed<true>(tc, a);
        if (s != FQ_OK) return s;
    }
    return check_flag(d_flag, a.st);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// LogicFunction: word-wise and/or of two bitmaps (16-byte loads/stores)
// ---------------------------------------------------------------------------
namespace fqk {

template <int OP>
__global__ void __launch_bounds__(256)
    logic_kernel(const uint64_t *__restrict__ l, const uint64_t *__restrict__ r, uint64_t *__restrict__ out,
                 int64_t nwords, int64_t len) {
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    const int64_t npairs = nwords / 2;
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    const u64x2 *lv = reinterpret_cast<const u64x2 *>(l), *rv = reinterpret_cast<const u64x2 *>(r);
    u64x2 *ov = reinterpret_cast<u64x2 *>(out);
    const bool vec = ((((uintptr_t)l) | ((uintptr_t)r) | ((uintptr_t)out)) & 15u) == 0;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t done = 0;
    if (vec) {
        for (int64_t p = g; p < npairs; p += T) {
            const u64x2 a = __builtin_nontemporal_load(lv + p), b = __builtin_nontemporal_load(rv + p);
            ov[p] = OP == FQ_LOGIC_AND ? (a & b) : (a | b);
        }
        done = npairs * 2;
    }
    for (int64_t w = done + g; w < nwords; w += T) {
        uint64_t v = OP == FQ_LOGIC_AND ? (l[w] & r[w]) : (l[w] | r[w]);
        if (w == nwords - 1 && (len & 63)) v &= (1ull << (len & 63)) - 1ull;
        out[w] = v;
    }
    // (an even word count puts the last word in the vector part: the host
    // clears its tail bits with logic_tail_kernel)
}

__global__ void logic_tail_kernel(uint64_t *out, int64_t nwords, int64_t len) {
    out[nwords - 1] &= (1ull << (len & 63)) - 1ull;
}

}  // namespace fqk

extern "C" fq_status fq_logic(int32_t op, const uint64_t *d_lhs, const uint64_t *d_rhs, uint64_t *d_out, int64_t len,
                              void *stream) {
    using namespace fqk;
    if (op != FQ_LOGIC_AND && op != FQ_LOGIC_OR) return fqc::fail(FQ_E_INVALID, "fq_logic: bad op");
    if (len < 0) return fqc::fail(FQ_E_INVALID, "fq_logic: negative length");
    if (len == 0) return FQ_OK;
    if (!d_lhs || !d_rhs || !d_out) return fqc::fail(FQ_E_INVALID, "fq_logic: NULL bitmap");
    hipStream_t st = (hipStream_t)stream;
    const int64_t nwords = (len + 63) / 64;
    const int64_t cap = (int64_t)fqc::device_cu_count() * 2;
    int64_t grid = (nwords / 2 + 255) / 256;
    if (grid < 1) grid = 1;
    if (grid > cap) grid = cap;
    if (op == FQ_LOGIC_AND)
        hipLaunchKernelGGL((logic_kernel<FQ_LOGIC_AND>), dim3((int)grid), dim3(256), 0, st, d_lhs, d_rhs, d_out, nwords, len);
    else
        hipLaunchKernelGGL((logic_kernel<FQ_LOGIC_OR>), dim3((int)grid), dim3(256), 0, st, d_lhs, d_rhs, d_out, nwords, len);
    FQ_HIP_TRY(hipGetLastError());
    const bool vec = ((((uintptr_t)d_lhs) | ((uintptr_t)d_rhs) | ((uintptr_t)d_out)) & 15u) == 0;
    if (vec && (len & 63) && (nwords & 1) == 0) {  // last word written by the vector loop
        hipLaunchKernelGGL(logic_tail_kernel, dim3(1), dim3(1), 0, st, d_out, nwords, len);
        FQ_HIP_TRY(hipGetLastError());
    }
    return FQ_OK;
}

