// Device-side building blocks shared by the gfx950 kernels: dtype traits,
// the lowered expression program (fused ArithmeticFunction chains) and the
// 64-bit wave reductions.  Not part of the public ABI (see include/fq_gpu.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fq_gpu.h"

namespace fqk {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

// ---------------------------------------------------------------------------
// Lowered step codes.  The host lowers fq_step (semantic: op, dtype, operand)
// into one of these, inserting explicit casts where numerical_coercion
// (src/datavalues/data_type.rs:27-90) widens the accumulator, and replacing
// u64 division/modulo by a constant with shift/and or a multiply-high magic.
// ---------------------------------------------------------------------------
enum Code : int32_t {
    K_NOP = 0,
    K_CAST_U2I,  // UInt64 -> Int64 (arrow cast: > i64::MAX becomes null)
    K_CAST_U2F,  // UInt64 -> Float64
    K_CAST_I2F,  // Int64  -> Float64
    K_ADD_I,     // wrapping 64-bit add (u64 and i64 share the bits)
    K_SUB_I,
    K_MUL_I,
    K_DIV_U,  // generic u64 '/', zero divisor -> DIV_ZERO flag
    K_MOD_U,
    K_DIV_S,  // generic i64 '/', truncating
    K_MOD_S,
    K_SHR_U,   // u64 '/' by a power of two
    K_AND_U,   // u64 '%' by a power of two
    K_DIVM_U,  // u64 '/' by a constant: multiply-high magic
    K_MODM_U,  // u64 '%' by a constant
    K_ADD_F,
    K_SUB_F,
    K_MUL_F,
    K_DIV_F,  // f64 '/', zero divisor -> DIV_ZERO (arrow 2.0 divide checks is_zero)
    K_MOD_F,
    K_PUSH,  // expression trees: push acc, acc = the column (hipRTC kernels only)
    K_MODM32_U,  // u64 '%' by a constant d <= 65535: both 32-bit halves reduced with a
                 // 32-bit magic, recombined as (hi % d) * (2^32 % d) + lo % d (< 2^32)
                 // and reduced once more -- 32-bit multiplies instead of a 64-bit mul-high
    K_DIVM32_U,  // u64 '/' by a constant d <= 65535: long division in 32/16/16-bit digits,
                 // each step a 32-bit magic divide (every partial dividend < d * 2^16)
};

struct KStep {
    int32_t code;
    int32_t operand;   // FQ_OPERAND_CONST / FQ_OPERAND_COLUMN
    int32_t reversed;  // operand OP acc
    int32_t dtype;     // FQ_DT_UINT64 / INT64 / FLOAT64 (type of this step)
    uint64_t c;        // constant bits
    uint64_t magic;    // K_DIVM_U / K_MODM_U
    uint32_t shift;
    uint32_t add;    // libdivide "add" marker
    int32_t sdtype;  // FQ_OPERAND_STACK: dtype of the popped value (cast to `dtype`)
    int32_t pad;
};

struct KProg {
    int32_t n;
    int32_t out_dtype;
    KStep s[FQ_MAX_STEPS + 4];  // room for inserted casts
};

// one comparison of an and/or predicate tree (FQ_PRED_TREE)
struct KLeaf {
    int32_t cmp;
    int32_t cmp_dtype;
    int32_t rhs_operand;
    int32_t pad;
    uint64_t rhs;
    KProg lhs;
};

struct KPred {
    int32_t kind;
    int32_t cmp;
    int32_t cmp_dtype;
    int32_t rhs_operand;
    uint64_t rhs;
    const uint64_t *bitmap;
    KProg lhs;
    // FQ_PRED_TREE: the leaves and the tree as a truth table over the leaf
    // results (bit i of `truth` = value for leaf bits i); `prog` is the
    // postfix form the hipRTC generator turns into a boolean expression
    int32_t n_leaves;
    uint32_t truth;
    int32_t n_prog;
    int32_t prog[2 * FQ_MAX_PRED_LEAVES];
    KLeaf leaves[FQ_MAX_PRED_LEAVES];
};

// Per-workgroup partial; same field order as fq_agg_state.
struct Partial {
    uint64_t sum, max, min, count, blocks;
    uint32_t flags;
    int32_t dtype;
};
static_assert(sizeof(Partial) == sizeof(fq_agg_state), "partial layout");

// ---------------------------------------------------------------------------
// value <-> 64-bit encoding (fq_value: ints sign/zero extended, floats binary64)
// ---------------------------------------------------------------------------
template <typename T>
__host__ __device__ inline uint64_t to_bits(T v) {
    if constexpr (sizeof(T) == 8 && __is_same(T, double)) {
        return __builtin_bit_cast(uint64_t, v);
    } else if constexpr (__is_same(T, float)) {
        return __builtin_bit_cast(uint64_t, (double)v);
    } else if constexpr (T(-1) < T(0)) {
        return (uint64_t)(int64_t)v;
    } else {
        return (uint64_t)v;
    }
}

template <typename T>
__host__ __device__ inline T from_bits(uint64_t b) {
    if constexpr (__is_same(T, double)) {
        return __builtin_bit_cast(double, b);
    } else if constexpr (__is_same(T, float)) {
        return (float)__builtin_bit_cast(double, b);
    } else {
        return (T)b;
    }
}

template <typename T>
struct Lim;
#define FQ_LIM(T, LO, HI)                              \
    template <>                                         \
    struct Lim<T> {                                     \
        __host__ __device__ static constexpr T lo() { return LO; } \
        __host__ __device__ static constexpr T hi() { return HI; } \
    };
FQ_LIM(int8_t, INT8_MIN, INT8_MAX)
FQ_LIM(int16_t, INT16_MIN, INT16_MAX)
FQ_LIM(int32_t, INT32_MIN, INT32_MAX)
FQ_LIM(int64_t, INT64_MIN, INT64_MAX)
FQ_LIM(uint8_t, 0, UINT8_MAX)
FQ_LIM(uint16_t, 0, UINT16_MAX)
FQ_LIM(uint32_t, 0, UINT32_MAX)
FQ_LIM(uint64_t, 0, UINT64_MAX)
FQ_LIM(float, -__builtin_huge_valf(), __builtin_huge_valf())
FQ_LIM(double, -__builtin_huge_val(), __builtin_huge_val())
#undef FQ_LIM

// max/min with arrow's comparison form (min_max_helper: keep the running value
// unless the candidate compares strictly better).
template <typename V>
__device__ __forceinline__ V vmax(V a, V b) { return b > a ? b : a; }
template <typename V>
__device__ __forceinline__ V vmin(V a, V b) { return b < a ? b : a; }

// ---------------------------------------------------------------------------
// Column element -> step dtype (operand = FQ_OPERAND_COLUMN)
// ---------------------------------------------------------------------------
template <typename TIn>
__device__ __forceinline__ uint64_t col_as(int32_t dtype, TIn x, bool live, uint32_t &flags) {
    if (dtype == FQ_DT_FLOAT64) {
        return __builtin_bit_cast(uint64_t, (double)x);
    }
    if constexpr (__is_same(TIn, uint64_t)) {
        if (dtype == FQ_DT_INT64 && (x >> 63) && live) flags |= FQ_STATE_CAST_NULL;
    }
    return to_bits<TIn>(x);
}

// u64 division by a constant (libdivide round-up method; magic built on host)
__device__ __forceinline__ uint64_t divm_u64(uint64_t x, uint64_t magic, uint32_t shift,
                                             uint32_t add) {
    uint64_t q = __umul64hi(x, magic);
    if (add) {
        uint64_t t = ((x - q) >> 1) + q;
        return t >> shift;
    }
    return q >> shift;
}

// u32 n % d with a 32-bit round-up magic (libdivide u32 method; host-built)
__device__ __forceinline__ uint32_t modm_u32(uint32_t n, uint32_t magic, uint32_t shift, uint32_t add, uint32_t d) {
    uint32_t q = __umulhi(n, magic);
    q = add ? ((((n - q) >> 1) + q) >> shift) : (q >> shift);
    return n - q * d;
}

// u64 x % d for d <= 65535 (K_MODM32_U): mm = magic | (2^32 % d) << 32
__device__ __forceinline__ uint64_t modm32_u64(uint64_t x, uint64_t mm, uint32_t shift, uint32_t add, uint64_t d) {
    const uint32_t m = (uint32_t)mm, c2 = (uint32_t)(mm >> 32), dd = (uint32_t)d;
    const uint32_t rh = modm_u32((uint32_t)(x >> 32), m, shift, add, dd);
    const uint32_t rl = modm_u32((uint32_t)x, m, shift, add, dd);
    return modm_u32(rh * c2 + rl, m, shift, add, dd);
}

__device__ __forceinline__ uint32_t divm_u32(uint32_t n, uint32_t magic, uint32_t shift, uint32_t add) {
    const uint32_t q = __umulhi(n, magic);
    return add ? ((((n - q) >> 1) + q) >> shift) : (q >> shift);
}

// u64 x / d for d <= 65535 (K_DIVM32_U): qh = hi / d, then the remainder and
// the low word's two 16-bit digits (each partial dividend < d * 2^16 < 2^32)
__device__ __forceinline__ uint64_t divm32_u64(uint64_t x, uint32_t magic, uint32_t shift, uint32_t add, uint32_t d) {
    const uint32_t hi = (uint32_t)(x >> 32), lo = (uint32_t)x;
    const uint32_t qh = divm_u32(hi, magic, shift, add), rh = hi - qh * d;
    const uint32_t t1 = (rh << 16) | (lo >> 16);
    const uint32_t q1 = divm_u32(t1, magic, shift, add), r1 = t1 - q1 * d;
    const uint32_t q0 = divm_u32((r1 << 16) | (lo & 0xffffu), magic, shift, add);
    return ((uint64_t)qh << 32) | ((q1 << 16) + q0);
}

// Rare, long operations are out-of-line calls so that the unrolled program
// interpreter stays small enough for the instruction cache (a 64-bit divide
// or fmod unrolled over E elements is thousands of instructions).
__device__ __noinline__ inline uint64_t slow_divmod(int32_t code, uint64_t a, uint64_t b);

// ---------------------------------------------------------------------------
// The expression program, run over E elements per lane.  Every switch is on a
// wave-uniform kernel argument, so each branch is a scalar jump; the element
// loops inside are fully unrolled with static register indices.
// `live` marks the elements whose rows reach this expression (in-range and,
// for the value expression, passing the predicate); only they raise flags,
// matching arrow evaluating the expression on the filtered block.
// ---------------------------------------------------------------------------
template <int E, typename TIn>
__device__ __forceinline__ void run_prog(const KProg &p, const TIn (&x)[E], uint64_t (&a)[E],
                                         uint32_t live, uint32_t &flags) {
    for (int s = 0; s < p.n; ++s) {
        const KStep st = p.s[s];
        const int32_t code = st.code;
        if (code == K_CAST_U2I) {
#pragma unroll
            for (int j = 0; j < E; ++j)
                if ((a[j] >> 63) && ((live >> j) & 1u)) flags |= FQ_STATE_CAST_NULL;
            continue;
        }
        if (code == K_CAST_U2F) {
#pragma unroll
            for (int j = 0; j < E; ++j) a[j] = __builtin_bit_cast(uint64_t, (double)a[j]);
            continue;
        }
        if (code == K_CAST_I2F) {
#pragma unroll
            for (int j = 0; j < E; ++j)
                a[j] = __builtin_bit_cast(uint64_t, (double)(int64_t)a[j]);
            continue;
        }
        uint64_t b[E];
        if (st.operand == FQ_OPERAND_COLUMN) {
#pragma unroll
            for (int j = 0; j < E; ++j) b[j] = col_as<TIn>(st.dtype, x[j], (live >> j) & 1u, flags);
        } else {
#pragma unroll
            for (int j = 0; j < E; ++j) b[j] = st.c;
        }
        if (st.reversed) {
#pragma unroll
            for (int j = 0; j < E; ++j) {
                uint64_t t = a[j];
                a[j] = b[j];
                b[j] = t;
            }
        }
        switch (code) {
            case K_ADD_I:
#pragma unroll
                for (int j = 0; j < E; ++j) a[j] = a[j] + b[j];
                break;
            case K_SUB_I:
#pragma unroll
                for (int j = 0; j < E; ++j) a[j] = a[j] - b[j];
                break;
            case K_MUL_I:
#pragma unroll
                for (int j = 0; j < E; ++j) a[j] = a[j] * b[j];
                break;
            case K_DIV_U:
            case K_MOD_U:
            case K_DIV_S:
            case K_MOD_S:
#pragma unroll
                for (int j = 0; j < E; ++j) {
                    if (b[j] == 0 && ((live >> j) & 1u)) flags |= FQ_STATE_DIV_ZERO;
                    a[j] = slow_divmod(code, a[j], b[j]);
                }
                break;
            case K_SHR_U:
#pragma unroll
                for (int j = 0; j < E; ++j) a[j] = a[j] >> st.shift;
                break;
            case K_AND_U:
#pragma unroll
                for (int j = 0; j < E; ++j) a[j] = a[j] & st.magic;
                break;
            case K_DIVM_U:
#pragma unroll
                for (int j = 0; j < E; ++j) a[j] = divm_u64(a[j], st.magic, st.shift, st.add);
                break;
            case K_MODM_U:
#pragma unroll
                for (int j = 0; j < E; ++j)
                    a[j] = a[j] - divm_u64(a[j], st.magic, st.shift, st.add) * st.c;
                break;
            case K_MODM32_U:
#pragma unroll
                for (int j = 0; j < E; ++j) a[j] = modm32_u64(a[j], st.magic, st.shift, st.add, st.c);
                break;
            case K_DIVM32_U:
#pragma unroll
                for (int j = 0; j < E; ++j) a[j] = divm32_u64(a[j], (uint32_t)st.magic, st.shift, st.add, (uint32_t)st.c);
                break;
            case K_ADD_F:
#pragma unroll
                for (int j = 0; j < E; ++j)
                    a[j] = __builtin_bit_cast(uint64_t, __builtin_bit_cast(double, a[j]) + __builtin_bit_cast(double, b[j]));
                break;
            case K_SUB_F:
#pragma unroll
                for (int j = 0; j < E; ++j)
                    a[j] = __builtin_bit_cast(uint64_t, __builtin_bit_cast(double, a[j]) - __builtin_bit_cast(double, b[j]));
                break;
            case K_MUL_F:
#pragma unroll
                for (int j = 0; j < E; ++j)
                    a[j] = __builtin_bit_cast(uint64_t, __builtin_bit_cast(double, a[j]) * __builtin_bit_cast(double, b[j]));
                break;
            case K_DIV_F:
            case K_MOD_F:
#pragma unroll
                for (int j = 0; j < E; ++j) {
                    if (__builtin_bit_cast(double, b[j]) == 0.0 && ((live >> j) & 1u)) flags |= FQ_STATE_DIV_ZERO;
                    a[j] = slow_divmod(code, a[j], b[j]);
                }
                break;
            default:
                break;
        }
    }
}

// a OP b for the generic divide/modulo codes; a zero divisor yields 0 (the
// caller raises DIV_ZERO for live rows).  i64::MIN / -1 wraps (unpinned in
// the reference).
__device__ __noinline__ inline uint64_t slow_divmod(int32_t code, uint64_t a, uint64_t b) {
    switch (code) {
        case K_DIV_U:
            return b ? a / b : 0;
        case K_MOD_U:
            return b ? a % b : 0;
        case K_DIV_S:
        case K_MOD_S: {
            const int64_t sa = (int64_t)a, sb = (int64_t)b;
            if (sb == 0) return 0;
            if (sb == -1) return code == K_DIV_S ? (uint64_t)0 - a : 0;
            return (uint64_t)(code == K_DIV_S ? sa / sb : sa % sb);
        }
        case K_DIV_F:
            return __builtin_bit_cast(uint64_t, __builtin_bit_cast(double, a) / __builtin_bit_cast(double, b));
        case K_MOD_F:
            return __builtin_bit_cast(uint64_t, fmod(__builtin_bit_cast(double, a), __builtin_bit_cast(double, b)));
        default:
            return a;
    }
}

// comparison of two values already in cmp_dtype; returns a bit per element
template <int E>
__device__ __forceinline__ uint32_t cmp_mask(int32_t cmp, int32_t dt, const uint64_t (&l)[E],
                                             const uint64_t (&r)[E]) {
    uint32_t m = 0;
#define FQ_CMP_LOOP(T, CONV, OP)                                \
    _Pragma("unroll") for (int j = 0; j < E; ++j) {             \
        const T lv = CONV(l[j]), rv = CONV(r[j]);               \
        m |= (uint32_t)(lv OP rv) << j;                         \
    }                                                           \
    break;
#define FQ_U(x) (x)
#define FQ_S(x) ((int64_t)(x))
#define FQ_F(x) (__builtin_bit_cast(double, (x)))
    const int32_t key = dt * 8 + cmp;
    switch (key) {
        case FQ_DT_UINT64 * 8 + FQ_CMP_EQ: FQ_CMP_LOOP(uint64_t, FQ_U, ==)
        case FQ_DT_UINT64 * 8 + FQ_CMP_LT: FQ_CMP_LOOP(uint64_t, FQ_U, <)
        case FQ_DT_UINT64 * 8 + FQ_CMP_LTEQ: FQ_CMP_LOOP(uint64_t, FQ_U, <=)
        case FQ_DT_UINT64 * 8 + FQ_CMP_GT: FQ_CMP_LOOP(uint64_t, FQ_U, >)
        case FQ_DT_UINT64 * 8 + FQ_CMP_GTEQ: FQ_CMP_LOOP(uint64_t, FQ_U, >=)
        case FQ_DT_INT64 * 8 + FQ_CMP_EQ: FQ_CMP_LOOP(int64_t, FQ_S, ==)
        case FQ_DT_INT64 * 8 + FQ_CMP_LT: FQ_CMP_LOOP(int64_t, FQ_S, <)
        case FQ_DT_INT64 * 8 + FQ_CMP_LTEQ: FQ_CMP_LOOP(int64_t, FQ_S, <=)
        case FQ_DT_INT64 * 8 + FQ_CMP_GT: FQ_CMP_LOOP(int64_t, FQ_S, >)
        case FQ_DT_INT64 * 8 + FQ_CMP_GTEQ: FQ_CMP_LOOP(int64_t, FQ_S, >=)
        case FQ_DT_FLOAT64 * 8 + FQ_CMP_EQ: FQ_CMP_LOOP(double, FQ_F, ==)
        case FQ_DT_FLOAT64 * 8 + FQ_CMP_LT: FQ_CMP_LOOP(double, FQ_F, <)
        case FQ_DT_FLOAT64 * 8 + FQ_CMP_LTEQ: FQ_CMP_LOOP(double, FQ_F, <=)
        case FQ_DT_FLOAT64 * 8 + FQ_CMP_GT: FQ_CMP_LOOP(double, FQ_F, >)
        case FQ_DT_FLOAT64 * 8 + FQ_CMP_GTEQ: FQ_CMP_LOOP(double, FQ_F, >=)
        default:
            break;
    }
#undef FQ_CMP_LOOP
#undef FQ_U
#undef FQ_S
#undef FQ_F
    return m;
}

// ---------------------------------------------------------------------------
// wave64 reductions (2 x 32-bit DPP/permute moves per 64-bit shuffle)
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T shfl_xor64(T v, int m) {
    if constexpr (sizeof(T) == 8) {
        const uint64_t b = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = __shfl_xor((unsigned)(b & 0xffffffffu), m, kWave);
        const uint32_t hi = __shfl_xor((unsigned)(b >> 32), m, kWave);
        return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
    } else if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, (unsigned)__shfl_xor(__builtin_bit_cast(unsigned, v), m, kWave));
    } else {
        return (T)__shfl_xor((int)v, m, kWave);
    }
}

// 64-bit value of lane `src` / of lane (lane - d) (2 x 32-bit moves)
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = __shfl((unsigned)(v & 0xffffffffu), src, kWave);
    const uint32_t hi = __shfl((unsigned)(v >> 32), src, kWave);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
    const uint32_t lo = __shfl_up((unsigned)(v & 0xffffffffu), d, kWave);
    const uint32_t hi = __shfl_up((unsigned)(v >> 32), d, kWave);
    return ((uint64_t)hi << 32) | lo;
}

}  // namespace fqk
