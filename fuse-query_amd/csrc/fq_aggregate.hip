// Fused AggregatePartial scan for gfx950.
//
// Replaces, per device block (one numbers_mt partition or one DataBlock):
//   FilterTransform::expression_executor  (transform_filter.rs:38-55)   -> predicate
//   AggregatorFunction::accumulate        (function_aggregator.rs:57-100)
//     arg.eval  -> ArithmeticFunction chain (function_arithmetic.rs:64-72)
//     data_array_aggregate_op sum/min/max (data_array_aggregate.rs:14-163)
// with ONE read of the column from HBM: coalesced 16-byte loads (4 in flight
// per lane), per-lane accumulators in registers, a wave64 butterfly reduce,
// an LDS combine across the 4 waves of a workgroup, one Partial per
// workgroup, and a single-workgroup finalize in a fixed order (so float sums
// are reproducible run to run).  No MFMA: nothing here is a contraction.
//
// Block mode: when a predicate is fused with sum(), the reference's per-block
// state machine errors if ANY 10,000-row block is empty after filtering
// (arrow sum -> None, data_value_arithmetic.rs:10-27).  Block mode assigns
// whole reference blocks to waves and reduces "any row passed" with one
// ballot per block, so that flag is exact.
#include <hip/hip_runtime.h>

#include <string>

#include "fq_common.h"
#include "fq_device.h"
#include "fq_scan.h"

namespace fqk {

template <typename V>
struct Acc {
    V sum, mx, mn;
    uint64_t cnt;
    uint32_t flags;
    __device__ void init() {
        sum = V(0);
        mx = Lim<V>::lo();
        mn = Lim<V>::hi();
        cnt = 0;
        flags = 0;
    }
};

// Evaluate predicate and value expression for M elements, accumulate.
// Returns the pass mask (bit j = element j passed and is live).
template <typename TIn, typename V, int PRED, bool CHAIN, int M>
__device__ __forceinline__ uint32_t process(const TIn (&x)[M], const int64_t (&idx)[M],
                                            uint32_t live, const KPred &pred, const KProg &val,
                                            uint32_t mask, Acc<V> &acc) {
    uint32_t pass = live;
    if constexpr (PRED == FQ_PRED_EXPR) {
        uint64_t l[M], r[M];
#pragma unroll
        for (int j = 0; j < M; ++j) l[j] = to_bits<TIn>(x[j]);
        run_prog<M, TIn>(pred.lhs, x, l, live, acc.flags);
        if (pred.rhs_operand == FQ_OPERAND_COLUMN) {
#pragma unroll
            for (int j = 0; j < M; ++j)
                r[j] = col_as<TIn>(pred.cmp_dtype, x[j], (live >> j) & 1u, acc.flags);
        } else {
#pragma unroll
            for (int j = 0; j < M; ++j) r[j] = pred.rhs;
        }
        pass &= cmp_mask<M>(pred.cmp, pred.cmp_dtype, l, r);
    } else if constexpr (PRED == FQ_PRED_BITMAP) {
#pragma unroll
        for (int j = 0; j < M; ++j) {
            if ((live >> j) & 1u) {
                const uint64_t w = pred.bitmap[idx[j] >> 6];
                if (!((w >> (idx[j] & 63)) & 1ull)) pass &= ~(1u << j);
            }
        }
    } else if constexpr (PRED == FQ_PRED_TREE) {
        // every leaf over every live row (arrow and/or evaluate both sides),
        // then the tree through its truth table
        uint32_t m[FQ_MAX_PRED_LEAVES] = {};
#pragma unroll
        for (int li = 0; li < FQ_MAX_PRED_LEAVES; ++li) {
            if (li >= pred.n_leaves) break;
            const KLeaf &lf = pred.leaves[li];
            uint64_t l[M], r[M];
#pragma unroll
            for (int j = 0; j < M; ++j) l[j] = to_bits<TIn>(x[j]);
            run_prog<M, TIn>(lf.lhs, x, l, live, acc.flags);
            if (lf.rhs_operand == FQ_OPERAND_COLUMN) {
#pragma unroll
                for (int j = 0; j < M; ++j) r[j] = col_as<TIn>(lf.cmp_dtype, x[j], (live >> j) & 1u, acc.flags);
            } else {
#pragma unroll
                for (int j = 0; j < M; ++j) r[j] = lf.rhs;
            }
            m[li] = cmp_mask<M>(lf.cmp, lf.cmp_dtype, l, r);
        }
        uint32_t t = 0;
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const uint32_t idxbits = ((m[0] >> j) & 1u) | (((m[1] >> j) & 1u) << 1) | (((m[2] >> j) & 1u) << 2) |
                                     (((m[3] >> j) & 1u) << 3);
            t |= ((pred.truth >> idxbits) & 1u) << j;
        }
        pass &= t;
    }
    V v[M];
    if constexpr (CHAIN) {
        uint64_t a[M];
#pragma unroll
        for (int j = 0; j < M; ++j) a[j] = to_bits<TIn>(x[j]);
        run_prog<M, TIn>(val, x, a, pass, acc.flags);
#pragma unroll
        for (int j = 0; j < M; ++j) v[j] = from_bits<V>(a[j]);
    } else {
#pragma unroll
        for (int j = 0; j < M; ++j) v[j] = (V)x[j];
    }
    if (mask & FQ_AGG_SUM) {
#pragma unroll
        for (int j = 0; j < M; ++j) acc.sum = acc.sum + (((pass >> j) & 1u) ? v[j] : V(0));
    }
    if (mask & FQ_AGG_MAX) {
#pragma unroll
        for (int j = 0; j < M; ++j) acc.mx = ((pass >> j) & 1u) ? vmax(acc.mx, v[j]) : acc.mx;
    }
    if (mask & FQ_AGG_MIN) {
#pragma unroll
        for (int j = 0; j < M; ++j) acc.mn = ((pass >> j) & 1u) ? vmin(acc.mn, v[j]) : acc.mn;
    }
    acc.cnt += __builtin_popcount(pass);
    return pass;
}

// wave butterfly + LDS combine; thread 0 of the workgroup stores the result
template <typename V>
__device__ __forceinline__ void reduce_and_store(Acc<V> &acc, Partial *out, int32_t dtype) {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
        acc.sum = acc.sum + shfl_xor64(acc.sum, off);
        acc.mx = vmax(acc.mx, shfl_xor64(acc.mx, off));
        acc.mn = vmin(acc.mn, shfl_xor64(acc.mn, off));
        acc.cnt += shfl_xor64(acc.cnt, off);
        acc.flags |= (uint32_t)__shfl_xor((int)acc.flags, off, kWave);
    }
    __shared__ V s_sum[kThreads / kWave], s_mx[kThreads / kWave], s_mn[kThreads / kWave];
    __shared__ uint64_t s_cnt[kThreads / kWave];
    __shared__ uint32_t s_flags[kThreads / kWave];
    const int wave = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
        s_sum[wave] = acc.sum;
        s_mx[wave] = acc.mx;
        s_mn[wave] = acc.mn;
        s_cnt[wave] = acc.cnt;
        s_flags[wave] = acc.flags;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        V sum = s_sum[0], mx = s_mx[0], mn = s_mn[0];
        uint64_t cnt = s_cnt[0];
        uint32_t flags = s_flags[0];
#pragma unroll
        for (int w = 1; w < kThreads / kWave; ++w) {
            sum = sum + s_sum[w];
            mx = vmax(mx, s_mx[w]);
            mn = vmin(mn, s_mn[w]);
            cnt += s_cnt[w];
            flags |= s_flags[w];
        }
        Partial p;
        p.sum = to_bits<V>(sum);
        p.max = to_bits<V>(mx);
        p.min = to_bits<V>(mn);
        p.count = cnt;
        p.blocks = 0;
        p.flags = flags;
        p.dtype = dtype;
        *out = p;
    }
}

// The launch's partials folded in a fixed order by ONE workgroup: thread t
// folds partials t, t+256, ... then the wave butterfly and the LDS combine,
// so a grid gives the same bytes run to run (float sums too).  An in-launch
// fold by the scan's last workgroup (agent-scope release / ticket / acquire)
// measured slower than this separate 4.4 us launch: 8 scans 11.07 against
// 11.02 ms (profiles/r05_b_scan_fin_ab.json), and was removed in round 6.
template <typename V>
__device__ __forceinline__ void fold_partials(Partial *parts, int nparts, uint64_t blocks, uint64_t rows,
                                              int32_t vdtype, int empty_if_zero, fq_agg_state *out) {
    Acc<V> acc;
    acc.init();
    if (threadIdx.x == 0) acc.cnt = rows;  // count-only scans: no column read (nparts == 0)
    for (int i = threadIdx.x; i < nparts; i += kThreads) {
        const Partial p = parts[i];
        acc.sum = acc.sum + from_bits<V>(p.sum);
        acc.mx = vmax(acc.mx, from_bits<V>(p.max));
        acc.mn = vmin(acc.mn, from_bits<V>(p.min));
        acc.cnt += p.count;
        acc.flags |= p.flags;
    }
    __shared__ Partial s_out;
    reduce_and_store<V>(acc, &s_out, vdtype);
    __syncthreads();
    if (threadIdx.x == 0) {
        fq_agg_state r;
        r.sum = s_out.sum;
        r.max = s_out.max;
        r.min = s_out.min;
        r.count = s_out.count;
        r.blocks = blocks;
        r.flags = s_out.flags;
        if (empty_if_zero && r.count == 0) r.flags |= FQ_STATE_ANY_EMPTY;
        r.dtype = vdtype;
        *out = r;
    }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Flat streaming mode: grid-stride over 16-byte vectors, U vectors in flight
// per lane.  `head` scalar elements precede the first 16-byte boundary.
template <typename TIn, typename V, int PRED, bool CHAIN, int U, bool PF = false>
__global__ void __launch_bounds__(kThreads)
    agg_flat_kernel(const TIn *__restrict__ col, int64_t n, int64_t head, KPred pred, KProg val,
                    uint32_t mask, int32_t vdtype, Partial *parts) {
    constexpr int VE = 16 / sizeof(TIn);
    constexpr int E = VE * U;
    static_assert(E <= 32, "pass mask is 32 bits");
    Acc<V> acc;
    acc.init();
    const int64_t T = (int64_t)gridDim.x * kThreads;
    const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const int64_t nvec = (n - head) / VE;
    const u32x4 *__restrict__ vp = reinterpret_cast<const u32x4 *>(col + head);
    constexpr uint32_t kFull = (E == 32) ? 0xffffffffu : ((1u << E) - 1u);

    // Tile-contiguous streaming: a workgroup reads one contiguous tile of
    // U * 256 vectors (16 KB for u64 at U=4) per iteration, non-temporal,
    // and strides over tiles by the grid.  Measured on MI355X against the
    // vector-granular grid stride: 7.2 vs 6.2 TB/s (tools/tune_scan.py,
    // profiles/r01_tune_*.json); few workgroups per CU (see launch) helps too.
    constexpr int64_t TV = (int64_t)U * kThreads;
    const int64_t ntiles = nvec / TV;
    u32x4 nxt[U];  // PF: the next tile's vectors in flight while this tile is reduced (launch_scan)
    if constexpr (PF) {
        if ((int64_t)blockIdx.x < ntiles) {
#pragma unroll
            for (int k = 0; k < U; ++k)
                nxt[k] = __builtin_nontemporal_load(vp + (int64_t)blockIdx.x * TV + threadIdx.x + (int64_t)k * kThreads);
        }
    }
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t base = t * TV + threadIdx.x;
        u32x4 raw[U];
        if constexpr (PF) {
#pragma unroll
            for (int k = 0; k < U; ++k) raw[k] = nxt[k];
            const int64_t tn = t + gridDim.x;
            if (tn < ntiles) {
#pragma unroll
                for (int k = 0; k < U; ++k)
                    nxt[k] = __builtin_nontemporal_load(vp + tn * TV + threadIdx.x + (int64_t)k * kThreads);
            }
        } else {
#pragma unroll
            for (int k = 0; k < U; ++k) raw[k] = __builtin_nontemporal_load(vp + base + (int64_t)k * kThreads);
        }
        TIn x[E];
        int64_t idx[E];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            __builtin_memcpy(&x[k * VE], &raw[k], 16);
#pragma unroll
            for (int e = 0; e < VE; ++e) idx[k * VE + e] = head + (base + (int64_t)k * kThreads) * VE + e;
        }
        process<TIn, V, PRED, CHAIN, E>(x, idx, kFull, pred, val, mask, acc);
    }
    for (int64_t v = ntiles * TV + g; v < nvec; v += T) {
        const u32x4 raw = __builtin_nontemporal_load(vp + v);
        TIn x[VE];
        int64_t idx[VE];
        __builtin_memcpy(&x[0], &raw, 16);
#pragma unroll
        for (int e = 0; e < VE; ++e) idx[e] = head + v * VE + e;
        process<TIn, V, PRED, CHAIN, VE>(x, idx, (1u << VE) - 1u, pred, val, mask, acc);
    }
    // scalar edges: [0, head) and [head + nvec*VE, n)
    const int64_t tail0 = head + nvec * VE;
    const int64_t nedge = head + (n - tail0);
    for (int64_t t = g; t < nedge; t += T) {
        const int64_t i = t < head ? t : tail0 + (t - head);
        TIn x[1] = {col[i]};
        int64_t idx[1] = {i};
        process<TIn, V, PRED, CHAIN, 1>(x, idx, 1u, pred, val, mask, acc);
    }
    reduce_and_store<V>(acc, parts + blockIdx.x, vdtype);
}

// Block mode: one wave owns whole reference blocks of R rows; one ballot per
// block tells whether any of its rows survived the predicate.
template <typename TIn, typename V, int PRED, bool CHAIN, int U>
__global__ void __launch_bounds__(kThreads)
    agg_block_kernel(const TIn *__restrict__ col, int64_t n, int64_t R, KPred pred, KProg val,
                     uint32_t mask, int32_t vdtype, Partial *parts) {
    Acc<V> acc;
    acc.init();
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t w = ((int64_t)blockIdx.x * kThreads + threadIdx.x) / kWave;
    const int64_t W = ((int64_t)gridDim.x * kThreads) / kWave;
    const int64_t nb = (n + R - 1) / R;
    for (int64_t b = w; b < nb; b += W) {
        const int64_t s = b * R;
        const int64_t e = (s + R < n) ? s + R : n;
        uint32_t any = 0;
        for (int64_t i = s + lane; i < e; i += (int64_t)kWave * U) {
            TIn x[U];
            int64_t idx[U];
            uint32_t live = 0;
#pragma unroll
            for (int k = 0; k < U; ++k) {
                idx[k] = i + (int64_t)k * kWave;
                if (idx[k] < e) {
                    x[k] = __builtin_nontemporal_load(col + idx[k]);
                    live |= 1u << k;
                } else {
                    x[k] = TIn(0);
                }
            }
            any |= process<TIn, V, PRED, CHAIN, U>(x, idx, live, pred, val, mask, acc);
        }
        if (__ballot(any != 0) == 0ull) acc.flags |= FQ_STATE_ANY_EMPTY;
    }
    reduce_and_store<V>(acc, parts + blockIdx.x, vdtype);
}

// Single workgroup, fixed order (fold_partials): the result is deterministic
// for a given grid.
template <typename V>
__global__ void __launch_bounds__(kThreads)
    agg_finalize_kernel(Partial *parts, int nparts, uint64_t blocks, uint64_t rows, int32_t vdtype,
                        int empty_if_zero, fq_agg_state *out) {
    fold_partials<V>(parts, nparts, blocks, rows, vdtype, empty_if_zero, out);
}

// ---------------------------------------------------------------------------
// host-side lowering and dispatch
// ---------------------------------------------------------------------------

static bool is_pow2(uint64_t v) { return v && !(v & (v - 1)); }

// Workgroups per CU for the flat scan (FQ_TUNE_SCAN_WG_PER_CU, default 2).
static int scan_wg_per_cu() { return (int)fqc::knob(FQ_TUNE_SCAN_WG_PER_CU); }

// libdivide's u64 round-up magic (branchful form)
static void u64_magic(uint64_t d, uint64_t &magic, uint32_t &shift, uint32_t &add) {
    const uint32_t l = 63 - __builtin_clzll(d);
    const unsigned __int128 num = (unsigned __int128)1 << (64 + l);
    uint64_t proposed = (uint64_t)(num / d);
    const uint64_t rem = (uint64_t)(num % d);
    const uint64_t e = d - rem;
    if (e < (1ull << l)) {
        add = 0;
    } else {
        proposed += proposed;
        const uint64_t twice_rem = rem + rem;
        if (twice_rem >= d || twice_rem < rem) proposed += 1;
        add = 1;
    }
    shift = l;
    magic = proposed + 1;
}

// libdivide's u32 round-up magic (branchful form), for K_MODM32_U
static void u32_magic(uint32_t d, uint32_t &magic, uint32_t &shift, uint32_t &add) {
    const uint32_t l = 31 - __builtin_clz(d);
    const uint64_t num = (uint64_t)1 << (32 + l);
    uint32_t proposed = (uint32_t)(num / d);
    const uint32_t rem = (uint32_t)(num % d);
    const uint32_t e = d - rem;
    if (e < (1u << l)) {
        add = 0;
    } else {
        proposed += proposed;
        const uint32_t twice_rem = rem + rem;
        if (twice_rem >= d || twice_rem < rem) proposed += 1;
        add = 1;
    }
    shift = l;
    magic = proposed + 1;
}

static bool is_chain_dtype(int32_t dt) {
    return dt == FQ_DT_UINT64 || dt == FQ_DT_INT64 || dt == FQ_DT_FLOAT64;
}

static fq_status push_cast(int32_t from, int32_t to, KProg &out) {
    if (from == to) return FQ_OK;
    if (out.n >= (int)(sizeof(out.s) / sizeof(out.s[0])))
        return fqc::fail(FQ_E_UNSUPPORTED, "expression too long for the fused device path");
    KStep &s = out.s[out.n++];
    s = KStep{};
    s.dtype = to;
    if (from == FQ_DT_UINT64 && to == FQ_DT_INT64) s.code = K_CAST_U2I;
    else if (from == FQ_DT_UINT64 && to == FQ_DT_FLOAT64) s.code = K_CAST_U2F;
    else if (from == FQ_DT_INT64 && to == FQ_DT_FLOAT64) s.code = K_CAST_I2F;
    else
        return fqc::fail(FQ_E_UNSUPPORTED, std::string("fused cast ") + fqc::dtype_name(from) + " -> " +
                                               fqc::dtype_name(to) + " is not supported on the device path");
    return FQ_OK;
}

// fq_expr (semantic) -> KProg (lowered).  Returns the resulting dtype.
fq_status lower_expr(const fq_expr &e, int32_t col_dtype, KProg &out, int32_t &res_dtype) {
    out.n = 0;
    int32_t acc = col_dtype;
    if (e.n_steps < 0 || e.n_steps > FQ_MAX_STEPS)
        return fqc::fail(FQ_E_INVALID, "fq_expr: n_steps out of range");
    if (e.n_steps > 0 && !is_chain_dtype(col_dtype))
        return fqc::fail(FQ_E_UNSUPPORTED, std::string("fused expressions over ") + fqc::dtype_name(col_dtype) +
                                               " columns are not supported on the device path");
    int32_t stack[FQ_MAX_STACK];
    int depth = 0;
    for (int i = 0; i < e.n_steps; ++i) {
        const fq_step &st = e.steps[i];
        if (st.op == FQ_OP_PUSH) {  // expression tree: acc onto the stack, restart from the column
            if (depth >= FQ_MAX_STACK) return fqc::fail(FQ_E_UNSUPPORTED, "expression tree too deep for the fused device path");
            if (!is_chain_dtype(col_dtype)) return fqc::fail(FQ_E_UNSUPPORTED, "fused expression trees need a 64-bit column");
            if (out.n >= (int)(sizeof(out.s) / sizeof(out.s[0])))
                return fqc::fail(FQ_E_UNSUPPORTED, "expression too long for the fused device path");
            KStep &k = out.s[out.n++];
            k = KStep{};
            k.code = K_PUSH;
            k.dtype = col_dtype;
            stack[depth++] = acc;
            acc = col_dtype;
            continue;
        }
        if (!is_chain_dtype(st.dtype))
            return fqc::fail(FQ_E_UNSUPPORTED, "fused step dtype must be UInt64, Int64 or Float64");
        int32_t sdt = 0;
        if (st.operand == FQ_OPERAND_STACK) {
            if (depth == 0) return fqc::fail(FQ_E_INVALID, "fq_step: stack operand without a pushed value");
            sdt = stack[--depth];
            if (sdt != st.dtype && !(sdt == FQ_DT_UINT64 && st.dtype != FQ_DT_UINT64) &&
                !(sdt == FQ_DT_INT64 && st.dtype == FQ_DT_FLOAT64))
                return fqc::fail(FQ_E_UNSUPPORTED, std::string("fused cast ") + fqc::dtype_name(sdt) + " -> " +
                                                       fqc::dtype_name(st.dtype) + " is not supported on the device path");
        } else if (st.operand != FQ_OPERAND_CONST && st.operand != FQ_OPERAND_COLUMN) {
            return fqc::fail(FQ_E_INVALID, "fq_step: bad operand kind");
        }
        fq_status s = push_cast(acc, st.dtype, out);
        if (s != FQ_OK) return s;
        if (st.operand == FQ_OPERAND_COLUMN && col_dtype == FQ_DT_FLOAT64 && st.dtype != FQ_DT_FLOAT64)
            return fqc::fail(FQ_E_INVALID, "fq_step: Float64 column operand in an integer step");
        if (out.n >= (int)(sizeof(out.s) / sizeof(out.s[0])))
            return fqc::fail(FQ_E_UNSUPPORTED, "expression too long for the fused device path");
        KStep &k = out.s[out.n++];
        k = KStep{};
        k.operand = st.operand;
        k.reversed = st.reversed;
        k.dtype = st.dtype;
        k.sdtype = sdt;
        k.c = st.bits;
        const bool konst = st.operand == FQ_OPERAND_CONST && !st.reversed;
        if (st.dtype == FQ_DT_FLOAT64) {
            switch (st.op) {
                case FQ_OP_ADD: k.code = K_ADD_F; break;
                case FQ_OP_SUB: k.code = K_SUB_F; break;
                case FQ_OP_MUL: k.code = K_MUL_F; break;
                case FQ_OP_DIV: k.code = K_DIV_F; break;
                case FQ_OP_MOD: k.code = K_MOD_F; break;
                default: return fqc::fail(FQ_E_INVALID, "fq_step: bad op");
            }
        } else {
            const bool u = st.dtype == FQ_DT_UINT64;
            switch (st.op) {
                case FQ_OP_ADD: k.code = K_ADD_I; break;
                case FQ_OP_SUB: k.code = K_SUB_I; break;
                case FQ_OP_MUL: k.code = K_MUL_I; break;
                case FQ_OP_DIV:
                    if (u && konst && st.bits != 0) {
                        if (is_pow2(st.bits)) {
                            k.code = K_SHR_U;
                            k.shift = (uint32_t)__builtin_ctzll(st.bits);
                        } else if (st.bits <= 65535) {
                            k.code = K_DIVM32_U;  // 32/16/16-bit long division
                            uint32_t m32 = 0;
                            u32_magic((uint32_t)st.bits, m32, k.shift, k.add);
                            k.magic = m32;
                        } else {
                            k.code = K_DIVM_U;
                            u64_magic(st.bits, k.magic, k.shift, k.add);
                        }
                    } else {
                        k.code = u ? K_DIV_U : K_DIV_S;
                    }
                    break;
                case FQ_OP_MOD:
                    if (u && konst && st.bits != 0) {
                        if (is_pow2(st.bits)) {
                            k.code = K_AND_U;
                            k.magic = st.bits - 1;
                        } else if (st.bits <= 65535) {
                            // 32-bit halves: (x>>32)%d * (2^32 % d) + (u32)x % d < 2^32
                            k.code = K_MODM32_U;
                            uint32_t m32 = 0;
                            u32_magic((uint32_t)st.bits, m32, k.shift, k.add);
                            k.magic = (uint64_t)m32 | ((((uint64_t)1 << 32) % st.bits) << 32);
                        } else {
                            k.code = K_MODM_U;
                            u64_magic(st.bits, k.magic, k.shift, k.add);
                        }
                    } else {
                        k.code = u ? K_MOD_U : K_MOD_S;
                    }
                    break;
                default: return fqc::fail(FQ_E_INVALID, "fq_step: bad op");
            }
        }
        acc = st.dtype;
    }
    if (depth != 0) return fqc::fail(FQ_E_INVALID, "fq_expr: pushed values left on the stack");
    if (e.n_steps > 0 && e.out_dtype != acc)
        return fqc::fail(FQ_E_INVALID, "fq_expr: out_dtype does not match the last step");
    res_dtype = acc;
    out.out_dtype = acc;
    return FQ_OK;
}

// fq_pred (semantic) -> KPred (lowered): predicate program cast to the
// comparison type.
fq_status lower_pred(const fq_pred *pred, int32_t col_dtype, int64_t len, bool need_data, KPred &out) {
    out = KPred{};
    out.kind = pred ? pred->kind : FQ_PRED_NONE;
    if (out.kind == FQ_PRED_EXPR) {
        int32_t ldt = col_dtype;
        fq_status s = lower_expr(pred->lhs, col_dtype, out.lhs, ldt);
        if (s != FQ_OK) return s;
        if (!is_chain_dtype(pred->cmp_dtype))
            return fqc::fail(FQ_E_UNSUPPORTED, "fused comparison type must be UInt64, Int64 or Float64");
        s = push_cast(ldt, pred->cmp_dtype, out.lhs);
        if (s != FQ_OK) return s;
        if (pred->rhs_operand == FQ_OPERAND_COLUMN && col_dtype == FQ_DT_FLOAT64 && pred->cmp_dtype != FQ_DT_FLOAT64)
            return fqc::fail(FQ_E_INVALID, "fq_pred: Float64 column compared as integer");
        out.cmp = pred->cmp;
        out.cmp_dtype = pred->cmp_dtype;
        out.rhs_operand = pred->rhs_operand;
        out.rhs = pred->rhs_bits;
    } else if (out.kind == FQ_PRED_BITMAP) {
        if (need_data && !pred->bitmap && len > 0) return fqc::fail(FQ_E_INVALID, "fq_pred: NULL bitmap");
        out.bitmap = pred->bitmap;
    } else if (out.kind == FQ_PRED_TREE) {
        const fq_pred_tree *t = pred->tree;
        if (!t) return fqc::fail(FQ_E_INVALID, "fq_pred: NULL tree");
        if (t->n_leaves < 1 || t->n_leaves > FQ_MAX_PRED_LEAVES || t->n_prog < 1 ||
            t->n_prog > 2 * FQ_MAX_PRED_LEAVES)
            return fqc::fail(FQ_E_INVALID, "fq_pred_tree: leaf / program count out of range");
        if (fqc::dtype_size(col_dtype) != 8)
            return fqc::fail(FQ_E_UNSUPPORTED, "fused predicates need a 64-bit column");
        out.n_leaves = t->n_leaves;
        out.n_prog = t->n_prog;
        for (int i = 0; i < t->n_leaves; ++i) {
            const fq_pred_leaf &lf = t->leaves[i];
            KLeaf &k = out.leaves[i];
            int32_t ldt = col_dtype;
            fq_status s = lower_expr(lf.lhs, col_dtype, k.lhs, ldt);
            if (s != FQ_OK) return s;
            if (!is_chain_dtype(lf.cmp_dtype))
                return fqc::fail(FQ_E_UNSUPPORTED, "fused comparison type must be UInt64, Int64 or Float64");
            s = push_cast(ldt, lf.cmp_dtype, k.lhs);
            if (s != FQ_OK) return s;
            if (lf.cmp < FQ_CMP_EQ || lf.cmp > FQ_CMP_GTEQ) return fqc::fail(FQ_E_INVALID, "fq_pred_leaf: bad cmp");
            if (lf.rhs_operand == FQ_OPERAND_COLUMN && col_dtype == FQ_DT_FLOAT64 && lf.cmp_dtype != FQ_DT_FLOAT64)
                return fqc::fail(FQ_E_INVALID, "fq_pred: Float64 column compared as integer");
            k.cmp = lf.cmp;
            k.cmp_dtype = lf.cmp_dtype;
            k.rhs_operand = lf.rhs_operand;
            k.rhs = lf.rhs_bits;
        }
        // validate the postfix program and tabulate it over the 2^n leaf outcomes
        uint32_t truth = 0;
        for (uint32_t combo = 0; combo < (1u << FQ_MAX_PRED_LEAVES); ++combo) {
            bool st[2 * FQ_MAX_PRED_LEAVES];
            int sp = 0;
            for (int i = 0; i < t->n_prog; ++i) {
                const int32_t tok = t->prog[i];
                out.prog[i] = tok;
                if (tok >= 0 && tok < t->n_leaves) {
                    st[sp++] = (combo >> tok) & 1u;
                } else if (tok == FQ_PRED_AND || tok == FQ_PRED_OR) {
                    if (sp < 2) return fqc::fail(FQ_E_INVALID, "fq_pred_tree: malformed program");
                    const bool b = st[--sp], a = st[--sp];
                    st[sp++] = tok == FQ_PRED_AND ? (a && b) : (a || b);
                } else {
                    return fqc::fail(FQ_E_INVALID, "fq_pred_tree: bad program token");
                }
            }
            if (sp != 1) return fqc::fail(FQ_E_INVALID, "fq_pred_tree: malformed program");
            if (st[0]) truth |= 1u << combo;
        }
        out.truth = truth;
    } else if (out.kind != FQ_PRED_NONE) {
        return fqc::fail(FQ_E_INVALID, "fq_pred: bad kind");
    }
    return FQ_OK;
}

template <typename TIn, typename V, int PRED, bool CHAIN>
static fq_status launch_scan(const Launch &L) {
    // vectors in flight per lane: 64 B for 64-bit columns, 16 elements otherwise
    constexpr int U = sizeof(TIn) >= 4 ? 4 : (sizeof(TIn) == 2 ? 2 : 1);
    if (PRED != FQ_PRED_NONE && L.block_mode) {
        hipLaunchKernelGGL((agg_block_kernel<TIn, V, PRED, CHAIN, 8>), dim3(L.grid), dim3(kThreads), 0,
                           L.stream, (const TIn *)L.col, L.n, L.block_rows, L.pred, L.val, L.mask,
                           L.vdtype, L.parts);
    } else {
        // the next tile's loads in flight while this one is reduced, for scans
        // without max/min: sum(number) 1.4132 -> 1.3991 ms per 10 GB, sum+count
        // 1.4094 -> 1.3939; with max or min it costs instead (C3 1.3800 ->
        // 1.3889, max 1.3904 -> 1.3959).  One process each, 6 rounds
        // alternating (profiles/r06_o_*_pf_ab.json); the arithmetic order is
        // the same either way.
        if (PRED == FQ_PRED_NONE && !CHAIN && !(L.mask & (FQ_AGG_MAX | FQ_AGG_MIN)))
            hipLaunchKernelGGL((agg_flat_kernel<TIn, V, PRED, CHAIN, U, true>), dim3(L.grid), dim3(kThreads), 0,
                               L.stream, (const TIn *)L.col, L.n, L.head, L.pred, L.val, L.mask, L.vdtype,
                               L.parts);
        else
            hipLaunchKernelGGL((agg_flat_kernel<TIn, V, PRED, CHAIN, U>), dim3(L.grid), dim3(kThreads), 0,
                               L.stream, (const TIn *)L.col, L.n, L.head, L.pred, L.val, L.mask, L.vdtype,
                               L.parts);
    }
    FQ_HIP_TRY(hipGetLastError());
    return FQ_OK;
}

template <typename TIn, typename V, bool CHAIN>
static fq_status dispatch_pred(const Launch &L) {
    switch (L.pred.kind) {
        case FQ_PRED_NONE: return launch_scan<TIn, V, FQ_PRED_NONE, CHAIN>(L);
        case FQ_PRED_BITMAP: return launch_scan<TIn, V, FQ_PRED_BITMAP, CHAIN>(L);
        case FQ_PRED_EXPR:
            if constexpr (sizeof(TIn) == 8) return launch_scan<TIn, V, FQ_PRED_EXPR, CHAIN>(L);
            return fqc::fail(FQ_E_UNSUPPORTED, "fused predicates need a 64-bit column");
        case FQ_PRED_TREE:
            if constexpr (sizeof(TIn) == 8) return launch_scan<TIn, V, FQ_PRED_TREE, CHAIN>(L);
            return fqc::fail(FQ_E_UNSUPPORTED, "fused predicates need a 64-bit column");
        default: return fqc::fail(FQ_E_INVALID, "fq_pred: bad kind");
    }
}

template <typename V>
static fq_status launch_finalize(const Launch &L, uint64_t blocks, int empty_if_zero, fq_agg_state *d_out) {
    // L.grid == 0: a count-only scan without predicate or expression -- the
    // reference's Count adds block.num_rows() (function_aggregator.rs:60-66),
    // no value is read, so neither is the column
    hipLaunchKernelGGL((agg_finalize_kernel<V>), dim3(1), dim3(kThreads), 0, L.stream, L.parts, L.grid,
                       blocks, L.grid == 0 ? (uint64_t)L.n : 0ull, L.vdtype, empty_if_zero, d_out);
    FQ_HIP_TRY(hipGetLastError());
    return FQ_OK;
}

static fq_status dispatch(int32_t col_dt, const Launch &L, bool chain) {
    const int32_t v = L.vdtype;
    if (!chain) {
        switch (col_dt) {
            case FQ_DT_INT8: return dispatch_pred<int8_t, int8_t, false>(L);
            case FQ_DT_INT16: return dispatch_pred<int16_t, int16_t, false>(L);
            case FQ_DT_INT32: return dispatch_pred<int32_t, int32_t, false>(L);
            case FQ_DT_INT64: return dispatch_pred<int64_t, int64_t, false>(L);
            case FQ_DT_UINT8: return dispatch_pred<uint8_t, uint8_t, false>(L);
            case FQ_DT_UINT16: return dispatch_pred<uint16_t, uint16_t, false>(L);
            case FQ_DT_UINT32: return dispatch_pred<uint32_t, uint32_t, false>(L);
            case FQ_DT_UINT64: return dispatch_pred<uint64_t, uint64_t, false>(L);
            case FQ_DT_FLOAT32: return dispatch_pred<float, float, false>(L);
            case FQ_DT_FLOAT64: return dispatch_pred<double, double, false>(L);
            default: break;
        }
    } else if (col_dt == FQ_DT_UINT64) {
        if (v == FQ_DT_UINT64) return dispatch_pred<uint64_t, uint64_t, true>(L);
        if (v == FQ_DT_INT64) return dispatch_pred<uint64_t, int64_t, true>(L);
        if (v == FQ_DT_FLOAT64) return dispatch_pred<uint64_t, double, true>(L);
    } else if (col_dt == FQ_DT_INT64) {
        if (v == FQ_DT_INT64) return dispatch_pred<int64_t, int64_t, true>(L);
        if (v == FQ_DT_FLOAT64) return dispatch_pred<int64_t, double, true>(L);
    } else if (col_dt == FQ_DT_FLOAT64) {
        if (v == FQ_DT_FLOAT64) return dispatch_pred<double, double, true>(L);
    }
    return fqc::fail(FQ_E_UNSUPPORTED, std::string("aggregate over ") + fqc::dtype_name(col_dt) +
                                           " column with " + fqc::dtype_name(v) +
                                           " value is not supported on the device path");
}

static fq_status dispatch_finalize(const Launch &L, uint64_t blocks, int empty_if_zero, fq_agg_state *d_out) {
    switch (L.vdtype) {
        case FQ_DT_INT8: return launch_finalize<int8_t>(L, blocks, empty_if_zero, d_out);
        case FQ_DT_INT16: return launch_finalize<int16_t>(L, blocks, empty_if_zero, d_out);
        case FQ_DT_INT32: return launch_finalize<int32_t>(L, blocks, empty_if_zero, d_out);
        case FQ_DT_INT64: return launch_finalize<int64_t>(L, blocks, empty_if_zero, d_out);
        case FQ_DT_UINT8: return launch_finalize<uint8_t>(L, blocks, empty_if_zero, d_out);
        case FQ_DT_UINT16: return launch_finalize<uint16_t>(L, blocks, empty_if_zero, d_out);
        case FQ_DT_UINT32: return launch_finalize<uint32_t>(L, blocks, empty_if_zero, d_out);
        case FQ_DT_UINT64: return launch_finalize<uint64_t>(L, blocks, empty_if_zero, d_out);
        case FQ_DT_FLOAT32: return launch_finalize<float>(L, blocks, empty_if_zero, d_out);
        case FQ_DT_FLOAT64: return launch_finalize<double>(L, blocks, empty_if_zero, d_out);
        default: return fqc::fail(FQ_E_INVALID, "finalize: bad dtype");
    }
}

}  // namespace fqk

extern "C" {

size_t fq_aggregate_workspace_bytes(int64_t len) {
    (void)len;
    return fqk::kPartialsBytes;
}

}  // extern "C"

namespace fqk {

// Validates the arguments and prepares the launch shared by fq_aggregate and
// fq_jit_prepare (lowered programs, flat/block mode, grid).
static fq_status plan_scan(const fq_col *col, int64_t block_rows, const fq_pred *pred, const fq_expr *value,
                           uint32_t agg_mask, bool need_data, Launch &L, bool &chain, uint64_t &blocks,
                           int &empty_if_zero) {
    if (!col) return fqc::fail(FQ_E_INVALID, "fq_aggregate: NULL argument");
    if (col->len < 0) return fqc::fail(FQ_E_INVALID, "fq_aggregate: negative length");
    const int esize = fqc::dtype_size(col->dtype);
    if (!fqc::dtype_is_numeric(col->dtype))
        return fqc::internal(std::string("Unsupported data_array_aggregate for data type: ") +
                             fqc::dtype_name(col->dtype));
    if (need_data && col->len > 0 && !col->data) return fqc::fail(FQ_E_INVALID, "fq_aggregate: NULL column data");
    if (((uintptr_t)col->data) % esize)
        return fqc::fail(FQ_E_INVALID, "fq_aggregate: column not aligned to its element size");
    if (block_rows <= 0) block_rows = col->len > 0 ? col->len : 1;

    L = Launch{};
    L.col = col->data;
    L.n = col->len;
    L.block_rows = block_rows;
    L.mask = agg_mask;

    // value expression
    chain = value && value->n_steps > 0;
    int32_t vdt = col->dtype;
    if (chain) {
        fq_status s = lower_expr(*value, col->dtype, L.val, vdt);
        if (s != FQ_OK) return s;
    }
    L.vdtype = vdt;

    // predicate
    fq_status ps = lower_pred(pred, col->dtype, col->len, need_data, L.pred);
    if (ps != FQ_OK) return ps;

    blocks = col->len == 0 ? 0 : (uint64_t)((col->len + block_rows - 1) / block_rows);
    // Block mode only where the per-block emptiness matters (filtered sum over
    // more than one reference block); otherwise stream flat.
    L.block_mode = L.pred.kind != FQ_PRED_NONE && (agg_mask & FQ_AGG_SUM) && blocks > 1;
    empty_if_zero = (L.pred.kind != FQ_PRED_NONE && blocks == 1) ? 1 : 0;

    const int cus = fqc::device_cu_count();
    const int max_grid = cus * 8 < kMaxPartials ? cus * 8 : kMaxPartials;
    if (L.block_mode) {
        const int64_t waves_needed = (int64_t)blocks;
        int64_t grid = (waves_needed + (kThreads / kWave) - 1) / (kThreads / kWave);
        L.grid = (int)(grid < max_grid ? (grid < 1 ? 1 : grid) : max_grid);
        L.head = 0;
    } else {
        const int64_t vec_elems = 16 / esize;
        const uintptr_t mis = ((uintptr_t)col->data) & 15u;
        int64_t head = mis ? (int64_t)((16 - mis) / esize) : 0;
        if (head > col->len) head = col->len;
        L.head = head;
        const int64_t nvec = (col->len - head) / vec_elems;
        const int64_t tile = (int64_t)kThreads * (esize >= 4 ? 4 : (esize == 2 ? 2 : 1));
        int64_t grid = (nvec + tile - 1) / tile;
        if (grid < 1) grid = 1;
        // 2 workgroups (8 waves) per CU streamed fastest (tools/tune_scan.py)
        const int64_t flat_max = (int64_t)cus * scan_wg_per_cu();
        L.grid = (int)(grid < flat_max ? grid : flat_max);
    }
    return FQ_OK;
}

// fq_aggregate: the scan, then the fold of its partials, both on `stream`
static fq_status aggregate(const fq_col *col, int64_t block_rows, const fq_pred *pred, const fq_expr *value,
                           uint32_t agg_mask, fq_agg_state *d_out, void *d_ws, size_t ws_bytes, hipStream_t stream) {
    if (!col || !d_out || !d_ws) return fqc::fail(FQ_E_INVALID, "fq_aggregate: NULL argument");
    if (ws_bytes < kPartialsBytes) return fqc::fail(FQ_E_INVALID, "fq_aggregate: workspace too small");
    if (agg_mask & ~(uint32_t)(FQ_AGG_MIN | FQ_AGG_MAX | FQ_AGG_SUM | FQ_AGG_COUNT))
        return fqc::fail(FQ_E_INVALID, "fq_aggregate: unknown bits in agg_mask");
    Launch L;
    bool chain = false;
    uint64_t blocks = 0;
    int empty_if_zero = 0;
    fq_status s = plan_scan(col, block_rows, pred, value, agg_mask, true, L, chain, blocks, empty_if_zero);
    if (s != FQ_OK) return s;
    L.stream = (hipStream_t)stream;
    L.parts = (Partial *)d_ws;
    if (agg_mask == FQ_AGG_COUNT && !chain && L.pred.kind == FQ_PRED_NONE) {
        L.grid = 0;  // count(column): rows, not values (see launch_finalize)
        return dispatch_finalize(L, blocks, empty_if_zero, d_out);
    }
    bool jitted = false;
    const bool tree = (chain && prog_has_tree(L.val)) || pred_has_tree(L.pred);
    s = jit_scan(col->dtype, chain, L, &jitted, tree);
    if (s != FQ_OK) return s;
    if (!jitted && tree)
        return fqc::fail(FQ_E_UNSUPPORTED, "fused expression trees run on the hipRTC kernels only (FQ_JIT is off "
                                           "or hipRTC is unavailable)");
    if (!jitted) {
        if (chain || L.pred.kind != FQ_PRED_NONE) jit_count_interp();
        s = dispatch(col->dtype, L, chain);
        if (s != FQ_OK) return s;
    }
    return dispatch_finalize(L, blocks, empty_if_zero, d_out);
}

}  // namespace fqk

extern "C" {

fq_status fq_aggregate(const fq_col *col, int64_t block_rows, const fq_pred *pred, const fq_expr *value,
                       uint32_t agg_mask, fq_agg_state *d_out, void *d_ws, size_t ws_bytes, void *stream) {
    return fqk::aggregate(col, block_rows, pred, value, agg_mask, d_out, d_ws, ws_bytes, (hipStream_t)stream);
}

fq_status fq_jit_prepare(const fq_col *col, int64_t block_rows, const fq_pred *pred, const fq_expr *value,
                         uint32_t agg_mask, int32_t *specialised) {
    using namespace fqk;
    if (specialised) *specialised = 0;
    Launch L;
    bool chain = false;
    uint64_t blocks = 0;
    int empty_if_zero = 0;
    fq_status s = plan_scan(col, block_rows, pred, value, agg_mask, false, L, chain, blocks, empty_if_zero);
    if (s != FQ_OK) return s;
    bool ok = false;
    s = jit_prepare(col->dtype, chain, L, &ok);
    if (s == FQ_OK && specialised) *specialised = ok ? 1 : 0;
    return s;
}

}  // extern "C"
