// GROUP BY hash aggregation (include/fq_gpu.h fq_group_*).
//
// No reference counterpart: fuse-query plans group_expr (plan_parser.rs:
// 284-308, plan_aggregate.rs:12) but PipelineBuilder (pipeline_builder.rs:
// 50-66) builds AggregatePartial/Final from aggr_expr only.  The semantics
// here are the ungrouped path's (fq_aggregate) applied per key.
//
// Table layout in the caller's device memory (all 64-bit words):
//   [0, 64)                     header: u32 flags (state flags | 256 = full),
//                               u32 sentinel-used, u64 scratch counter,
//                               u32 groups claimed, u32 "an LDS table saturated"
//   keys[capacity + 1]          0xFFFF...FF = empty; slot `capacity` holds the
//                               key 0xFFFF...FF itself when it occurs
//   states[a][r][capacity + 1]  per aggregate a and replica r < R (see
//                               group_replicas: workgroup b updates replica
//                               b % R), initialised to the identity of its
//                               kind (0, +max, lowest) so atomics need no
//                               occupancy check; extract folds the replicas
// The accumulate kernel is generated per shape with hipRTC (fq_jit.hip
// gen_groupby_source); init / count / extract are precompiled here.
#include <hip/hip_runtime.h>

#include <string>

#include "fq_common.h"
#include "fq_device.h"
#include "fq_scan.h"

namespace fqk {

constexpr uint64_t kEmpty = ~0ull;
constexpr uint32_t kFull = 256u;
constexpr uint32_t kPartOverflow = 512u;  // fq_jit_gpart: more blocks than the workspace bound (never expected)
constexpr uint32_t kNarrowOverflow = 1024u;  // fq_jit_gpart: a value outside col[0] +- 2^31 (FQ_GROUP_NARROW_ROWS)
constexpr size_t kHdrBytes = 64;

struct TableView {
    uint32_t *hdr;
    uint64_t *counter;
    uint64_t *keys;
    uint64_t *states[FQ_MAX_GROUP_AGGS];  // replica 0; replica r at + r * (cap + 1)
    int64_t cap;
    int replicas;
};

static uint64_t identity_bits(int32_t kind, int32_t dt) {
    if (kind == FQ_AGG_COUNT || kind == FQ_AGG_SUM) return 0;
    if (dt == FQ_DT_UINT64) return kind == FQ_AGG_MAX ? 0ull : ~0ull;
    if (dt == FQ_DT_INT64) return kind == FQ_AGG_MAX ? 0x8000000000000000ull : 0x7fffffffffffffffull;
    return kind == FQ_AGG_MAX ? 0xfff0000000000000ull : 0x7ff0000000000000ull;  // -inf / +inf
}

static fq_status view(const fq_group_table *t, TableView &v) {
    if (!t || !t->d_mem) return fqc::fail(FQ_E_INVALID, "fq_group_table: NULL table");
    if (t->capacity < 64 || (t->capacity & (t->capacity - 1)))
        return fqc::fail(FQ_E_INVALID, "fq_group_table: capacity must be a power of two >= 64");
    if (t->n_aggs < 1 || t->n_aggs > FQ_MAX_GROUP_AGGS)
        return fqc::fail(FQ_E_INVALID, "fq_group_table: n_aggs out of range");
    if (t->key_dtype != FQ_DT_UINT64 && t->key_dtype != FQ_DT_INT64)
        return fqc::fail(FQ_E_UNSUPPORTED, "GROUP BY keys must be UInt64 or Int64");
    for (int a = 0; a < t->n_aggs; ++a) {
        const int32_t k = t->kinds[a], d = t->dtypes[a];
        if (k != FQ_AGG_COUNT && k != FQ_AGG_SUM && k != FQ_AGG_MIN && k != FQ_AGG_MAX)
            return fqc::fail(FQ_E_INVALID, "fq_group_table: bad aggregate kind");
        if (k == FQ_AGG_COUNT ? d != FQ_DT_UINT64 : (d != FQ_DT_UINT64 && d != FQ_DT_INT64 && d != FQ_DT_FLOAT64))
            return fqc::fail(FQ_E_UNSUPPORTED, "GROUP BY states must be 64-bit (Count: UInt64)");
    }
    char *m = (char *)t->d_mem;
    v.hdr = (uint32_t *)m;
    v.counter = (uint64_t *)(m + 8);
    v.keys = (uint64_t *)(m + kHdrBytes);
    v.cap = t->capacity;
    v.replicas = group_replicas(t->capacity);
    for (int a = 0; a < FQ_MAX_GROUP_AGGS; ++a)
        v.states[a] = a < t->n_aggs ? v.keys + (size_t)(1 + a * v.replicas) * (size_t)(t->capacity + 1) : nullptr;
    return FQ_OK;
}

struct InitArgs {
    uint64_t *keys;
    uint64_t *states[FQ_MAX_GROUP_AGGS];
    uint64_t ident[FQ_MAX_GROUP_AGGS];
    int32_t n_aggs;
    int64_t slots;     // capacity + 1
    int32_t replicas;
};

__global__ void __launch_bounds__(256) group_init_kernel(InitArgs a) {
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    const int64_t all = a.slots * a.replicas;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < all; i += T) {
        if (i < a.slots) a.keys[i] = kEmpty;
        for (int s = 0; s < a.n_aggs; ++s) a.states[s][i] = a.ident[s];
    }
}

// fold of two states of one aggregate (the atomics' operation)
__device__ __forceinline__ uint64_t fold(int32_t kind, int32_t dt, uint64_t x, uint64_t y) {
    if (kind == FQ_AGG_COUNT) return x + y;
    if (dt == FQ_DT_FLOAT64) {
        const double a = __builtin_bit_cast(double, x), b = __builtin_bit_cast(double, y);
        if (kind == FQ_AGG_SUM) return __builtin_bit_cast(uint64_t, a + b);
        if (kind == FQ_AGG_MAX) return b > a ? y : x;
        return b < a ? y : x;
    }
    if (kind == FQ_AGG_SUM) return x + y;
    if (dt == FQ_DT_INT64) {
        const int64_t a = (int64_t)x, b = (int64_t)y;
        if (kind == FQ_AGG_MAX) return b > a ? y : x;
        return b < a ? y : x;
    }
    if (kind == FQ_AGG_MAX) return y > x ? y : x;
    return y < x ? y : x;
}

// counts occupied slots into *counter (wave-aggregated atomics)
__global__ void __launch_bounds__(256)
    group_count_kernel(const uint64_t *__restrict__ keys, int64_t cap, const uint32_t *hdr, uint64_t *counter) {
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    uint64_t c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += T) c += keys[i] != kEmpty;
    if (blockIdx.x == 0 && threadIdx.x == 0 && hdr[1]) c += 1;
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) c += shfl_xor64(c, off);
    if ((threadIdx.x & (kWave - 1)) == 0 && c) atomicAdd((unsigned long long *)counter, (unsigned long long)c);
}

struct ExtractArgs {
    const uint64_t *keys;
    const uint64_t *states[FQ_MAX_GROUP_AGGS];
    uint64_t *out_keys;
    uint64_t *out_states[FQ_MAX_GROUP_AGGS];
    int32_t n_aggs;
    int32_t kinds[FQ_MAX_GROUP_AGGS];
    int32_t dtypes[FQ_MAX_GROUP_AGGS];
    int32_t replicas;
    int64_t cap;
    int64_t out_cap;
    const uint32_t *hdr;
    uint64_t *counter;
};

__global__ void __launch_bounds__(256) group_extract_kernel(ExtractArgs a) {
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    const int lane = threadIdx.x & (kWave - 1);
    // slot `cap` is the sentinel key's slot: scanned iff it was used
    const int64_t slots = a.cap + 1;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < slots; base += T) {
        const int64_t i = base + threadIdx.x;
        bool occ = false;
        if (i < a.cap) occ = a.keys[i] != kEmpty;
        else if (i == a.cap) occ = a.hdr[1] != 0;
        const uint64_t m = __ballot(occ);
        if (m == 0) continue;
        uint64_t first = 0;
        if (lane == 0) first = atomicAdd((unsigned long long *)a.counter, (unsigned long long)__popcll(m));
        first = __shfl((unsigned long long)first, 0, kWave);
        if (!occ) continue;
        const uint64_t pos = first + (uint64_t)__popcll(m & ((1ull << lane) - 1ull));
        if ((int64_t)pos >= a.out_cap) continue;
        a.out_keys[pos] = i < a.cap ? a.keys[i] : kEmpty;
        for (int s = 0; s < a.n_aggs; ++s) {
            uint64_t v = a.states[s][i];
            for (int r = 1; r < a.replicas; ++r)
                v = fold(a.kinds[s], a.dtypes[s], v, a.states[s][(int64_t)r * slots + i]);
            a.out_states[s][pos] = v;
        }
    }
}

// fq_group_table_merge: exchanged rows into a table (replica 0 of each
// state; extract folds the replicas).  A key's home slot is its 64-bit mixer
// mod the capacity, linear probing, claimed with a CAS (keys only go EMPTY ->
// key); the sentinel key has its own slot (cap) and header flag, as in the
// generated kernels' ginsert.
struct MergeArgs {
    const uint64_t *in_keys;
    const uint64_t *in_states[FQ_MAX_GROUP_AGGS];
    uint64_t *keys;
    uint64_t *states[FQ_MAX_GROUP_AGGS];
    int32_t kinds[FQ_MAX_GROUP_AGGS];
    int32_t dtypes[FQ_MAX_GROUP_AGGS];
    int32_t n_aggs;
    int64_t n, cap;
    uint32_t *hdr;
};

__device__ __forceinline__ uint64_t merge_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ void atomic_fold(int32_t kind, int32_t dt, uint64_t *p, uint64_t v) {
    if (kind == FQ_AGG_COUNT || (kind == FQ_AGG_SUM && dt != FQ_DT_FLOAT64)) {
        atomicAdd((unsigned long long *)p, (unsigned long long)v);
        return;
    }
    uint64_t old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
        const uint64_t nv = fold(kind, dt, old, v);
        if (nv == old) return;
        const uint64_t prev = atomicCAS((unsigned long long *)p, old, nv);
        if (prev == old) return;
        old = prev;
    }
}

__global__ void __launch_bounds__(256) group_merge_kernel(MergeArgs a) {
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    const uint64_t mask = (uint64_t)a.cap - 1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += T) {
        const uint64_t k = a.in_keys[i];
        int64_t slot = -1;
        if (k == kEmpty) {
            atomicOr(&a.hdr[1], 1u);
            slot = a.cap;
        } else {
            // the home slot ginsert (fq_jit.hip) uses -- the top log2(cap) bits of
            // the mixer -- so merged rows meet the keys aggregated into the same table
            uint64_t h = mask ? merge_mix(k) >> __clzll(mask) : 0;
            for (int64_t p = 0; p < a.cap; ++p) {
                const uint64_t cur = __hip_atomic_load(&a.keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (cur == k) {
                    slot = (int64_t)h;
                    break;
                }
                if (cur == kEmpty) {
                    const uint64_t old = atomicCAS((unsigned long long *)&a.keys[h], kEmpty, k);
                    if (old == kEmpty || old == k) {
                        slot = (int64_t)h;
                        break;
                    }
                }
                h = (h + 1) & mask;
            }
        }
        if (slot < 0) {
            atomicOr(&a.hdr[0], 256u);  // table full (read_header reports FQ_E_TABLE_FULL)
            continue;
        }
        for (int s = 0; s < a.n_aggs; ++s) atomic_fold(a.kinds[s], a.dtypes[s], &a.states[s][slot], a.in_states[s][i]);
    }
}

static int small_grid(int64_t work) {
    const int64_t cap = (int64_t)fqc::device_cu_count() * 4;
    int64_t g = (work + 255) / 256;
    if (g < 1) g = 1;
    return (int)(g < cap ? g : cap);
}

static fq_status read_header(const TableView &v, uint32_t &flags, uint64_t &count, hipStream_t st) {
    uint64_t h[2] = {0, 0};
    FQ_HIP_TRY(hipMemcpyAsync(h, v.hdr, 16, hipMemcpyDeviceToHost, st));
    FQ_HIP_TRY(hipStreamSynchronize(st));
    flags = (uint32_t)(h[0] & 0xffffffffu);
    count = h[1];
    if (flags & kFull) return fqc::fail(FQ_E_TABLE_FULL, "GROUP BY hash table is full");
    if (flags & kPartOverflow) return fqc::fail(FQ_E_INTERNAL, "GROUP BY partition workspace overflow");
    if (flags & kNarrowOverflow)
        return fqc::fail(FQ_E_INVALID, "GROUP BY narrow rows: a value outside col[0] +- 2^31 (FQ_GROUP_NARROW_ROWS)");
    if (flags & FQ_STATE_DIV_ZERO) return fqc::fail(FQ_E_DIVIDE_BY_ZERO, "Internal Error: Divide by zero error");
    if (flags & FQ_STATE_CAST_NULL)
        return fqc::fail(FQ_E_UNSUPPORTED, "cast produced nulls (nulls are not supported on the device path)");
    return FQ_OK;
}

// The blocks of fq_jit_gpart grouped by bin, for fq_jit_groupby_bins: one
// 256-thread workgroup scans the P <= 256 per-bin block counts into the bin
// starts, then a scatter over the workgroup regions' blocks (used[w] of each
// region's q, read on the device) places each block number -- with its rows,
// order[i] = block | rows << 32 -- at its bin's cursor.  The scatter ranks in
// LDS first: one global atomic per (workgroup, bin).  Block order within a
// bin is arbitrary.
constexpr int kBlkThreads = 256;
constexpr int kBlkPerThread = 4;

__global__ void __launch_bounds__(kBlkThreads)
    group_blk_scan_kernel(const uint32_t *__restrict__ bin_blocks, uint32_t *__restrict__ bstart,
                          uint32_t *__restrict__ cursor, int P) {
    __shared__ uint32_t s[kBlkThreads];
    const int t = threadIdx.x;
    const uint32_t v = t < P ? bin_blocks[t] : 0u;
    s[t] = v;
    __syncthreads();
    for (int o = 1; o < kBlkThreads; o <<= 1) {
        const uint32_t y = t >= o ? s[t - o] : 0u;
        __syncthreads();
        s[t] += y;
        __syncthreads();
    }
    if (t < P) {
        bstart[t] = s[t] - v;
        cursor[t] = s[t] - v;
    }
    if (t == P - 1) bstart[P] = s[t];
}

__global__ void __launch_bounds__(kBlkThreads)
    group_blk_scatter_kernel(const uint32_t *__restrict__ used, const uint32_t *__restrict__ blk_bin,
                             const uint32_t *__restrict__ blk_fill, uint32_t *__restrict__ cursor,
                             uint64_t *__restrict__ order, uint32_t q, uint32_t slots, uint32_t P) {
    __shared__ uint32_t s_cnt[256], s_base[256];
    const uint32_t first = blockIdx.x * (uint32_t)(kBlkThreads * kBlkPerThread);
    s_cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t bin[kBlkPerThread], rank[kBlkPerThread];
    bool ok[kBlkPerThread];
#pragma unroll
    for (int k = 0; k < kBlkPerThread; ++k) {
        const uint32_t i = first + k * kBlkThreads + threadIdx.x;
        ok[k] = i < slots && i - (i / q) * q < used[i / q];
        bin[k] = ok[k] ? blk_bin[i] : 0u;
        ok[k] = ok[k] && bin[k] < P;  // never index s_cnt with a block the partition kernel did not write
        if (!ok[k]) bin[k] = 0u;
        rank[k] = ok[k] ? atomicAdd(&s_cnt[bin[k]], 1u) : 0u;
    }
    __syncthreads();
    const uint32_t c = s_cnt[threadIdx.x];
    if (c) s_base[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], c);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kBlkPerThread; ++k) {
        const uint32_t i = first + k * kBlkThreads + threadIdx.x;
        if (ok[k]) order[s_base[bin[k]] + rank[k]] = (uint64_t)i | ((uint64_t)blk_fill[i] << 32);
    }
}

fq_status launch_group_part_blocks(const GroupPartition &X, hipStream_t stream) {
    const int P = 1 << (X.log2p & 255);  // (bits 8..15: the range-bin shift)
    hipLaunchKernelGGL(group_blk_scan_kernel, dim3(1), dim3(kBlkThreads), 0, stream, X.bin_blocks, X.bstart,
                       X.cursor, P);
    FQ_HIP_TRY(hipGetLastError());
    const uint32_t per = kBlkThreads * kBlkPerThread, slots = (uint32_t)X.grid * X.q;
    const uint32_t grid = (slots + per - 1) / per;
    hipLaunchKernelGGL(group_blk_scatter_kernel, dim3(grid > 0 ? grid : 1), dim3(kBlkThreads), 0, stream, X.used,
                       X.blk_bin, X.blk_fill, X.cursor, X.order, X.q, slots, (uint32_t)P);
    FQ_HIP_TRY(hipGetLastError());
    return FQ_OK;
}

// Workgroups of fq_jit_gpart for len rows: two 1,024-thread workgroups per CU
// (its 77 KB of LDS; FQ_TUNE_GPART_WG_PER_CU tunes it), at most one per 8-row tile
// of 256 threads -- the bound the workspace is sized by (FQ_TUNE_GPART_WG_PER_CU)
static int part_wg_per_cu() { return (int)fqc::knob(FQ_TUNE_GPART_WG_PER_CU); }
static int group_threads() { return (int)fqc::knob(FQ_TUNE_GROUP_THREADS); }
// (at least 4 tiles per workgroup: every workgroup's region holds a partial
// block per bin, P x 2 KB, which for a small column would outweigh its rows)
static int64_t part_grid_bound(int64_t len) {
    int64_t g = (int64_t)fqc::device_cu_count() * part_wg_per_cu();
    if (g > kMaxPartGrid) g = kMaxPartGrid;
    const int64_t tile = (int64_t)group_threads() * 8, tiles = (len + tile - 1) / tile;
    if (g > (tiles + 3) / 4) g = (tiles + 3) / 4;
    return g < 1 ? 1 : g;
}

// Region of one fq_jit_gpart workgroup: the blocks of its tiles' rows (grid-
// stride tiles of tile_rows), every (workgroup, bin) chain being full blocks
// but its last
static uint32_t part_region_blocks(int64_t len, int64_t tile_rows, int grid, int P) {
    const int64_t tiles = (len + tile_rows - 1) / tile_rows, per = (tiles + grid - 1) / grid;
    return (uint32_t)((per * tile_rows + kPartBlockRows - 1) / kPartBlockRows + P);
}

// Workspace of fq_group_aggregate_partitioned:
// [head: used u32 x kMaxPartGrid, blocks per bin u32 x 256][bstart u32 x 257, cursor u32 x 256]
// [blk_bin u32 x B][blk_fill u32 x B][order u64 x B][vals: B blocks of kPartBlockRows rows]
// with B blocks bounding grid x part_region_blocks for any grid <= the bound
// g and tiles <= 8,192 rows (1,024 threads x 8): ceil(len / kPartBlockRows)
// + (g + 1) x 8,192 / kPartBlockRows + g x (P + 1) + 1
static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
static size_t part_ws_bytes(int64_t len, int log2p, GroupPartition *X, void *ws) {
    const size_t P = (size_t)1 << log2p, n = (size_t)(len > 0 ? len : 0);
    const size_t g = (size_t)part_grid_bound(len);
    const size_t B = (n + kPartBlockRows - 1) / kPartBlockRows + (g + 1) * (8192 / kPartBlockRows) + g * (P + 1) + 1;
    const size_t head = align256((kMaxPartGrid + 256) * 4), sc = align256((257 + 256) * 4);
    const size_t bb = align256(B * 4), ord = align256(B * 8), vals = align256(B * kPartBlockRows * 8);
    if (X) {
        char *m = (char *)ws;
        X->head = (uint32_t *)m;
        X->head_bytes = head;
        X->used = X->head;
        X->bin_blocks = X->head + kMaxPartGrid;
        X->bstart = (uint32_t *)(m + head);
        X->cursor = X->bstart + 257;
        X->blk_bin = (uint32_t *)(m + head + sc);
        X->blk_fill = (uint32_t *)(m + head + sc + bb);
        X->order = (uint64_t *)(m + head + sc + 2 * bb);
        X->vals = m + head + sc + 2 * bb + ord;
        X->max_blocks = (uint32_t)B;
    }
    return head + sc + 2 * bb + ord + vals;
}

// LDS table budget of the GROUP BY launch (FQ_TUNE_GROUP_LDS_KB; tools/groupby_sweep.py)
static int group_lds_bytes() { return (int)fqc::knob(FQ_TUNE_GROUP_LDS_KB) * 1024; }

// validation + lowering shared by both aggregate entry points
static fq_status prepare_group(const fq_group_table *t, const fq_col *col, const fq_pred *pred,
                               const fq_expr *key_expr, const fq_expr *values, void *stream, GroupLaunch &G) {
    TableView v;
    fq_status s = view(t, v);
    if (s != FQ_OK) return s;
    if (!col) return fqc::fail(FQ_E_INVALID, "fq_group_aggregate: NULL column");
    if (col->len < 0) return fqc::fail(FQ_E_INVALID, "fq_group_aggregate: negative length");
    if (col->len > 0 && !col->data) return fqc::fail(FQ_E_INVALID, "fq_group_aggregate: NULL column data");
    if (fqc::dtype_size(col->dtype) != 8 || !fqc::dtype_is_numeric(col->dtype))
        return fqc::fail(FQ_E_UNSUPPORTED, "GROUP BY needs a 64-bit column on the device path");
    if ((uintptr_t)col->data & 7u) return fqc::fail(FQ_E_INVALID, "fq_group_aggregate: misaligned column");
    G = GroupLaunch{};
    G.col = col->data;
    G.n = col->len;
    s = lower_pred(pred, col->dtype, col->len, true, G.pred);
    if (s != FQ_OK) return s;
    int32_t kdt = col->dtype;
    if (key_expr && key_expr->n_steps > 0) {
        s = lower_expr(*key_expr, col->dtype, G.key, kdt);
        if (s != FQ_OK) return s;
    }
    if (kdt != t->key_dtype)
        return fqc::fail(FQ_E_INVALID, std::string("fq_group_aggregate: key expression is ") + fqc::dtype_name(kdt) +
                                           ", table key is " + fqc::dtype_name(t->key_dtype));
    G.key_dtype = kdt;
    G.n_aggs = t->n_aggs;
    for (int a = 0; a < t->n_aggs; ++a) {
        G.kinds[a] = t->kinds[a];
        G.dtypes[a] = t->dtypes[a];
        if (t->kinds[a] == FQ_AGG_COUNT) continue;
        int32_t vdt = col->dtype;
        if (values && values[a].n_steps > 0) {
            s = lower_expr(values[a], col->dtype, G.vals[a], vdt);
            if (s != FQ_OK) return s;
            G.chain[a] = true;
        }
        if (vdt != t->dtypes[a])
            return fqc::fail(FQ_E_INVALID, "fq_group_aggregate: argument dtype does not match the table state");
    }
    for (int a = 0; a < FQ_MAX_GROUP_AGGS; ++a) G.states[a] = v.states[a];
    G.keys = v.keys;
    G.hdr = v.hdr;
    G.capacity = t->capacity;
    G.stream = (hipStream_t)stream;
    const uintptr_t mis = ((uintptr_t)col->data) & 15u;
    G.head = mis ? 1 : 0;
    if (G.head > G.n) G.head = G.n;
    // one 1,024-thread workgroup per CU with a 128 KB LDS table: 16 waves
    // share one table (tools/groupby_sweep.py: 256-thread workgroups with a
    // 64 KB table each, 2 per CU, ran 1,000 groups x 3 aggregates in 2.98 ms
    // against 2.25 ms here, and the table holds twice the groups)
    G.lds_bytes = group_lds_bytes();
    G.threads = group_threads();
    G.rowmap = 1;  // lane-consecutive rows (row pairs per lane measured 1.6x slower)
    const int64_t nvec = (G.n - G.head) / 2;
    int64_t grid = (nvec + 4 * G.threads - 1) / (4 * G.threads);
    if (grid < 1) grid = 1;
    const int64_t cap = (int64_t)fqc::device_cu_count() * fqc::knob(FQ_TUNE_GROUP_WG_PER_CU);
    G.grid = (int)(grid < cap ? grid : cap);
    return FQ_OK;
}

}  // namespace fqk

extern "C" {

size_t fq_group_table_bytes(int64_t capacity, int32_t n_aggs) {
    if (capacity < 0 || n_aggs < 0) return 0;
    return fqk::kHdrBytes + (size_t)(capacity + 1) * 8u * (size_t)(1 + n_aggs * fqk::group_replicas(capacity));
}

fq_status fq_group_table_init(const fq_group_table *t, void *stream) {
    using namespace fqk;
    TableView v;
    fq_status s = view(t, v);
    if (s != FQ_OK) return s;
    hipStream_t st = (hipStream_t)stream;
    FQ_HIP_TRY(hipMemsetAsync(v.hdr, 0, kHdrBytes, st));
    InitArgs a{};
    a.keys = v.keys;
    a.n_aggs = t->n_aggs;
    a.slots = t->capacity + 1;
    a.replicas = v.replicas;
    for (int i = 0; i < t->n_aggs; ++i) {
        a.states[i] = v.states[i];
        a.ident[i] = identity_bits(t->kinds[i], t->dtypes[i]);
    }
    hipLaunchKernelGGL(group_init_kernel, dim3(small_grid(a.slots * a.replicas)), dim3(256), 0, st, a);
    FQ_HIP_TRY(hipGetLastError());
    return FQ_OK;
}

fq_status fq_group_aggregate(const fq_group_table *t, const fq_col *col, const fq_pred *pred,
                             const fq_expr *key_expr, const fq_expr *values, void *stream) {
    using namespace fqk;
    GroupLaunch G;
    fq_status s = prepare_group(t, col, pred, key_expr, values, stream, G);
    if (s != FQ_OK) return s;
    return jit_groupby(col->dtype, G);
}

int64_t fq_group_dense_keys(int32_t col_dtype, const fq_expr *key_expr, int32_t n_aggs) {
    using namespace fqk;
    if (!key_expr || key_expr->n_steps < 1 || n_aggs < 1 || n_aggs > FQ_MAX_GROUP_AGGS) return 0;
    KProg k;
    int32_t kdt = col_dtype;
    if (lower_expr(*key_expr, col_dtype, k, kdt) != FQ_OK) return 0;
    return group_dense_bound(k, kdt, n_aggs, group_lds_bytes());
}

size_t fq_group_partition_workspace_bytes(int64_t len, int32_t log2_parts) {
    log2_parts &= ~FQ_GROUP_NARROW_ROWS;
    if (log2_parts < 1 || log2_parts > 8) return 0;
    return fqk::part_ws_bytes(len, log2_parts, nullptr, nullptr);
}

fq_status fq_group_aggregate_partitioned(const fq_group_table *t, const fq_col *col, const fq_pred *pred,
                                         const fq_expr *key_expr, const fq_expr *values, int32_t log2_parts,
                                         void *d_ws, size_t ws_bytes, void *stream) {
    using namespace fqk;
    const bool narrow = (log2_parts & FQ_GROUP_NARROW_ROWS) != 0;
    log2_parts &= ~FQ_GROUP_NARROW_ROWS;
    if (log2_parts < 1 || log2_parts > 8)
        return fqc::fail(FQ_E_INVALID, "fq_group_aggregate_partitioned: log2_parts must be in [1, 8]");
    GroupLaunch G;
    fq_status s = prepare_group(t, col, pred, key_expr, values, stream, G);
    if (s != FQ_OK) return s;
    // 4-byte rows for 8-byte integer columns the caller vouches for
    G.narrow = narrow && fqc::knob(FQ_TUNE_GROUP_NARROW) && (col->dtype == FQ_DT_UINT64 || col->dtype == FQ_DT_INT64) ? 1 : 0;
    if (G.n > 0 && (!d_ws || ws_bytes < part_ws_bytes(G.n, log2_parts, nullptr, nullptr)))
        return fqc::fail(FQ_E_INVALID, "fq_group_aggregate_partitioned: workspace too small");
    if (((uintptr_t)d_ws) & 255u) return fqc::fail(FQ_E_INVALID, "fq_group_aggregate_partitioned: workspace not 256-B aligned");
    GroupPartition X{};
    X.log2p = log2_parts;
    // Keys known to lie in [0, d) (`% d`, `& (d - 1)`) are binned by range
    // when d fits the 2^log2_parts bins with at most S keys each: bin = key >>
    // shift, and each bin's LDS table is indexed by the key's low bits (no
    // hash, no probe, no claim).  The kernels get log2p | shift << 8.
    // profiles/r02_groupby_range_bins.txt
    int lp_arg = log2_parts;
    bool fitted = false;
    const int64_t d = group_key_range(G.key, G.key_dtype);
    const int64_t S = group_lds_slots(G.n_aggs, G.lds_bytes);
    if (d > 0 && fqc::knob(FQ_TUNE_GROUP_RANGE_BINS)) {
        int sh = 0;
        while (((int64_t)1 << log2_parts << sh) < d) ++sh;
        if (((int64_t)1 << sh) <= S) {
            G.range_bins = 1;
            lp_arg = log2_parts | (sh << 8);
            // the bins pass's table then needs one bin's 2^sh slots only: a
            // smaller S, so more than one workgroup per CU fits its LDS
            const int64_t fit = ((int64_t)1 << sh) * 8 * (1 + G.n_aggs);
            if (fit < G.lds_bytes) {
                G.lds_bytes = (int)fit;
                fitted = true;
            }
        }
    }
    part_ws_bytes(G.n, X.log2p, &X, d_ws);
    X.log2p = lp_arg;
    // the partition kernel's grid: within the bound the workspace holds
    // chains for (part_grid_bound)
    const int64_t tile = (int64_t)G.threads * 8;
    const int64_t ntiles = (G.n + tile - 1) / tile;
    int64_t g = part_grid_bound(G.n);
    if (g > ntiles) g = ntiles;
    X.grid = (int)(g < 1 ? 1 : g);
    X.q = part_region_blocks(G.n, tile, X.grid, 1 << log2_parts);
    if ((uint64_t)X.q * (uint64_t)X.grid > X.max_blocks)
        return fqc::fail(FQ_E_INTERNAL, "fq_group_aggregate_partitioned: partition regions exceed the workspace");
    // more than one bins workgroup per CU only where both its table (fitted) and its registers (4-byte rows, 4
    // per thread: 54 VGPRs) leave room for it: g2's kernel set 4.58 -> 4.46 ms per partition
    // (profiles/r04_o_gbins_ab/)
    const bool two = fitted && G.narrow;  // 4 rows per thread in the narrow bins pass (fq_jit.hip)
    X.bins_grid = fqc::device_cu_count() * (two ? (int)fqc::knob(FQ_TUNE_GBINS_WG_PER_CU) : 1);
    return jit_groupby_partitioned(col->dtype, G, X);
}

fq_status fq_group_table_count(const fq_group_table *t, int64_t *groups, void *stream) {
    using namespace fqk;
    if (!groups) return fqc::fail(FQ_E_INVALID, "fq_group_table_count: NULL argument");
    *groups = 0;
    TableView v;
    fq_status s = view(t, v);
    if (s != FQ_OK) return s;
    hipStream_t st = (hipStream_t)stream;
    FQ_HIP_TRY(hipMemsetAsync(v.counter, 0, 8, st));
    hipLaunchKernelGGL(group_count_kernel, dim3(small_grid(v.cap)), dim3(256), 0, st, v.keys, v.cap, v.hdr,
                       v.counter);
    FQ_HIP_TRY(hipGetLastError());
    uint32_t flags;
    uint64_t c;
    s = read_header(v, flags, c, st);
    if (s != FQ_OK) return s;
    *groups = (int64_t)c;
    return FQ_OK;
}

fq_status fq_group_table_extract(const fq_group_table *t, uint64_t *d_keys, uint64_t *const *d_states, int64_t cap,
                                 int64_t *groups, void *stream) {
    using namespace fqk;
    if (!groups || !d_keys || !d_states) return fqc::fail(FQ_E_INVALID, "fq_group_table_extract: NULL argument");
    *groups = 0;
    TableView v;
    fq_status s = view(t, v);
    if (s != FQ_OK) return s;
    hipStream_t st = (hipStream_t)stream;
    ExtractArgs a{};
    a.keys = v.keys;
    a.out_keys = d_keys;
    a.n_aggs = t->n_aggs;
    for (int i = 0; i < t->n_aggs; ++i) {
        if (!d_states[i]) return fqc::fail(FQ_E_INVALID, "fq_group_table_extract: NULL state output");
        a.states[i] = v.states[i];
        a.out_states[i] = d_states[i];
        a.kinds[i] = t->kinds[i];
        a.dtypes[i] = t->dtypes[i];
    }
    a.replicas = v.replicas;
    a.cap = v.cap;
    a.out_cap = cap;
    a.hdr = v.hdr;
    a.counter = v.counter;
    FQ_HIP_TRY(hipMemsetAsync(v.counter, 0, 8, st));
    hipLaunchKernelGGL(group_extract_kernel, dim3(small_grid(v.cap + 1)), dim3(256), 0, st, a);
    FQ_HIP_TRY(hipGetLastError());
    uint32_t flags;
    uint64_t c;
    s = read_header(v, flags, c, st);
    if (s != FQ_OK) return s;
    if ((int64_t)c > cap) return fqc::fail(FQ_E_INVALID, "fq_group_table_extract: output arrays too small");
    *groups = (int64_t)c;
    return FQ_OK;
}

fq_status fq_group_table_merge(const fq_group_table *t, const uint64_t *d_keys, const uint64_t *const *d_states,
                               int64_t n, void *stream) {
    using namespace fqk;
    if (n < 0) return fqc::fail(FQ_E_INVALID, "fq_group_table_merge: negative row count");
    if (n > 0 && (!d_keys || !d_states)) return fqc::fail(FQ_E_INVALID, "fq_group_table_merge: NULL argument");
    TableView v;
    fq_status s = view(t, v);
    if (s != FQ_OK) return s;
    if (n == 0) return FQ_OK;
    MergeArgs a{};
    a.in_keys = d_keys;
    a.keys = v.keys;
    a.n_aggs = t->n_aggs;
    for (int i = 0; i < t->n_aggs; ++i) {
        if (!d_states[i]) return fqc::fail(FQ_E_INVALID, "fq_group_table_merge: NULL state array");
        a.in_states[i] = d_states[i];
        a.states[i] = v.states[i];
        a.kinds[i] = t->kinds[i];
        a.dtypes[i] = t->dtypes[i];
    }
    a.n = n;
    a.cap = v.cap;
    a.hdr = v.hdr;
    hipLaunchKernelGGL(group_merge_kernel, dim3(small_grid(n)), dim3(256), 0, (hipStream_t)stream, a);
    FQ_HIP_TRY(hipGetLastError());
    return FQ_OK;
}

}  // extern "C"
