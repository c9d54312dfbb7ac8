// One fused-scan launch as prepared by fq_aggregate (fq_aggregate.hip) and
// consumed by either the precompiled program-interpreting kernels or a
// hipRTC-specialised kernel (fq_jit.hip).  Internal; not part of the ABI.
#pragma once

#include <stdlib.h>

#include "fq_common.h"
#include "fq_device.h"

namespace fqk {

constexpr int kThreads = 256;       // 4 waves per workgroup
constexpr int kMaxPartials = 4096;  // workgroups per launch upper bound
// the workspace: kMaxPartials Partials, folded by agg_finalize_kernel
constexpr size_t kPartialsBytes = (size_t)kMaxPartials * sizeof(Partial);

struct Launch {
    const void *col;
    int64_t n;
    int64_t head;  // flat mode: scalar elements before the first 16-byte boundary
    int64_t block_rows;
    bool block_mode;
    KPred pred;
    KProg val;
    uint32_t mask;
    int32_t vdtype;
    Partial *parts;
    int grid;
    hipStream_t stream;
};

// Host lowering (fq_aggregate.hip): fq_expr -> KProg (res_dtype = result
// type) and fq_pred -> KPred.
fq_status lower_expr(const fq_expr &e, int32_t col_dtype, KProg &out, int32_t &res_dtype);
fq_status lower_pred(const fq_pred *pred, int32_t col_dtype, int64_t len, bool need_data, KPred &out);

// Launches the scan of `L` from a specialised kernel when the JIT policy
// (fq_jit_config) selects it -- or, with `force` (expression trees, which the
// interpreter does not run), whenever the JIT is not off; *used tells the
// caller whether it did.
fq_status jit_scan(int32_t col_dtype, bool chain, const Launch &L, bool *used, bool force = false);

// expression trees (FQ_OP_PUSH / FQ_OPERAND_STACK) in a lowered program
inline bool prog_has_tree(const KProg &p) {
    for (int i = 0; i < p.n; ++i)
        if (p.s[i].code == K_PUSH) return true;
    return false;
}
inline bool pred_has_tree(const KPred &p) {
    if (p.kind == FQ_PRED_EXPR) return prog_has_tree(p.lhs);
    if (p.kind == FQ_PRED_TREE)
        for (int l = 0; l < p.n_leaves; ++l)
            if (prog_has_tree(p.leaves[l].lhs)) return true;
    return false;
}

// Compiles (and caches) the specialised kernel for L's shape ahead of the
// first scan; *ready = the shape is specialisable.  Without a device the
// source is compiled for gfx950 only to validate it.
fq_status jit_prepare(int32_t col_dtype, bool chain, const Launch &L, bool *ready);

// State replicas of a group table of `cap` slots: workgroup b updates replica
// b % R, so the 256 flushing workgroups (one per CU) contend at most 16-fold
// for one group's state words (the extract folds the replicas).
// R * cap <= 2^22 words per aggregate (32 MB), at most 16 replicas; tables
// of 2^22 slots and more get one.
inline int group_replicas(int64_t cap) {
    int r = 1;
    while (r < 16 && cap * (int64_t)r * 2 <= ((int64_t)1 << 22)) r *= 2;
    return r;
}

// One fq_group_aggregate launch (fq_groupby.hip -> fq_jit.hip).
struct GroupLaunch {
    const void *col;
    int64_t n;
    int64_t head;
    KPred pred;
    KProg key;  // key expression (lowered); n == 0 = the column itself
    int32_t key_dtype;
    int32_t n_aggs;
    int32_t kinds[FQ_MAX_GROUP_AGGS];
    int32_t dtypes[FQ_MAX_GROUP_AGGS];
    bool chain[FQ_MAX_GROUP_AGGS];
    KProg vals[FQ_MAX_GROUP_AGGS];
    uint64_t *keys;  // capacity + 1 slots
    uint64_t *states[FQ_MAX_GROUP_AGGS];
    uint32_t *hdr;
    int64_t capacity;
    int lds_bytes;  // LDS hash table budget per workgroup (sets S and the occupancy)
    int threads;    // workgroup size
    int rowmap;     // 1: lane-consecutive rows (8-byte loads), 0: row pairs per lane (16-byte loads)
    int narrow;     // partitioned path: 4-byte rows (offsets from col[0] - 2^31, FQ_GROUP_NARROW_ROWS)
    int range_bins; // partitioned path: bin = key >> log2(S) and LDS slot = key & (S - 1) (a UInt64
                    // key below d <= P * S: `% d`), else bins by the key's hash
    int grid;
    hipStream_t stream;
};

// Keys of a dense GROUP BY key (a UInt64 key ending in `% d`, d <= the LDS
// slots for n_aggs states in lds_bytes): d, else 0 (fq_jit.hip)
int64_t group_dense_bound(const KProg &key, int32_t key_dtype, int n_aggs, int lds_bytes);
// d for a UInt64 key ending in `% d` / `& (d - 1)` (keys in [0, d)), else 0;
// and the LDS table slots S for n_aggs states in lds_bytes
int64_t group_key_range(const KProg &key, int32_t key_dtype);
int group_lds_slots(int n_aggs, int lds_bytes);

// Launches the hipRTC-specialised group-by kernel for G.
fq_status jit_groupby(int32_t col_dtype, const GroupLaunch &G);

// The partitioned (high-cardinality) path of fq_group_aggregate_partitioned:
// partition into block chains -> blocks grouped by bin -> per-bin
// aggregation, in the caller's workspace (fq_groupby.hip lays it out).
constexpr int kMaxPartGrid = 1024;    // workgroups of the partition kernel
constexpr int kPartBlockRows = 256;   // rows per partition block (2 KB of u64; narrow blocks hold 2x the rows)
struct GroupPartition {
    int log2p;            // bits 0..7: 1..8, P = 2^log2p bins; bits 8..15: the key shift of range bins
    int grid;             // workgroups of fq_jit_gpart
    int bins_grid;        // workgroups of fq_jit_groupby_bins
    uint32_t max_blocks;  // blocks the workspace holds
    uint32_t q;           // blocks per workgroup region: workgroup w of fq_jit_gpart owns [w q, (w + 1) q)
    uint32_t *head;       // [kMaxPartGrid] blocks used per region + [256] blocks per bin: zeroed per launch
    size_t head_bytes;
    uint32_t *used;       // [grid] (head)
    uint32_t *bin_blocks; // [P] blocks per bin (head + kMaxPartGrid)
    uint32_t *bstart;     // [P + 1] each bin's first entry in order
    uint32_t *cursor;     // [P] scatter cursors
    uint32_t *blk_bin;    // [max_blocks] each block's bin
    uint32_t *blk_fill;   // [max_blocks] its rows
    uint64_t *order;      // [max_blocks] block | rows << 32, grouped by bin
    void *vals;           // max_blocks x kPartBlockRows rows (8-byte values, or 4-byte offsets when narrow)
};
fq_status jit_groupby_partitioned(int32_t col_dtype, const GroupLaunch &G, const GroupPartition &X);
// the blocks of fq_jit_gpart grouped by bin: a scan of X.bin_blocks into
// X.bstart, then a scatter of the block numbers into X.order (fq_groupby.hip)
fq_status launch_group_part_blocks(const GroupPartition &X, hipStream_t stream);

// One fq_filter_project / fq_predicate_bitmap call (fq_filter.hip ->
// fq_jit.hip): FilterTransform's predicate and ProjectionTransform's
// expressions over one 64-bit column, hipRTC-specialised per shape.
struct ProjLaunch {
    const void *col;
    int64_t n;
    KPred pred;  // FQ_PRED_NONE / EXPR / TREE (a BITMAP predicate skips the bits kernel)
    int32_t n_out;
    KProg vals[FQ_MAX_PROJECT];
    bool chain[FQ_MAX_PROJECT];
    int32_t dtypes[FQ_MAX_PROJECT];
    void *out[FQ_MAX_PROJECT];
    hipStream_t stream;
};

// predicate -> LSB-first bitmap words; predicate errors OR-ed into *d_flag
fq_status jit_project_bits(int32_t col_dtype, const ProjLaunch &P, uint64_t *d_bitmap, uint32_t *d_flag);
// one pass: predicate (or P.pred.bitmap), decoupled look-back over tiles of
// select_tile_rows() rows for the output offsets, the n_out outputs of the kept
// rows.  status: one zeroed word per tile; ticket: one zeroed word;
// d_flags[0] predicate errors, d_flags[1] expression errors (bit 31: the
// look-back gave up); *d_total = rows kept.
// tile = select_threads() x select_rows_per_thread() rows, s_sleep
// select_sleep() between look-back polls of a predecessor that has not
// published (round-2 sweeps, tools/select_sweep.sh; their knobs were removed
// in round 6)
constexpr int select_threads() { return 256; }
constexpr int select_rows_per_thread() { return 32; }
constexpr int select_sleep() { return 2; }
constexpr int64_t select_tile_rows() { return (int64_t)select_threads() * select_rows_per_thread(); }
fq_status jit_project_select(int32_t col_dtype, const ProjLaunch &P, const uint64_t *d_bitmap, uint64_t *status,
                             uint32_t *ticket, uint32_t *d_flags, uint64_t *d_total);
// stream of DataBlocks of block_rows rows (fq_filter_project_blocks): block b's
// kept rows -> output rows [b * block_rows, + d_counts[b]); tiles of
// kProjectBlockTile rows (kProjectBlockThreads threads), block_rows >= the tile;
// d_flags / *d_total / *d_ticket as jit_project_select (zeroed by the caller)
constexpr int kProjectBlockThreads = 256;
constexpr int64_t kProjectBlockTile = 256 * 32;
fq_status jit_project_blocks(int32_t col_dtype, const ProjLaunch &P, int64_t block_rows, const uint64_t *d_bitmap,
                             int64_t *d_counts, uint32_t *d_flags, uint64_t *d_total, uint32_t *d_ticket);
// filter_project_blocks_enqueue / _result: fq_common.h (the engine calls them)
// no predicate: every row -> the n_out outputs
fq_status jit_project_map(int32_t col_dtype, const ProjLaunch &P, uint32_t *d_flag);
// hipRTC loadable and the policy not FQ_JIT_OFF
bool jit_project_available();
// compiles (and caches) P's module; without a device the source is compiled
// for gfx950 only to validate it
fq_status jit_project_prepare(int32_t col_dtype, const ProjLaunch &P);

// Counts a fused (non-identity) scan that ran on the interpreting kernel.
void jit_count_interp();

}  // namespace fqk
