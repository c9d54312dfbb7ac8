/*
 * fq_gpu.h -- C ABI of the MI355X (gfx950) kernels behind fuse-query's
 * DataBlock expression + aggregation hot path.
 *
 * Every entry point replaces one call site of the reference's CPU path
 * (dantengsky/fuse-query @ /root/reference, Rust + arrow 2.0 compute):
 *
 *   fq_fill_numbers_u64   NumbersStream::poll_next        src/datasources/system/numbers_stream.rs:65-83
 *   fq_fill_value         DataValue::to_array             src/datavalues/data_value.rs:77-111
 *   fq_aggregate          AggregatorFunction::accumulate  src/functions/function_aggregator.rs:57-100
 *                         (-> data_array_aggregate_op     src/datavalues/data_array_aggregate.rs:14-163,
 *                             arrow::compute::sum/min/max src/datavalues/macros.rs:143-157)
 *                         fused with the argument eval    src/functions/function_arithmetic.rs:64-72
 *                         and the WHERE predicate         src/transforms/transform_filter.rs:38-55
 *   fq_arith              data_array_arithmetic_op        src/datavalues/data_array_arithmetic.rs:14-55
 *   fq_compare            data_array_comparison_op        src/datavalues/data_array_comparison.rs:14-94
 *   fq_filter_compact     arrow filter_record_batch       src/transforms/transform_filter.rs:51
 *   fq_logic              data_array_logic_op             src/datavalues/data_array_logic.rs:10-31
 *   fq_state_merge        AggregatorFunction::merge_state src/functions/function_aggregator.rs:106-139
 *
 * Conventions:
 *   - plain pointers and sizes only; device buffers are owned by the caller and
 *     are never freed by the library;
 *   - column values use the Arrow layout: a contiguous values buffer (16-byte
 *     aligned for the vector path), no null bitmap; Boolean columns are
 *     LSB-first bit-packed into little-endian uint64 words;
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream); every
 *     call is asynchronous on that stream unless documented otherwise;
 *   - errors are returned as fq_status and the message (the reference's
 *     FuseQueryError display text where one exists, e.g.
 *     "Internal Error: Divide by zero error") is kept in a thread-local buffer
 *     readable with fq_last_error().
 */
#ifndef FQ_GPU_H
#define FQ_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FQ_ABI_VERSION 3

/* ---- status (src/error.rs:10-22 FuseQueryError{SQLParse,Plan,Internal}) ---- */
typedef int32_t fq_status;
#define FQ_OK 0
#define FQ_E_INTERNAL 1       /* FuseQueryError::Internal                       */
#define FQ_E_PLAN 2           /* FuseQueryError::Plan                           */
#define FQ_E_DIVIDE_BY_ZERO 3 /* ArrowError::DivideByZero -> Internal (error.rs:24-28) */
#define FQ_E_UNSUPPORTED 4    /* not supported on the device path (message says what) */
#define FQ_E_HIP 5            /* HIP runtime error / no GPU                     */
#define FQ_E_RCCL 6           /* RCCL error                                     */
#define FQ_E_INVALID 7        /* bad argument (null pointer, misaligned buffer, ...) */

/* ---- DataType (arrow::datatypes::DataType as used by src/datavalues/data_type.rs) ---- */
#define FQ_DT_NULL 0
#define FQ_DT_BOOLEAN 1
#define FQ_DT_INT8 2
#define FQ_DT_INT16 3
#define FQ_DT_INT32 4
#define FQ_DT_INT64 5
#define FQ_DT_UINT8 6
#define FQ_DT_UINT16 7
#define FQ_DT_UINT32 8
#define FQ_DT_UINT64 9
#define FQ_DT_FLOAT32 10
#define FQ_DT_FLOAT64 11
#define FQ_DT_UTF8 12

/* ---- operators (src/datavalues/data_value_operator.rs:5-81) ---- */
#define FQ_OP_ADD 0
#define FQ_OP_SUB 1
#define FQ_OP_MUL 2
#define FQ_OP_DIV 3
#define FQ_OP_MOD 4 /* EXTENSION: '%' has no arm in function_factory.rs:17-39 */
#define FQ_OP_PUSH 5 /* fq_step only: push acc, acc = the column (see FQ_OPERAND_STACK) */

#define FQ_CMP_EQ 0
#define FQ_CMP_LT 1
#define FQ_CMP_LTEQ 2
#define FQ_CMP_GT 3
#define FQ_CMP_GTEQ 4

/* aggregate op bit mask (DataValueAggregateOperator) */
#define FQ_AGG_MIN 1u
#define FQ_AGG_MAX 2u
#define FQ_AGG_SUM 4u
#define FQ_AGG_COUNT 8u

/*
 * A scalar DataValue (src/datavalues/data_value.rs:20-35), numeric/boolean
 * subset.  dtype FQ_DT_NULL is DataValue::Null; is_some=0 is `X(None)`.
 * bits: integers hold the value sign/zero-extended to 64 bits, floats hold
 * the IEEE binary64 bits (Float32 values are widened exactly), booleans 0/1.
 */
typedef struct fq_value {
    int32_t dtype;
    int32_t is_some;
    uint64_t bits;
} fq_value;

/* A device column: Arrow PrimitiveArray values buffer (or Boolean bitmap). */
typedef struct fq_col {
    void *data; /* device pointer */
    int64_t len;
    int32_t dtype;
    int32_t reserved;
} fq_col;

/*
 * Fusable expression: a chain of binary operators applied to one column x,
 *   acc = x;  for each step: acc = acc OP operand   (or operand OP acc if reversed)
 * where operand is a constant or x itself.  This is the shape that
 * Function::eval produces for ArithmeticFunction trees whose every right (or
 * left) child is a Constant/Field leaf (function_arithmetic.rs:64-72).
 * Each step carries the coerced type of that step
 * (numerical_coercion, data_type.rs:27-90); the library inserts the casts.
 */
#define FQ_MAX_STEPS 8
#define FQ_OPERAND_CONST 0
#define FQ_OPERAND_COLUMN 1
/* Expression TREES over the one column (e.g. (x + 1) + (x / 2)) use a
 * two-deep value stack: FQ_OP_PUSH pushes acc and restarts acc = x; a later
 * step with operand FQ_OPERAND_STACK pops that value as its operand
 * (reversed = 1: popped OP acc, the left subtree first, as the reference
 * evaluates ArithmeticFunction's children, function_arithmetic.rs:64-72).
 * The popped value is cast to the step's dtype like acc.  Trees run on the
 * hipRTC-specialised kernels only (FQ_E_UNSUPPORTED with FQ_JIT_OFF).     */
#define FQ_OPERAND_STACK 2
#define FQ_MAX_STACK 2
typedef struct fq_step {
    int32_t op;       /* FQ_OP_*                                  */
    int32_t operand;  /* FQ_OPERAND_CONST / FQ_OPERAND_COLUMN     */
    int32_t reversed; /* 1: operand OP acc (scalar-array form)    */
    int32_t dtype;    /* UINT64 / INT64 / FLOAT64                 */
    uint64_t bits;    /* constant in `dtype` (fq_value encoding)  */
} fq_step;

typedef struct fq_expr {
    int32_t n_steps; /* 0 = identity (the column itself)            */
    int32_t out_dtype; /* type of the result; == column type if n_steps==0 */
    fq_step steps[FQ_MAX_STEPS];
} fq_expr;

/* WHERE predicate, fused into the aggregate scan (transform_filter.rs:38-55). */
#define FQ_PRED_NONE 0
#define FQ_PRED_EXPR 1   /* cmp(lhs(x), rhs) with rhs a constant or x            */
#define FQ_PRED_BITMAP 2 /* precomputed Boolean column (from fq_compare)          */
#define FQ_PRED_TREE 3   /* and/or of up to FQ_MAX_PRED_LEAVES comparisons        */

/* One comparison leaf of an and/or predicate tree: cmp(lhs(x), rhs). */
typedef struct fq_pred_leaf {
    int32_t cmp, cmp_dtype, rhs_operand, reserved;
    uint64_t rhs_bits;
    fq_expr lhs;
} fq_pred_leaf;

/* LogicFunction trees (function_logic.rs) over comparisons of one column, as
 * a postfix program: prog[i] < FQ_MAX_PRED_LEAVES pushes leaf prog[i],
 * FQ_PRED_AND / FQ_PRED_OR pop two and push their and/or.  Both sides are
 * always evaluated (arrow and/or work on whole arrays), so an error in
 * either raises.                                                          */
#define FQ_MAX_PRED_LEAVES 4
#define FQ_PRED_AND 100
#define FQ_PRED_OR 101
typedef struct fq_pred_tree {
    int32_t n_leaves;
    int32_t n_prog;
    int32_t prog[2 * FQ_MAX_PRED_LEAVES];
    fq_pred_leaf leaves[FQ_MAX_PRED_LEAVES];
} fq_pred_tree;

typedef struct fq_pred {
    int32_t kind;
    int32_t cmp;         /* FQ_CMP_*  (already flipped for scalar-array forms)   */
    int32_t cmp_dtype;   /* equal_coercion type: UINT64 / INT64 / FLOAT64         */
    int32_t rhs_operand; /* FQ_OPERAND_CONST / FQ_OPERAND_COLUMN                  */
    uint64_t rhs_bits;   /* constant in cmp_dtype                                */
    fq_expr lhs;         /* lhs.out_dtype must equal cmp_dtype                   */
    const uint64_t *bitmap; /* device, kind == FQ_PRED_BITMAP                    */
    const fq_pred_tree *tree; /* host, kind == FQ_PRED_TREE (read during the call) */
} fq_pred;

/*
 * Partial aggregate over one device block = a run of `blocks` reference
 * blocks of `block_rows` rows (numbers_stream.rs:29 block_size = 10000; the
 * last one may be shorter).  Values are in `dtype` (fq_value bit encoding).
 * flags lets the host replay the reference's per-block state machine exactly:
 *   FQ_STATE_ANY_EMPTY   some reference block had no row left after the
 *                        predicate (arrow sum -> None -> the Sum state errors,
 *                        data_value_arithmetic.rs:10-27)
 *   FQ_STATE_DIV_ZERO    a row reaching an integer/float '/' or '%' had a zero
 *                        divisor (ArrowError::DivideByZero)
 *   FQ_STATE_CAST_NULL   a coercion cast overflowed (arrow cast -> null; nulls
 *                        are not representable on the device path)
 */
#define FQ_STATE_ANY_EMPTY 1u
#define FQ_STATE_DIV_ZERO 2u
#define FQ_STATE_CAST_NULL 4u
typedef struct fq_agg_state {
    uint64_t sum;   /* wrapping sum (integers) / binary64 sum bits (floats)      */
    uint64_t max;
    uint64_t min;
    uint64_t count;  /* rows that passed the predicate                           */
    uint64_t blocks; /* reference blocks covered                                 */
    uint32_t flags;
    int32_t dtype; /* value dtype                                               */
} fq_agg_state;

/* ---- library ---- */
int32_t fq_abi_version(void);
const char *fq_last_error(void);
fq_status fq_device_count(int32_t *out);

/* ---- SourceTransform: system.numbers_mt (numbers_stream.rs:65-83) ----
 * Writes d_out[i] = begin + i for i in [0, count).  One partition of
 * numbers_mt is one contiguous range (see SURVEY.md finding 8).            */
fq_status fq_fill_numbers_u64(uint64_t *d_out, uint64_t begin, uint64_t count, void *stream);
/* Anti-closed-form control column: d_out[i] = splitmix64(seed, first_index + i). */
fq_status fq_fill_splitmix64(uint64_t *d_out, uint64_t seed, uint64_t first_index,
                             uint64_t count, void *stream);

/* DataValue::to_array(size) (data_value.rs:77-111): broadcast one scalar.
 * dtype is a numeric type (bits in fq_value encoding) or FQ_DT_BOOLEAN
 * (writes ceil(n/64) bitmap words, bits past n cleared).                   */
fq_status fq_fill_value(void *d_out, int64_t n, int32_t dtype, uint64_t bits, void *stream);

/* ---- AggregatePartial: fused predicate + argument expression + sum/max/min/count ----
 * One pass over `col`; writes one fq_agg_state to device memory d_out.
 * block_rows: reference block size of this device block (10000 for
 * numbers_mt, or col->len for a single DataBlock).  Workspace is device
 * memory of at least fq_aggregate_workspace_bytes(col->len) bytes.
 * value may be NULL (identity).  pred may be NULL (no WHERE).
 *
 * The scan writes one partial per workgroup into the workspace; a second,
 * one-workgroup launch folds them into *d_out in a fixed order (the same
 * bytes run to run, float sums too).  Calls sharing a workspace must be
 * ordered (one stream).                                                     */
size_t fq_aggregate_workspace_bytes(int64_t len);
fq_status fq_aggregate(const fq_col *col, int64_t block_rows, const fq_pred *pred,
                       const fq_expr *value, uint32_t agg_mask, fq_agg_state *d_out,
                       void *d_ws, size_t ws_bytes, void *stream);

/* ---- ArithmeticFunction::eval (data_array_arithmetic.rs:14-55) ----
 * Exactly one of {lhs, lhs_scalar} and one of {rhs, rhs_scalar} is non-NULL.
 * out->data must hold out->len elements of the coercion type returned by
 * fq_arith_result_type.  d_flag: 4 bytes of device scratch; when non-NULL the
 * call synchronises `stream` and reports FQ_E_DIVIDE_BY_ZERO / cast nulls.   */
fq_status fq_arith_result_type(int32_t op, int32_t lhs_dtype, int32_t rhs_dtype, int32_t *out);
fq_status fq_arith(int32_t op, const fq_col *lhs, const fq_value *lhs_scalar, const fq_col *rhs,
                   const fq_value *rhs_scalar, fq_col *out, uint32_t *d_flag, void *stream);

/* ---- ComparisonFunction::eval (data_array_comparison.rs:14-94) ----
 * Writes an LSB-first bitmap of ceil(len/64) uint64 words (bits past len are 0).
 * Scalar-array forms flip the operator as the reference does (:76-84).       */
fq_status fq_compare(int32_t cmp, const fq_col *lhs, const fq_value *lhs_scalar,
                     const fq_col *rhs, const fq_value *rhs_scalar, uint64_t *d_bitmap,
                     int64_t len, uint32_t *d_flag, void *stream);

/* ---- LogicFunction::eval (function_logic.rs:47-53 -> data_array_logic.rs:10-31) ----
 * out = lhs AND/OR rhs over two Boolean bitmaps of `len` rows (ceil(len/64)
 * words each; bits past len are cleared in the output).  Both sides must be
 * Boolean ARRAYS: the reference errors on a scalar side ("Cannot do
 * data_array and, left:..., right:...") and on a non-Boolean array
 * ("Cannot downcast_array from datatype:<T> item to:BooleanArray"); those
 * checks are the caller's (engine/functions.cpp LogicFunction).          */
#define FQ_LOGIC_AND 0
#define FQ_LOGIC_OR 1
fq_status fq_logic(int32_t op, const uint64_t *d_lhs, const uint64_t *d_rhs, uint64_t *d_out, int64_t len,
                   void *stream);

/* ---- FilterTransform: order-preserving compaction (arrow filter_record_batch) ----
 * Synchronises `stream`; *out_len receives the number of rows kept.          */
size_t fq_filter_workspace_bytes(int64_t len);
fq_status fq_filter_compact(const fq_col *in, const uint64_t *d_bitmap, void *d_out,
                            int64_t *out_len, void *d_ws, size_t ws_bytes, void *stream);

/* ---- FilterTransform -> ProjectionTransform fused over one column ----
 * (transform_filter.rs:38-55 then transform_projection.rs:45-56 /
 * stream_expression.rs:37-50, for a predicate and expressions over the same
 * 64-bit column).  Keeps the rows of `col` where `pred` holds (NULL or
 * FQ_PRED_NONE: every row; FQ_PRED_BITMAP: the given bitmap) in order and
 * writes d_out[j][r] = values[j](kept row r) for j < n_out
 * (values[j].n_steps == 0: the column itself; the element type is
 * values[j].out_dtype, 8 bytes).  Errors follow the reference's order: a
 * predicate error on any row first ("Internal Error: Divide by zero error",
 * cast nulls), then an expression error on a kept row.  hipRTC-specialised
 * per expression shape (FQ_E_UNSUPPORTED when hipRTC is unavailable or the
 * JIT is off: the caller then runs fq_compare / fq_filter_compact /
 * fq_arith).  Synchronises `stream`; *out_len = rows kept.                  */
#define FQ_MAX_PROJECT 8
size_t fq_filter_project_workspace_bytes(int64_t len);
fq_status fq_filter_project(const fq_col *col, const fq_pred *pred, const fq_expr *values, int32_t n_out,
                            void *const *d_out, int64_t *out_len, void *d_ws, size_t ws_bytes, void *stream);
/* ---- FilterTransform -> ProjectionTransform over a stream of DataBlocks ----
 * The reference runs both transforms block by block: ExpressionStream applies
 * FilterTransform::expression_executor (transform_filter.rs:38-55) to every
 * block the numbers stream yields (numbers_stream.rs:29-48, 10,000 rows), then
 * ProjectionTransform (transform_projection.rs:45-56) to each filtered block.
 * This is that loop over a batch of blocks in one call: `col` holds
 * ceil(len / block_rows) blocks of block_rows consecutive rows (the last may
 * be short); block b's kept rows are written in order to
 * d_out[j][b * block_rows + r] for r < d_counts[b] (device int64, one per
 * block): each output block starts where its input block does, so no block
 * waits on another's count.  d_out[j] must hold len rows; rows of a block past
 * its count are left as they were.  block_rows >= FQ_PROJECT_MIN_BLOCK_ROWS
 * (the kernel's tile); blocks are independent, so a call runs on up to
 * ceil(len / block_rows) workgroups.  *out_len = rows kept over all blocks.
 * Predicate kinds, expressions and the error order are fq_filter_project's.
 * Synchronises `stream`.                                                    */
#define FQ_PROJECT_MIN_BLOCK_ROWS 8192
size_t fq_filter_project_blocks_workspace_bytes(void);
fq_status fq_filter_project_blocks(const fq_col *col, int64_t block_rows, const fq_pred *pred,
                                   const fq_expr *values, int32_t n_out, void *const *d_out, int64_t *d_counts,
                                   int64_t *out_len, void *d_ws, size_t ws_bytes, void *stream);
/* A block stream's valid rows as one array: for each of n_cols 64-bit columns
 * of the geometry above (len rows, ceil(len / block_rows) blocks, block b's
 * valid rows the first d_counts[b] of its range), d_out[j] receives block 0's
 * rows, then block 1's, ... (what arrow's concat of the reference's filtered
 * blocks would hold).  *out_len (optional: the call then synchronises
 * `stream`) = the rows written.  Workspace: fq_blocks_compact_workspace_bytes.
 */
size_t fq_blocks_compact_workspace_bytes(int64_t n_blocks);
fq_status fq_blocks_compact(int32_t n_cols, const void *const *d_in, int64_t len, int64_t block_rows,
                            const int64_t *d_counts, void *const *d_out, int64_t *out_len, void *d_ws, size_t ws_bytes,
                            void *stream);
/* FilterTransform's predicate alone as a Boolean column: LSB-first bitmap of
 * ceil(len/64) words, bits past len cleared (one kernel instead of one
 * fq_arith per expression node plus fq_compare).  d_flag: 4 bytes of device
 * scratch; the call synchronises `stream` and reports predicate errors.    */
fq_status fq_predicate_bitmap(const fq_col *col, const fq_pred *pred, uint64_t *d_bitmap, uint32_t *d_flag,
                              void *stream);

/* ---- AggregateFinal state merge (host, function_aggregator.rs:106-139) ----
 * Merges `n` partial states in the given order into *out (wrapping sum,
 * summed counts/blocks, max, min, OR-ed flags).  All dtypes must match.      */
fq_status fq_state_merge(const fq_agg_state *states, int32_t n, fq_agg_state *out);

/* ---- Expression specialisation for fq_aggregate (no reference counterpart:
 * the reference evaluates each Function node per block, function.rs:17-132).
 * A fused predicate/argument expression is compiled once per expression
 * SHAPE (ops, operand kinds, dtypes; constants stay kernel arguments) with
 * hipRTC into a straight-line gfx950 scan kernel and cached for the process.
 * Shapes below `min_rows` rows, or with the JIT off, run the precompiled
 * program-interpreting kernel (same results, bit for bit).
 *   mode FQ_JIT_OFF    always interpret
 *   mode FQ_JIT_AUTO   specialise when col->len >= min_rows (default 2^22;
 *                      silently interprets if hipRTC cannot be loaded)
 *   mode FQ_JIT_ALWAYS specialise every fused expression; fails with
 *                      FQ_E_UNSUPPORTED if hipRTC cannot be loaded
 * Initial values come from $FQ_JIT (0/1/2) and $FQ_JIT_MIN_ROWS.           */
#define FQ_JIT_OFF 0
#define FQ_JIT_AUTO 1
#define FQ_JIT_ALWAYS 2
typedef struct fq_jit_stats {
    int64_t kernels_compiled; /* distinct shapes compiled in this process        */
    int64_t jit_launches;     /* fq_aggregate scans run by a specialised kernel  */
    int64_t interp_launches;  /* fused scans run by the interpreting kernel      */
    double compile_ms;        /* total hipRTC compile + module load time         */
    int32_t available;        /* 1 if hipRTC loaded, 0 if not, -1 not tried yet  */
    int32_t mode;
    int64_t min_rows;
} fq_jit_stats;
fq_status fq_jit_config(int32_t mode, int64_t min_rows);
fq_status fq_jit_get_stats(fq_jit_stats *out);
/* Compiles (and caches) the specialised kernel fq_aggregate would use for
 * this call shape, so the first scan does not pay the compile; col->data may
 * be NULL.  *specialised = 1 if the shape has a specialised kernel (mode not
 * OFF, a fused 64-bit expression).  Without a GPU the generated source is
 * compiled for gfx950 only to validate it.                                  */
fq_status fq_jit_prepare(const fq_col *col, int64_t block_rows, const fq_pred *pred,
                         const fq_expr *value, uint32_t agg_mask, int32_t *specialised);

/* ---- Launch-shape knobs (tuning tools only; no reference counterpart) ----
 * Every knob has a compiled-in default, the measured best on MI355X
 * (DESIGN.md "Launch-shape knobs" names the sweep each came from).  The
 * library reads no environment variable for them and never prints: the sweep
 * tools (bench.py --tune, tools/) set them here.  Knobs read by a hipRTC
 * kernel are part of its shape key, so a change applies from the next launch. */
#define FQ_TUNE_SCAN_WG_PER_CU 0      /* fused aggregate scan: workgroups per CU, 2 (1..16)           */
#define FQ_TUNE_EW_WG_PER_CU 1        /* arith/compare kernels: 0 = per-op defaults (8/2), 1..16      */
#define FQ_TUNE_BLOCK_U 2             /* block-mode scan: 16-B vectors per lane in flight, 8 (4/8/16) */
#define FQ_TUNE_SELECT_WG_PER_CU 3    /* filter+projection (look-back kernel): workgroups per CU, 8 (1..16) */
#define FQ_TUNE_SELECT_BLOCKS_WG_PER_CU 4 /* block-stream filter+projection: workgroups per CU, 8 (1..16) */
#define FQ_TUNE_SELECT_BLOCKS_ROWS 5  /* block-stream filter+projection: rows per thread per tile, 32 (8/16/32) */
#define FQ_TUNE_SELECT_BLOCKS_STAGE 6 /* block-stream filter+projection: kept rows staged in LDS and written by
                                         consecutive threads, the stage 1/S of a tile: S = 2 (0 = off, 1/2/4) */
#define FQ_TUNE_BLOCK_CACHE 7         /* engine's stream-ordered device block cache, 1 (0/1)          */
#define FQ_TUNE_POOL_SPIN_US 8        /* engine pipe threads poll for the next task before sleeping, 0 us (0..100000) */
#define FQ_TUNE_GROUP_THREADS 9       /* GROUP BY kernels: threads per workgroup, 1024 (256..1024 step 256) */
#define FQ_TUNE_GROUP_LDS_KB 10       /* GROUP BY LDS table budget, 128 (8..160)                      */
#define FQ_TUNE_GROUP_WG_PER_CU 11    /* GROUP BY LDS kernel workgroups per CU: 1 (1..8)              */
#define FQ_TUNE_GROUP_CLUSTER 12      /* clustered row layout threshold (key changes/wave): 160 (0..512) */
#define FQ_TUNE_GROUP_CHUNKED 13      /* contiguous tile runs per workgroup: 1 (0/1)                  */
#define FQ_TUNE_GROUP_RANGE_BINS 14   /* partitioned GROUP BY: range bins for `% d` keys, 1 (0/1)     */
#define FQ_TUNE_GROUP_NARROW 15       /* partitioned GROUP BY: honour FQ_GROUP_NARROW_ROWS, 1 (0/1)   */
#define FQ_TUNE_GPART_WG_PER_CU 16    /* GROUP BY partition kernel: workgroups per CU, 2 (1..4)       */
#define FQ_TUNE_GBINS_WG_PER_CU 17    /* GROUP BY bins pass, fitted table: workgroups per CU, 2 (1..4) */
#define FQ_TUNE_COUNT 18
/* FQ_E_INVALID for an unknown knob or a value outside the knob's set */
fq_status fq_tune_set(int32_t knob, int64_t value);
/* the knob's current value; -1 for an unknown knob */
int64_t fq_tune_get(int32_t knob);
/* every knob back to its default */
fq_status fq_tune_reset(void);
/* dir != NULL: every hipRTC source compiled from now on is written to dir
 * (with its code object) for ISA inspection; NULL turns it off.            */
fq_status fq_tune_jit_dump_dir(const char *dir);

/* ---- GROUP BY hash aggregation (NO reference counterpart:
 * plan_parser.rs:284-308 plans group_expr but pipeline_builder.rs:50-66 builds
 * AggregatePartial/Final from aggr_expr only, so the reference has no grouped
 * semantics to match.  Here a group is a distinct value of an integer key
 * expression over the column; each aggregate is count/sum/min/max of an
 * argument expression over the rows of the group that pass the predicate,
 * with the same value semantics as fq_aggregate (wrapping integer sums, f64
 * IEEE sums in unspecified order).
 *
 * The table is caller-owned device memory of fq_group_table_bytes(capacity,
 * n_aggs) bytes described by an fq_group_table; capacity is a power of two.
 * One extra slot holds the key 0xFFFFFFFFFFFFFFFF (the empty marker).
 * fq_group_aggregate streams a column once: every workgroup pre-aggregates
 * in an LDS hash table and flushes its groups into the HBM table with
 * atomics; keys that do not fit in LDS go to HBM directly.  The kernel is
 * specialised per expression shape with hipRTC (see fq_jit_config); there is
 * no interpreting fallback, so it fails with FQ_E_UNSUPPORTED if hipRTC
 * cannot be loaded.  A table that runs out of slots is reported by
 * fq_group_table_count (FQ_E_TABLE_FULL): re-run into a larger table.       */
#define FQ_MAX_GROUP_AGGS 8
#define FQ_E_TABLE_FULL 8
typedef struct fq_group_table {
    void *d_mem;       /* fq_group_table_bytes(capacity, n_aggs) bytes, device */
    int64_t capacity;  /* slots, a power of two >= 64                          */
    int32_t key_dtype; /* FQ_DT_UINT64 or FQ_DT_INT64                          */
    int32_t n_aggs;    /* 1..FQ_MAX_GROUP_AGGS                                 */
    int32_t kinds[FQ_MAX_GROUP_AGGS];  /* FQ_AGG_COUNT / SUM / MIN / MAX        */
    int32_t dtypes[FQ_MAX_GROUP_AGGS]; /* state dtype: COUNT UInt64, else the
                                          argument's dtype (64-bit types)      */
} fq_group_table;
size_t fq_group_table_bytes(int64_t capacity, int32_t n_aggs);
/* Empties the table (async on stream). */
fq_status fq_group_table_init(const fq_group_table *t, void *stream);
/* Accumulates one device block: key = key_expr(x) (fq_expr over col, integer
 * result of dtype t->key_dtype), aggregate i over values[i](x), rows kept by
 * pred (may be NULL).  Asynchronous. */
fq_status fq_group_aggregate(const fq_group_table *t, const fq_col *col, const fq_pred *pred,
                             const fq_expr *key_expr, const fq_expr *values, void *stream);
/* High-cardinality variant: the rows kept by pred are radix-partitioned by
 * key (range for a `% d` key, else hash) into 2^log2_parts bins (1..8) -- one
 * read + write pass over col into 2 KB block chains in d_ws, the blocks then
 * grouped by bin -- and then aggregated bin by bin, so each workgroup's LDS
 * table only meets the groups of one bin (about groups / 2^log2_parts of
 * them).  Same table, results and errors as fq_group_aggregate; 24 B of HBM
 * traffic per kept row instead of 8 B plus random HBM atomics once the groups
 * outgrow LDS.  d_ws: 256-B aligned, at least
 * fq_group_partition_workspace_bytes(col->len, log2_parts) bytes (about 8 B
 * per row plus ~2 KB per (workgroup, bin) chain).  Asynchronous. */
/* FQ_GROUP_NARROW_ROWS or-ed into log2_parts: the caller guarantees that every
 * value v of the (8-byte integer) column lies within 2^31 of col[0] (e.g. a
 * numbers_mt block: consecutive integers).  The partition pass then writes
 * each kept row as a 4-byte offset from col[0] - 2^31 instead of the 8-byte
 * value: 16 B of HBM traffic per kept row instead of 24.  A value outside
 * the range is reported at count/extract (FQ_E_INVALID); Float64 columns
 * ignore the flag.                                                          */
#define FQ_GROUP_NARROW_ROWS 0x10000
size_t fq_group_partition_workspace_bytes(int64_t len, int32_t log2_parts);
fq_status fq_group_aggregate_partitioned(const fq_group_table *t, const fq_col *col, const fq_pred *pred,
                                         const fq_expr *key_expr, const fq_expr *values, int32_t log2_parts,
                                         void *d_ws, size_t ws_bytes, void *stream);
/* Dense keys: when key_expr over a column of col_dtype is a UInt64 key
 * ending in `% d` by a constant and d fits the kernel's LDS table for n_aggs
 * states, the kernel indexes that table by the key itself (no hashing, never
 * saturated) and the query has at most d groups: returns d, else 0. */
int64_t fq_group_dense_keys(int32_t col_dtype, const fq_expr *key_expr, int32_t n_aggs);
/* Number of groups (synchronises stream); FQ_E_TABLE_FULL if any insert
 * found no free slot, FQ_E_DIVIDE_BY_ZERO / FQ_E_UNSUPPORTED for the flags
 * fq_aggregate reports. */
fq_status fq_group_table_count(const fq_group_table *t, int64_t *groups, void *stream);
/* Compacts the occupied slots into d_keys[0..groups) and, per aggregate i,
 * d_states[i][0..groups) (64-bit state bits; slot order, unsorted);
 * *groups = the number written (synchronises stream).  cap = room in the
 * output arrays. */
fq_status fq_group_table_extract(const fq_group_table *t, uint64_t *d_keys, uint64_t *const *d_states,
                                 int64_t cap, int64_t *groups, void *stream);
/* Merge n (key, state) rows -- d_keys[n] and d_states[a][n] as the table's
 * state bits, e.g. other GPUs' extracted tables -- into t: a new key claims a
 * slot, an existing one folds with the table's kinds (Count / Sum add, Max /
 * Min keep the extreme), atomically.  The cross-GPU AggregateFinal of a GROUP
 * BY (no reference counterpart: the reference has no GROUP BY execution).
 * A table too small for the keys reports FQ_E_TABLE_FULL on count/extract.  */
fq_status fq_group_table_merge(const fq_group_table *t, const uint64_t *d_keys, const uint64_t *const *d_states,
                               int64_t n, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* FQ_GPU_H */
