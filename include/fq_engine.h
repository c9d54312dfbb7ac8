/*
 * fq_engine.h -- C ABI of the pipeline layer: the C++ restatement of the
 * reference's query path (SQL -> plan -> PipelineBuilder -> IProcessor
 * transforms) running its DataBlocks on the gfx950 kernels of fq_gpu.h.
 *
 *   fq_engine_execute        SelectExecutor::execute        src/executors/executor_select.rs:35-40
 *                            (PipelineBuilder::build        src/processors/pipeline_builder.rs:26-106,
 *                             Pipeline::execute             src/processors/pipeline.rs:129-134)
 *   fq_engine_explain        ExplainExecutor::execute       src/executors/executor_explain.rs:38-59
 *   fq_engine_execute_partial / fq_engine_execute_final
 *                            the AggregatePartial -> Merge -> AggregateFinal split
 *                            (transform_aggregate_partial.rs:50-78, transform_aggregate_final.rs:50-78)
 *                            cut at the merge so ranks on different GPUs can exchange
 *                            their partial states (one RCCL all-reduce) in between
 *   fq_engine_materialize_numbers
 *                            system.numbers_mt partitions pinned in HBM
 *                            (NumbersTable::read, numbers_table.rs:94-96)
 *
 * Results are host copies: one fq_result per query, column names as the
 * reference formats them (`format!("{:?}", func)`, plan_expression.rs:31-38),
 * values as fq_value (see fq_gpu.h).
 */
#ifndef FQ_ENGINE_H
#define FQ_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#include "fq_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fq_engine fq_engine;
typedef struct fq_result fq_result;

/* engine options */
#define FQ_OPT_WORKER_THREADS 1 /* FuseQueryContext::worker_threads (context.rs:11); default 8 */
#define FQ_OPT_MODULO 2         /* 1 (default): '%' extension on; 0: reference behaviour
                                   ("Unsupported Function: %", function_factory.rs:34-37) */
#define FQ_OPT_PROFILE 3        /* 1: time every fused scan launch with a HIP event pair;
                                   2: one span per query -- a timing event right before
                                   its first scan and the query's end event behind its
                                   last (scan_ms then includes the launch gaps between
                                   the scans, and on a generated partition its fills):
                                   no event between two scans.  Row-pipeline and GROUP
                                   BY launches are timed per launch with 1 or 2 */
#define FQ_OPT_STREAMS 4        /* device queues the aggregate pipes share (default 1: the scans
                                   are HBM-bound; two cost 5.5 %).  Row pipelines without a LIMIT
                                   use two row queues of their own, with a LIMIT one private
                                   queue per pipe.  Set it between queries: the call waits for
                                   the device, and a new count flushes the block cache */
#define FQ_OPT_CHUNK_ROWS 5     /* rows per device block of a numbers_mt partition that is NOT
                                   resident (a multiple of 10,000; default 400,000,000 = 3.2 GB):
                                   aggregates over numbers_mt(1e12) stream through bounded HBM
                                   like the reference's 10,000-row blocks do through RAM */
#define FQ_OPT_GROUP_CHUNK_ROWS 6 /* rows per radix-partitioned GROUP BY launch (a positive
                                   multiple of 64; default 500,000,000: at most a ~4.3 GB
                                   partition workspace, which the device block cache keeps per
                                   queue; a block is split into equal chunks of at most this) */
#define FQ_OPT_FAULT_PIPE 7     /* testing: pipe k (1-based; 0 = off, the default) of the next
                                   merged queries fails while it sets up its device context, as a
                                   failed workspace allocation would -- the query must return
                                   that error, never wait for the pipe (processor_merge.rs:50-54) */

typedef struct fq_engine_stats {
    uint64_t scan_launches; /* fused aggregate scans launched                    */
    uint64_t scan_rows;     /* rows those scans read                            */
    uint64_t scan_bytes;    /* algorithmic bytes those scans read               */
    double scan_ms;         /* summed event time of those launches (FQ_OPT_PROFILE 1),
                               or of the queries' scan spans (FQ_OPT_PROFILE 2) */
    uint64_t queries;
    double plan_ms;         /* host: SQL parse + plan + PipelineBuilder, summed   */
    double exec_ms;         /* host: pipeline execution until the result block    */
    double first_launch_ms; /* host: query start -> first scan enqueued, summed   */
    /* the distributed split (fq_engine_execute_partial / _final and the
     * exchange between them, fq_comm.h), host wall time summed over calls    */
    double partial_ms;       /* fq_engine_execute_partial                      */
    double exchange_ms;      /* the exchange's all-reduce rounds (incl. waiting
                                for the slowest rank to arrive)                */
    double final_ms;         /* fq_engine_execute_final                        */
    uint64_t exchanges;      /* exchanges run                                  */
    uint64_t exchange_rounds; /* all-reduce rounds those took (1 or 2 each)    */
    uint64_t exchange_bytes; /* bytes all-reduced, summed over rounds          */
    /* gauges (the process's device block cache now; not reset) */
    uint64_t cached_block_bytes;     /* idle small blocks kept for reuse       */
    uint64_t cached_workspace_bytes; /* idle per-queue GROUP BY workspaces     */
    /* FilterTransform -> ProjectionTransform over block streams (one
     * fq_filter_project_blocks launch per device block of a partition)       */
    uint64_t project_launches;
    uint64_t project_rows;  /* rows those launches read                       */
    uint64_t project_kept;  /* rows they kept                                 */
    uint64_t project_bytes; /* algorithmic bytes: 8 per row read + 8 per kept
                               row per projected column                       */
    double project_ms;      /* FQ_OPT_PROFILE 1: the launches' event pairs, summed;
                               2: per query, earliest first-launch start to latest
                               end over the row queues (overlap counted once) */
    double tail_ms;         /* host, FQ_OPT_PROFILE 2: the scans' end event seen ->
                               the result block (merge + AggregateFinal), summed */
    double complete_ms;     /* of tail_ms: reading the partitions' states into their
                               aggregators (AggregatePartial's deferred blocks)  */
} fq_engine_stats;

/* device: HIP device ordinal.  Fails with FQ_E_HIP when no GPU is present.
 * device = -1 creates a host-only engine: SQL planning, EXPLAIN and
 * fq_engine_execute_final (the AggregateFinal merge of exchanged states,
 * which the reference also runs on the host) work; anything that touches a
 * column fails with FQ_E_HIP -- there is no CPU fallback for the hot path. */
fq_status fq_engine_create(int32_t device, fq_engine **out);
void fq_engine_destroy(fq_engine *e);
fq_status fq_engine_set_option(fq_engine *e, int32_t option, int64_t value);

/* Materialise (and keep resident) the numbers_mt(total) partitions that rank
 * `rank` of `world` owns ([8r/G, 8(r+1)/G) of generate_parts).  Queries over
 * numbers_mt(total) then read these instead of regenerating them.          */
fq_status fq_engine_materialize_numbers(fq_engine *e, uint64_t total, int32_t rank, int32_t world);
fq_status fq_engine_release_numbers(fq_engine *e);

/* Hand the engine's idle device memory back to the driver: the stream-ordered
 * block cache is flushed and the default memory pool trimmed to 0.  The engine
 * does this by itself before every retry of a failed allocation; a host that
 * shares the GPU with another allocator (e.g. PyTorch's caching allocator)
 * calls it before a large allocation of its own.                           */
fq_status fq_engine_trim_memory(fq_engine *e);

/* Run a SELECT through the whole pipeline on this engine's GPU. */
fq_status fq_engine_execute(fq_engine *e, const char *sql, fq_result **out);

/* EXPLAIN-style text: the plan and the pipeline (processor.rs:33-57 format). */
fq_status fq_engine_explain(fq_engine *e, const char *sql, char *buf, size_t cap, size_t *len);

/* Distributed aggregate: rank r runs Source -> Filter -> AggregatePartial for
 * its partitions and merges them locally; the merged partial states are
 * serialised into buf (fixed 16-byte DataValue records).  *len gets the size;
 * when cap is too small the call fails with FQ_E_INVALID and *len holds the
 * size needed.                                                              */
fq_status fq_engine_execute_partial(fq_engine *e, const char *sql, int32_t rank, int32_t world,
                                    void *buf, size_t cap, size_t *len);
/* Size in bytes of the serialised partial states fq_engine_execute_partial
 * produces for `sql` on ANY rank: an ungrouped aggregate's states have one
 * fixed-size record per state value of each function (the shape of
 * accumulate_result(), function.rs:28-131), so every rank can size the
 * exchange without first exchanging lengths.  0 when the size depends on the
 * data (GROUP BY: one row per group).                                       */
fq_status fq_engine_partial_state_bytes(fq_engine *e, const char *sql, size_t *bytes);
/* AggregateFinal over `world` serialised partial states laid out back to back
 * with a stride of `stride` bytes (rank order). */
fq_status fq_engine_execute_final(fq_engine *e, const char *sql, const void *states, size_t stride,
                                  int32_t world, fq_result **out);

/* ---- Row pipelines as a stream of device DataBlocks ----
 * SelectExecutor::execute hands its caller the pipeline's SendableDataBlockStream
 * (executor_select.rs:35-40, stream.rs:8-9); for Filter -> Projection over
 * numbers_mt that stream is one filtered + projected DataBlock per 10,000-row
 * source block (stream_expression.rs:38-50, transform_projection.rs:45-56).
 * fq_engine_execute_blocks returns that stream with the blocks left in HBM:
 * each fq_device_block is one device block of a partition pipe, which holds a
 * run of the reference's blocks in its block-stream layout -- block b's rows
 * are rows [b * block_rows, b * block_rows + d_counts[b]) of every column
 * (fq_filter_project_blocks) -- or plain columns (block_rows = 0: every one of
 * `rows` rows valid; e.g. after a LIMIT, or a projection without a filter).
 * Blocks of one pipe arrive in row order; pipes interleave in arrival order
 * like the reference's MergeProcessor channel (processor_merge.rs:45-63).
 * The block's device memory and the pointers in *out stay valid until the next
 * fq_block_stream_next or fq_block_stream_free on the stream; the device work
 * that produced it is complete when next returns, and the caller's own work
 * reading it must be complete before that next call.  Row pipelines only
 * (aggregates: fq_engine_execute, FQ_E_UNSUPPORTED here).                   */
typedef struct fq_block_stream fq_block_stream;
typedef struct fq_device_block {
    int32_t n_columns;
    int32_t pipe;              /* partition pipe (partition order) it came from; a stream
                                  with a single pipe reports 0; -1 only at the end */
    const char *const *names;  /* the plan's output schema                 */
    const fq_col *columns;     /* device columns (len = rows spanned)       */
    int64_t rows;              /* valid rows                                */
    int64_t block_rows;        /* > 0: block-stream layout of n_blocks blocks */
    int64_t n_blocks;
    const int64_t *d_counts;   /* device, n_blocks valid-row counts (NULL when block_rows = 0) */
} fq_device_block;
/* rank of world: the stream covers this rank's numbers_mt partitions
 * [8r/G, 8(r+1)/G) (world 1: all of them), as fq_engine_execute_partial.  */
fq_status fq_engine_execute_blocks(fq_engine *e, const char *sql, int32_t rank, int32_t world,
                                   fq_block_stream **out);
/* *has_block = 0 at the end of the stream (and *out is zeroed) */
fq_status fq_block_stream_next(fq_block_stream *s, fq_device_block *out, int32_t *has_block);
/* Lifetime: a stream's pipes run on its engine's threads and device queues.
 * fq_engine_destroy closes every stream still open (the pipes are stopped and
 * joined, their blocks freed); such a stream's next call fails with
 * FQ_E_INVALID and fq_block_stream_free still releases it.  Calls on one stream
 * or engine must not run concurrently with fq_engine_destroy.               */
void fq_block_stream_free(fq_block_stream *s);

fq_status fq_engine_get_stats(fq_engine *e, fq_engine_stats *out);
fq_status fq_engine_reset_stats(fq_engine *e);

/* A statement whose result is one row (an ungrouped aggregate): its values in
 * one call -- fq_engine_execute, the row's first min(cap, columns) values into
 * row[], *ncols = its columns, the result freed.  Fails with FQ_E_INVALID when
 * the statement returns another number of rows.                             */
fq_status fq_engine_execute_row(fq_engine *e, const char *sql, fq_value *row, int32_t cap, int32_t *ncols);

/* results */
int64_t fq_result_num_rows(const fq_result *r);
int32_t fq_result_num_columns(const fq_result *r);
const char *fq_result_column_name(const fq_result *r, int32_t col);
int32_t fq_result_column_type(const fq_result *r, int32_t col);
fq_status fq_result_value(const fq_result *r, int64_t row, int32_t col, fq_value *out);
/* rows 0..n-1 of one column in one call (n <= fq_result_num_rows) */
fq_status fq_result_values(const fq_result *r, int32_t col, fq_value *out, int64_t n);
/* the value as text, DataValue's Display (NULL for None); valid until fq_result_free */
const char *fq_result_text(const fq_result *r, int64_t row, int32_t col);
/* MySQL column type the reference's result writer declares for a column
 * (MySQLStream::execute, src/servers/mysql/mysql_stream.rs:30-62): integer
 * types -> MYSQL_TYPE_LONG, Float32/64 -> MYSQL_TYPE_FLOAT, Utf8 ->
 * MYSQL_TYPE_VARCHAR; anything else fails with "Internal Error: Unsupported
 * column type:<DataType>".  Row values are fq_result_text (arrow
 * array_value_to_string), column names fq_result_column_name.              */
#define FQ_MYSQL_TYPE_LONG 3
#define FQ_MYSQL_TYPE_FLOAT 4
#define FQ_MYSQL_TYPE_VARCHAR 15
fq_status fq_result_mysql_type(const fq_result *r, int32_t col, int32_t *out);
void fq_result_free(fq_result *r);

/* ---- Function handles: the reference's expression/aggregate trait surface ----
 * A Rust host that keeps its own transforms binds these in place of its
 * `Function` enum (src/functions/function.rs:28-131); the engine's
 * AggregatePartial/AggregateFinal run the same C++ objects.
 *
 *   fq_function_field        FieldFunction::try_create        function_field.rs:20-25
 *   fq_function_constant     ConstantFunction::try_create     function_constant.rs:20-24
 *   fq_function_create       ScalarFunctionFactory::get       function_factory.rs:14-40
 *                            (+ - * / = < > <= >= and or; the aggregators
 *                             count min max sum, AggregatorFunction::try_create
 *                             function_aggregator.rs:24-36)
 *   fq_function_clone        #[derive(Clone)] (deep: the aggregate state too)
 *   fq_function_display      fmt::Debug of Function             function.rs:134-146
 *   fq_function_return_type / nullable / set_depth / eval / accumulate /
 *   accumulate_result / merge_state / merge_result
 *                            Function::*                        function.rs:28-131
 *
 * Blocks are the caller's device columns (Arrow PrimitiveArray value buffers,
 * Boolean as LSB-first bitmap words), borrowed for the call.  eval and
 * accumulate run on the engine's GPU; the state protocol (accumulate_result,
 * merge_state, merge_result) is host work, as in the reference, and also works
 * on a host-only engine.                                                     */
typedef struct fq_function fq_function;

typedef struct fq_block {
    int32_t n_columns;
    const char *const *names; /* DataSchema field names                       */
    const fq_col *columns;    /* device columns of equal len                  */
    /* The reference's block geometry: > 0 -- the columns hold ceil(len /
     * block_rows) of its blocks, block_rows rows each but the last
     * (NumbersStream's 10,000, numbers_stream.rs:29), and accumulate replays
     * the per-block state machine of function_aggregator.rs:57-100 over them
     * (a Sum that meets an empty block after >= 2 blocks fails as the
     * reference does); 0 -- the columns are ONE block.  One call can then
     * stand for a whole partition instead of 125,000 calls.                 */
    int64_t block_rows;
    /* A pending FilterTransform (transform_filter.rs:38-55) or NULL: a Boolean
     * Function handle (a comparison, or an and/or tree of them) over these
     * columns; the block holds only the rows where it is true, each reference
     * block filtered on its own (ExpressionStream, stream_expression.rs:38-50).
     * accumulate fuses it into the scan; eval evaluates the kept rows.       */
    const fq_function *filter;
} fq_block;

/* A DataValue of any type (data_value.rs:20-38), Utf8 included.
 * kind: FQ_SCALAR_NULL = DataValue::Null, FQ_SCALAR_NONE = X(None),
 * FQ_SCALAR_SOME = X(Some(v)); numeric/Boolean payloads in `bits` (fq_value
 * encoding), Utf8 in str/str_len.  Scalars the library returns point into
 * thread-local storage valid until the thread's next call that returns one. */
#define FQ_SCALAR_NULL 0
#define FQ_SCALAR_NONE 1
#define FQ_SCALAR_SOME 2
typedef struct fq_scalar {
    int32_t kind;
    int32_t dtype;
    uint64_t bits;
    const char *str;
    uint64_t str_len;
} fq_scalar;

fq_status fq_function_field(const char *name, fq_function **out);
fq_status fq_function_constant(const fq_scalar *value, fq_function **out);
/* name: an operator or function name as the factory resolves it
 * (case-insensitive); args are cloned, the caller keeps its handles.
 * Errors as the reference: "Internal Error: Unsupported Function: <name>";
 * '%' resolves too (the FQ_OP_MOD extension, FQ_OPT_MODULO's default).    */
fq_status fq_function_create(const char *name, fq_function *const *args, int32_t n_args, fq_function **out);
fq_status fq_function_clone(const fq_function *f, fq_function **out);
void fq_function_free(fq_function *f);
/* NUL-terminated display text; *len = its length (needed cap = len + 1)     */
fq_status fq_function_display(const fq_function *f, char *buf, size_t cap, size_t *len);
fq_status fq_function_set_depth(fq_function *f, uint64_t depth);
/* schema = the block's names with its columns' dtypes (nullable false)     */
fq_status fq_function_return_type(const fq_function *f, const fq_block *schema, int32_t *out);
fq_status fq_function_nullable(const fq_function *f, const fq_block *schema, int32_t *out);
/* DataColumnarValue result: an array is copied into d_out (device memory of
 * `cap` bytes; the needed size is reported in *out_bytes, FQ_E_INVALID when
 * cap is short), *is_array = 1, *out_dtype and *out_len describe it; a scalar
 * result sets *is_array = 0 and *scalar.  Work runs on the engine's queue
 * and is complete when the call returns.                                    */
fq_status fq_function_eval(fq_engine *e, fq_function *f, const fq_block *b, void *d_out, size_t cap,
                           size_t *out_bytes, int32_t *out_dtype, int64_t *out_len, int32_t *is_array,
                           fq_scalar *scalar);
fq_status fq_function_accumulate(fq_engine *e, fq_function *f, const fq_block *b);
/* AggregatePartialTransform's loop body for one block
 * (transform_aggregate_partial.rs:53-58: `for func in funcs { func.accumulate(&block) }`)
 * over n handles at once: the aggregator leaves of all n functions that share
 * an argument expression (and the block's filter) are served by ONE fused scan
 * of the column -- C3's sum/count, max and min by one read instead of four --
 * and the states are replayed in the reference's (block, function) order, so
 * every handle ends in the state n fq_function_accumulate calls leave.  The
 * first failing function's error is returned (the reference's `?`); the
 * functions before it have accumulated.  Complete when the call returns.   */
fq_status fq_functions_accumulate(fq_engine *e, fq_function *const *fs, int32_t n, const fq_block *b);
/* states: the function's partial state vector (aggregates in depth order);
 * *n = its length (FQ_E_INVALID when cap is short, *n = the size needed)   */
fq_status fq_function_accumulate_result(const fq_function *f, fq_scalar *states, size_t cap, size_t *n);
fq_status fq_function_merge_state(fq_function *f, const fq_scalar *states, size_t n);
fq_status fq_function_merge_result(const fq_function *f, fq_scalar *out);

/* Scalar DataValue ops (the merge arithmetic of AggregateFinal):
 *   fq_data_value_arithmetic_op   data_value_arithmetic.rs:10-27 (op FQ_OP_*)
 *   fq_data_value_aggregate_op    data_value_aggregate.rs:8-101  (agg FQ_AGG_*)
 * Errors carry the reference's texts, e.g. "Internal Error: Unsupported
 * data_value_sum for data type: left:Utf8, right:Int8".                    */
fq_status fq_data_value_arithmetic_op(int32_t op, const fq_scalar *l, const fq_scalar *r, fq_scalar *out);
fq_status fq_data_value_aggregate_op(uint32_t agg, const fq_scalar *l, const fq_scalar *r, fq_scalar *out);

#ifdef __cplusplus
}
#endif

#endif /* FQ_ENGINE_H */
