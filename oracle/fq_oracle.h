/*
 * fq_oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
 * (dantengsky/fuse-query, Rust) hot path, used as the parity checker and as
 * bench.py's cpu_baseline.  Never linked into or called by the product
 * library (fuse-query_amd/lib/libfq_amd.so).
 *
 * Restates, with the reference's structure kept on purpose (10,000-row blocks
 * regenerated per block, one pass per aggregator, constant broadcast
 * materialised, compaction filter, one thread per partition):
 *   NumbersTable::generate_parts        src/datasources/system/numbers_table.rs:29-55
 *   NumbersStream::create / poll_next   src/datasources/system/numbers_stream.rs:27-83
 *   FilterTransform::expression_executor src/transforms/transform_filter.rs:38-55
 *   data_array_arithmetic_op            src/datavalues/data_array_arithmetic.rs:14-55
 *   data_array_comparison_op            src/datavalues/data_array_comparison.rs:14-94
 *   data_array_aggregate_op             src/datavalues/data_array_aggregate.rs:14-163
 *   data_value_arithmetic_op            src/datavalues/data_value_arithmetic.rs:10-27
 *   data_value_aggregate_op             src/datavalues/data_value_aggregate.rs:8-101
 *   AggregatorFunction::accumulate      src/functions/function_aggregator.rs:57-100
 *   AggregatePartialTransform::execute  src/transforms/transform_aggregate_partial.rs:50-78
 *
 * Parity pinning: checked against the reference's own golden vectors
 * (tests/golden/ JSON fixtures, transcribed from the reference test tables)
 * and the README results; see DESIGN.md "Oracle".
 *
 * Expressions use the fq_expr / fq_pred layouts of include/fq_gpu.h (the
 * oracle only borrows the struct definitions; it does not call the library).
 */
#ifndef FQ_ORACLE_H
#define FQ_ORACLE_H

#include <stdint.h>

#include "fq_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* DataValue state: kind 0 = DataValue::Null, 1 = X(None), 2 = X(Some(bits)) */
#define FQO_NULL 0
#define FQO_NONE 1
#define FQO_SOME 2
typedef struct fqo_state {
    int32_t kind;
    int32_t dtype;
    uint64_t bits;
} fqo_state;

/* column sources */
#define FQO_SRC_NUMBERS 0   /* numbers_mt: value = row number                 */
#define FQO_SRC_SPLITMIX 1  /* value = splitmix64(seed, row number)            */

/* number of partitions generate_parts(total) yields (8, or 1 when total < 8) */
int32_t fqo_num_partitions(uint64_t total);
/* partition p -> first/last row number (inclusive), as in the partition name */
void fqo_partition_range(uint64_t total, int32_t p, uint64_t *begin, uint64_t *end);
/* rows NumbersStream really yields for partition p (the quirk of finding 8) */
uint64_t fqo_partition_rows(uint64_t total, int32_t p);

uint64_t fqo_splitmix64(uint64_t seed, uint64_t i);

/*
 * AggregatePartial over partitions [p0, p1) of numbers_mt(total):
 * out_states[(p - p0) * n_aggs + a] receives aggregator a's partial state for
 * partition p (one SourceTransform per partition, pipeline_builder.rs:73-95).
 * part_status[p - p0] = 0 or an fq_status; the error text of the first
 * failing partition goes to errbuf.  n_threads <= 0: one thread per partition.
 * agg_ops: FQ_AGG_MIN/MAX/SUM/COUNT (single bit each).
 * Returns 0 when every partition succeeded.
 */
int32_t fqo_numbers_partial(uint64_t total, int32_t src, uint64_t seed, int32_t p0, int32_t p1,
                            const fq_pred *pred, int32_t n_aggs, const int32_t *agg_ops,
                            const fq_expr *agg_args, int32_t n_threads, fqo_state *out_states,
                            int32_t *part_status, char *errbuf, int32_t errlen);

/* The same work in 8 * slices tasks (each partition's blocks cut into
 * `slices` runs of whole blocks), n_threads at a time: more parallelism than
 * the reference's 8 fixed partitions allow (the all-cores baseline leg).
 * out_states: [8 * slices][n_aggs]; merging all rows gives the same result. */
int32_t fqo_numbers_partial_split(uint64_t total, const fq_pred *pred, int32_t n_aggs, const int32_t *agg_ops,
                                  const fq_expr *agg_args, int32_t n_threads, int32_t slices,
                                  fqo_state *out_states, char *errbuf, int32_t errlen);

/* Same over an explicit host column cut into blocks of block_rows rows. */
int32_t fqo_column_partial(const void *col, int32_t col_dtype, int64_t len, int64_t block_rows,
                           const fq_pred *pred, int32_t n_aggs, const int32_t *agg_ops,
                           const fq_expr *agg_args, fqo_state *out_states, char *errbuf,
                           int32_t errlen);

/* GROUP BY over numbers_mt(total) (no reference transform; the ungrouped
 * path's semantics per group): per partition thread, per 10,000-row block
 * materialise, filter, key.eval, argument.eval, then one hash-table insert
 * per row; the partition tables merge in partition order.  Writes up to
 * cap_groups (key, n_aggs state bits) rows, unordered; *out_groups = groups.
 * agg_dtypes: the state types (UInt64 / Int64 / Float64).                   */
int32_t fqo_numbers_group(uint64_t total, int32_t src, uint64_t seed, const fq_pred *pred, const fq_expr *key,
                          int32_t n_aggs, const int32_t *agg_ops, const int32_t *agg_dtypes, const fq_expr *agg_args,
                          int32_t n_threads, uint64_t cap_groups, uint64_t *out_keys, uint64_t *out_states,
                          uint64_t *out_groups, char *errbuf, int32_t errlen);

/* FilterTransform -> ProjectionTransform over numbers_mt(total), per
 * 10,000-row block (compaction, then every expression into its own array),
 * one thread per partition; the outputs folded into *out_kept and per-output
 * wrapping sums of the value bits (out_sums[n_out]).                         */
int32_t fqo_numbers_project(uint64_t total, const fq_pred *pred, int32_t n_out, const fq_expr *outs,
                            int32_t n_threads, uint64_t *out_kept, uint64_t *out_sums, char *errbuf, int32_t errlen);

#ifdef __cplusplus
}
#endif

#endif
