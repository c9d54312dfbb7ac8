/*
 * fq_comm.h -- cross-GPU AggregateFinal exchange: RCCL over xGMI, C ABI.
 *
 * The reference has one in-process exchange: every AggregatePartial pipe
 * sends its states as JSON through the MergeProcessor channel and ONE
 * AggregateFinal merges them (processor_merge.rs:37-66,
 * transform_aggregate_partial.rs:61-72, transform_aggregate_final.rs:50-78).
 * Across GPUs each rank owns numbers_mt partitions
 * [8r/G, 8(r+1)/G), runs Source -> Filter -> AggregatePartial on them and the
 * merged partial states of all ranks meet in ONE all-reduce:
 *
 *   every rank writes its serialised states (fq_engine_execute_partial) into
 *   its own row of a zeroed [world x (1 + cap/8)] u64 buffer (word 0 = length)
 *   and a wrapping u64 SUM all-reduce turns that into an all-gather (each word
 *   has exactly one non-zero contributor -> bit-exact).  cap is the states'
 *   size when the SQL fixes it (ungrouped aggregates), else 0.  States longer
 *   than `cap` (GROUP BY states grow with the groups, error records) are sent
 *   in a second all-reduce sized by the lengths every rank now knows, so all
 *   ranks take the same number of collectives.  AggregateFinal then merges in rank order
 *   on every rank (fq_engine_execute_final), so all ranks agree.
 *
 * Host-language neutral: the collective is a callback, so the same protocol
 * runs over RCCL (fq_comm_allreduce_u64) or any other transport (the CPU
 * tests drive it over gloo).  No torch types; the caller owns everything.
 */
#ifndef FQ_COMM_H
#define FQ_COMM_H

#include <stddef.h>
#include <stdint.h>

#include "fq_engine.h"
#include "fq_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* In-place wrapping u64 sum over all ranks of `n_words` words of HOST memory.
 * Returns FQ_OK or an fq_status (message via fq_last_error()).             */
typedef fq_status (*fq_allreduce_fn)(uint64_t *buf, int64_t n_words, void *user);

/* For an fq_allreduce_fn that fails: sets this thread's fq_last_error() text
 * (the exchange runs the callback on the calling thread) and returns st, so
 * the caller of the exchange sees why, e.g. which rank timed out.          */
fq_status fq_exchange_fail(fq_status st, const char *msg);

/* Payload words per rank carried by the first all-reduce (4 KB: an ungrouped
 * query's states are 8 + 16 per value + 8 per function bytes).             */
#define FQ_EXCHANGE_CAP_BYTES 4096

/* The exchange itself: all-gather one byte string per rank (this rank's
 * `local`, `len` bytes) in one all-reduce (two when some rank's string is
 * longer than FQ_EXCHANGE_CAP_BYTES).  *rows receives world rows of *stride
 * bytes in rank order, zero padded; the storage is the library's and stays
 * valid until the next call on this thread.  Collective: every rank calls. */
fq_status fq_exchange_states(const void *local, size_t len, int32_t rank, int32_t world, fq_allreduce_fn allreduce,
                             void *user, const void **rows, size_t *stride);
/* The same with round 1 carrying `cap` payload bytes per rank (rounded up to
 * 8; every rank must pass the same cap).  A string longer than cap on any
 * rank sends every rank through round 2.  cap = 0: round 1 carries only the
 * lengths.  fq_engine_execute_exchange passes fq_engine_partial_state_bytes,
 * so an ungrouped aggregate takes ONE all-reduce of world x (8 + its states)
 * bytes (C3 at world 8: 8 x 104 B) and GROUP BY rows send lengths first.    */
fq_status fq_exchange_states_sized(const void *local, size_t len, size_t cap, int32_t rank, int32_t world,
                                   fq_allreduce_fn allreduce, void *user, const void **rows, size_t *stride);

/* Distributed aggregate query on rank `rank` of `world`: partial on this
 * rank's shard -> exchange through `allreduce` -> AggregateFinal in rank
 * order.  Every rank must call it with the same sql/world.  Covers the
 * queries fq_engine_execute_partial covers (aggregates, GROUP BY).  A rank
 * whose partial fails still takes part in the exchange with an error record
 * ("FQE1", status, message) instead of its states, so no rank waits in the
 * collective; every rank then returns the error of the lowest failing rank. */
fq_status fq_engine_execute_exchange(fq_engine *e, const char *sql, int32_t rank, int32_t world,
                                     fq_allreduce_fn allreduce, void *user, fq_result **out);

/* One-call forms for a statement whose result is one row (an ungrouped
 * aggregate; fq_engine_execute_row's contract): the exchange, then the row's
 * first min(cap, columns) values into row[], *ncols = its columns, the result
 * freed.  Collective like fq_engine_execute_exchange.                      */
fq_status fq_engine_execute_exchange_row(fq_engine *e, const char *sql, int32_t rank, int32_t world,
                                         fq_allreduce_fn allreduce, void *user, fq_value *row, int32_t cap,
                                         int32_t *ncols);

/* ---- RCCL communicator (one process per GPU, non-blocking) ---- */
typedef struct fq_comm fq_comm;
#define FQ_COMM_ID_BYTES 128 /* NCCL_UNIQUE_ID_BYTES */
/* Every RCCL step of a communicator -- its init, each all-reduce -- is
 * bounded: the communicator is non-blocking (ncclCommInitRankConfig,
 * blocking = 0) and the library polls ncclCommGetAsyncError against this
 * deadline.  A peer that crashed or never reaches the collective fails the
 * call with FQ_E_RCCL ("rank r of G: <step> did not complete within T ms: a
 * peer rank failed or never reached it") after ncclCommAbort, instead of a
 * wait without end; every later call on the communicator fails the same way
 * (the reference's merge gets a failed task's Err, processor_merge.rs:50-54). */
#define FQ_COMM_TIMEOUT_MS 60000

/* rank 0 creates the id and ships it to the other ranks (any host channel) */
fq_status fq_comm_unique_id(void *id_out /* FQ_COMM_ID_BYTES */);
/* collective over all `world` ranks; `device` is this rank's HIP ordinal;
 * every rank must arrive within FQ_COMM_TIMEOUT_MS (or timeout_ms)        */
fq_status fq_comm_init(int32_t device, int32_t world, int32_t rank, const void *id, fq_comm **out);
fq_status fq_comm_init_timeout(int32_t device, int32_t world, int32_t rank, const void *id, int64_t timeout_ms,
                               fq_comm **out);
/* the deadline of the communicator's later steps (> 0 ms) */
fq_status fq_comm_set_timeout(fq_comm *c, int64_t timeout_ms);
fq_status fq_comm_info(const fq_comm *c, int32_t *rank, int32_t *world);
/* finalizes (bounded by the deadline, else aborts) and frees */
void fq_comm_destroy(fq_comm *c);

/* SURVEY 8b `fq_state_allreduce`: in-place wrapping u64 SUM all-reduce of a
 * DEVICE buffer on `stream` (one ncclAllReduce, ncclUint64/ncclSum).  Does
 * not synchronise.                                                         */
fq_status fq_state_allreduce(fq_comm *c, uint64_t *d_buf, int64_t n_words, void *stream);

/* An fq_allreduce_fn over `comm` (pass the fq_comm* as `user`): stages the
 * host words through pinned + device buffers the comm owns, one
 * ncclAllReduce on the comm's stream, and waits for it (bounded by the
 * communicator's deadline).                                                */
fq_status fq_comm_allreduce_u64(uint64_t *buf, int64_t n_words, void *comm);

/* fq_engine_execute_exchange over RCCL: rank/world from the comm. */
fq_status fq_engine_execute_rccl(fq_engine *e, const char *sql, fq_comm *c, fq_result **out);
/* the same in one call for a one-row statement (fq_engine_execute_exchange_row) */
fq_status fq_engine_execute_rccl_row(fq_engine *e, const char *sql, fq_comm *c, fq_value *row, int32_t cap,
                                     int32_t *ncols);

#ifdef __cplusplus
}
#endif

#endif /* FQ_COMM_H */
