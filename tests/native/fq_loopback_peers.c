/* The peers of one rank of a multi-GPU query, for a one-GPU rehearsal
 * (tools/rank_rehearsal.py) -- test infrastructure, not product.
 *
 * An fq_allreduce_fn that runs the real RCCL all-reduce over the library's
 * world-1 communicator (the same [world x row] buffer a world-G rank sends),
 * then copies this rank's row into every other rank's row: as if the G - 1
 * peers had arrived at once with the same partial states.  Through
 * fq_engine_execute_exchange_row it runs rank R of G's whole step on one GPU:
 * the partial over R's shard, the exchange of G rows, AggregateFinal over G
 * rows -- everything but the wait for slower peers and the xGMI hops. */
#include <stdint.h>
#include <string.h>

#include "fq_comm.h"

typedef struct fq_loopback {
    fq_comm *comm;
    int32_t rank, world;
} fq_loopback;

fq_status fq_loopback_allreduce(uint64_t *buf, int64_t n_words, void *user) {
    const fq_loopback *l = (const fq_loopback *)user;
    fq_status st = fq_comm_allreduce_u64(buf, n_words, l->comm);
    if (st != FQ_OK) return st;
    const int64_t row = n_words / l->world;
    for (int32_t r = 0; r < l->world; ++r)
        if (r != l->rank) memcpy(buf + (size_t)(r * row), buf + (size_t)(l->rank * row), (size_t)row * 8);
    return FQ_OK;
}
