// Cross-GPU AggregateFinal exchange (include/fq_comm.h): the state
// all-gather-by-all-reduce protocol over a caller-supplied collective, and the
// RCCL communicator that supplies it natively (one process per GPU, xGMI).
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "fq_comm.h"
#include "fq_common.h"

struct fq_comm {
    ncclComm_t nccl = nullptr;
    int device = 0, rank = 0, world = 1;
    hipStream_t stream = nullptr;
    uint64_t *d_buf = nullptr;  // device staging for fq_comm_allreduce_u64
    uint64_t *h_buf = nullptr;  // pinned host staging
    int64_t cap_words = 0;
    int64_t timeout_ms = FQ_COMM_TIMEOUT_MS;  // fq_comm_set_timeout
    bool aborted = false;                    // ncclCommAbort ran: every later call fails
    std::string abort_reason;
};

// engine/capi_engine.cpp
void fq_engine_note_exchange(fq_engine *e, int64_t ns, uint64_t rounds, uint64_t bytes);
extern "C" fq_status fq_result_take_row(fq_result *r, fq_value *row, int32_t cap, int32_t *ncols, const char *what);

namespace {

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// ncclCommAbort, once: the communicator is unusable afterwards (its collective
// kernels stopped, its staging buffers possibly half written)
fq_status fq_comm_abort_reason(fq_comm *c, const std::string &why) {
    if (!c->aborted) {
        c->aborted = true;
        c->abort_reason = "rank " + std::to_string(c->rank) + " of " + std::to_string(c->world) + ": " + why;
        (void)ncclCommAbort(c->nccl);
        c->nccl = nullptr;
    }
    return fqc::fail(FQ_E_RCCL, c->abort_reason);
}

// first bytes of an exchanged row that carries a rank's error instead of its
// partial states (those start with "FQS1", pipeline.cpp encode_states)
constexpr char kErrMagic[5] = "FQE1";

fq_status nccl_fail(ncclResult_t r, const char *what) {
    return fqc::fail(FQ_E_RCCL, std::string("RCCL error: ") + what + ": " + ncclGetErrorString(r));
}

#define FQ_NCCL_TRY(expr)                                        \
    do {                                                         \
        ncclResult_t fq_r_ = (expr);                             \
        if (fq_r_ != ncclSuccess) return nccl_fail(fq_r_, #expr); \
    } while (0)

// The communicator is non-blocking (ncclCommInitRankConfig, blocking = 0):
// every RCCL step returns at once and this loop waits for it -- `done` true --
// while watching the communicator's asynchronous error and a deadline.  A
// peer that crashed, or never reaches the collective, would otherwise leave
// this rank spinning in it for ever (the reference's merge sees a failed
// task's Err on its channel instead, processor_merge.rs:50-54): past the
// deadline, or on an RCCL error, the communicator is aborted (ncclCommAbort
// also stops this rank's collective kernel) and the call fails with the rank
// and the step named.
template <class Done>
fq_status comm_wait(fq_comm *c, const char *what, Done done) {
    const int64_t t0 = now_ns();
    const int64_t limit = c->timeout_ms * 1000000;
    for (int spin = 0;; ++spin) {
        const int d = done();  // 1 done, 0 not yet, -1 failed (message set)
        if (d > 0) return FQ_OK;
        if (d < 0) return fq_comm_abort_reason(c, fq_last_error());
        ncclResult_t ae = ncclSuccess;
        const ncclResult_t qr = ncclCommGetAsyncError(c->nccl, &ae);
        if (qr != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress))
            return fq_comm_abort_reason(c, std::string("RCCL error: ") + what + ": " +
                                               ncclGetErrorString(qr != ncclSuccess ? qr : ae));
        if (now_ns() - t0 > limit)
            return fq_comm_abort_reason(c, std::string(what) + " did not complete within " + std::to_string(c->timeout_ms) +
                                               " ms: a peer rank failed or never reached it");
        if (spin < 4096) {
            __builtin_ia32_pause();
        } else {
            std::this_thread::sleep_for(std::chrono::microseconds(spin < 65536 ? 5 : 200));
        }
    }
}

// fq_engine_execute_partial into a growing buffer.
fq_status run_partial(fq_engine *e, const char *sql, int32_t rank, int32_t world, std::vector<uint8_t> &out) {
    size_t len = 0;
    out.resize(std::max<size_t>(out.size(), FQ_EXCHANGE_CAP_BYTES));
    for (;;) {
        fq_status st = fq_engine_execute_partial(e, sql, rank, world, out.data(), out.size(), &len);
        if (st == FQ_E_INVALID && len > out.size()) {
            out.resize(len);
            continue;
        }
        if (st != FQ_OK) return st;
        out.resize(len);
        return FQ_OK;
    }
}

// One all-reduce of a [world x row_words] buffer in which this rank filled its row.
// rounds and bytes of this thread's last exchange (fq_engine_note_exchange)
thread_local uint64_t t_rounds = 0, t_bytes = 0;

fq_status exchange_round(std::vector<uint64_t> &buf, fq_allreduce_fn allreduce, void *user) {
    t_rounds++;
    t_bytes += buf.size() * 8;
    fqc::fail(FQ_OK, "");  // a callback that fails without a message gets the generic one
    fq_status st = allreduce(buf.data(), (int64_t)buf.size(), user);
    if (st != FQ_OK && fq_last_error()[0] == '\0') return fqc::fail(st, "state exchange: all-reduce failed");
    return st;
}

}  // namespace

extern "C" {

fq_status fq_exchange_fail(fq_status st, const char *msg) {
    if (st == FQ_OK) return FQ_OK;
    return fqc::fail(st, msg ? msg : "state exchange: all-reduce failed");
}

fq_status fq_exchange_states_sized(const void *local, size_t len, size_t cap, int32_t rank, int32_t world,
                                   fq_allreduce_fn allreduce, void *user, const void **rows, size_t *stride) {
    if ((!local && len) || !allreduce || !rows || !stride) return fqc::fail(FQ_E_INVALID, "fq_exchange_states: NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return fqc::fail(FQ_E_INVALID, "bad rank/world");
    thread_local std::vector<uint8_t> states;
    t_rounds = 0;
    t_bytes = 0;
    fq_status st;

    // Round 1: [length, first `cap` bytes] per rank.
    const int64_t cap_words = (int64_t)((cap + 7) / 8);
    const int64_t row1 = 1 + cap_words;
    std::vector<uint64_t> buf((size_t)(world * row1), 0);
    buf[(size_t)(rank * row1)] = len;
    if (len) memcpy(&buf[(size_t)(rank * row1 + 1)], local, std::min<size_t>(len, (size_t)cap_words * 8));
    if ((st = exchange_round(buf, allreduce, user)) != FQ_OK) return st;

    uint64_t max_len = 0;
    for (int32_t r = 0; r < world; ++r) max_len = std::max<uint64_t>(max_len, buf[(size_t)(r * row1)]);
    if (max_len <= (uint64_t)cap_words * 8) {
        *stride = (size_t)cap_words * 8;
        states.resize((size_t)world * *stride);
        for (int32_t r = 0; r < world; ++r)
            if (*stride) memcpy(&states[(size_t)r * *stride], &buf[(size_t)(r * row1 + 1)], *stride);
    } else {
        // Round 2: every rank saw the same lengths, so every rank takes it.
        const int64_t row2 = (int64_t)((max_len + 7) / 8);
        std::vector<uint64_t> buf2((size_t)(world * row2), 0);
        memcpy(&buf2[(size_t)(rank * row2)], local, len);
        if ((st = exchange_round(buf2, allreduce, user)) != FQ_OK) return st;
        *stride = (size_t)row2 * 8;
        states.resize(buf2.size() * 8);
        memcpy(states.data(), buf2.data(), states.size());
    }
    *rows = states.data();
    return FQ_OK;
}

fq_status fq_exchange_states(const void *local, size_t len, int32_t rank, int32_t world, fq_allreduce_fn allreduce,
                             void *user, const void **rows, size_t *stride) {
    return fq_exchange_states_sized(local, len, FQ_EXCHANGE_CAP_BYTES, rank, world, allreduce, user, rows, stride);
}

fq_status fq_engine_execute_exchange(fq_engine *e, const char *sql, int32_t rank, int32_t world,
                                     fq_allreduce_fn allreduce, void *user, fq_result **out) {
    if (!e || !sql || !allreduce || !out) return fqc::fail(FQ_E_INVALID, "fq_engine_execute_exchange: NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return fqc::fail(FQ_E_INVALID, "bad rank/world");
    *out = nullptr;
    thread_local std::vector<uint8_t> local;
    fq_status st = run_partial(e, sql, rank, world, local);
    if (st != FQ_OK) {
        // A rank whose partitions fail still takes part in the exchange (the
        // others would wait in the collective forever): it ships an error
        // record instead of states, and every rank reports the error of the
        // lowest failing rank -- the earliest partitions, as on one GPU.
        const std::string msg = fq_last_error();
        local.assign(kErrMagic, kErrMagic + 4);
        const int32_t code = st;
        local.insert(local.end(), (const uint8_t *)&code, (const uint8_t *)&code + 4);
        local.insert(local.end(), msg.begin(), msg.begin() + (long)std::min<size_t>(msg.size(), FQ_EXCHANGE_CAP_BYTES - 16));
    }
    // Round 1 sized to the states: an ungrouped aggregate's are the same size on
    // every rank (fq_engine_partial_state_bytes, a function of the SQL alone), so
    // one all-reduce of world x (8 + that) bytes carries them; GROUP BY rows
    // (data-dependent) send lengths first.  Planning is deterministic, so a
    // statement that fails to plan falls back to the same cap on every rank.
    size_t cap = 0;
    // 0 = data-dependent (GROUP BY rows): the default cap, so a small result
    // still takes ONE round and only a large one a second
    if (fq_engine_partial_state_bytes(e, sql, &cap) != FQ_OK || cap == 0) cap = FQ_EXCHANGE_CAP_BYTES;
    const void *rows = nullptr;
    size_t stride = 0;
    const int64_t t0 = now_ns();
    fq_status xs = fq_exchange_states_sized(local.data(), local.size(), cap, rank, world, allreduce, user, &rows, &stride);
    fq_engine_note_exchange(e, now_ns() - t0, t_rounds, t_bytes);
    if (xs != FQ_OK) return xs;
    for (int32_t r = 0; r < world; ++r) {
        const uint8_t *row = (const uint8_t *)rows + (size_t)r * stride;
        if (stride >= 8 && memcmp(row, kErrMagic, 4) == 0) {
            int32_t code;
            memcpy(&code, row + 4, 4);
            const char *m = (const char *)row + 8;
            return fqc::fail(code, std::string(m, strnlen(m, stride - 8)));
        }
    }
    return fq_engine_execute_final(e, sql, rows, stride, world, out);
}

fq_status fq_comm_unique_id(void *id_out) {
    if (!id_out) return fqc::fail(FQ_E_INVALID, "fq_comm_unique_id: NULL argument");
    static_assert(sizeof(ncclUniqueId) == FQ_COMM_ID_BYTES, "unique id size");
    ncclUniqueId id;
    FQ_NCCL_TRY(ncclGetUniqueId(&id));
    memcpy(id_out, &id, sizeof(id));
    return FQ_OK;
}

fq_status fq_comm_init(int32_t device, int32_t world, int32_t rank, const void *id, fq_comm **out) {
    return fq_comm_init_timeout(device, world, rank, id, FQ_COMM_TIMEOUT_MS, out);
}

fq_status fq_comm_init_timeout(int32_t device, int32_t world, int32_t rank, const void *id, int64_t timeout_ms,
                               fq_comm **out) {
    if (!id || !out) return fqc::fail(FQ_E_INVALID, "fq_comm_init: NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return fqc::fail(FQ_E_INVALID, "bad rank/world");
    if (timeout_ms <= 0) return fqc::fail(FQ_E_INVALID, "fq_comm_init: the timeout must be positive");
    *out = nullptr;
    FQ_HIP_TRY(hipSetDevice(device));
    auto *c = new fq_comm();
    c->device = device;
    c->rank = rank;
    c->world = world;
    c->timeout_ms = timeout_ms;
    hipError_t he = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
        delete c;
        return fqc::hip_fail(he, "hipStreamCreateWithFlags");
    }
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;  // every call returns at once; comm_wait bounds the wait
    ncclResult_t r = ncclCommInitRankConfig(&c->nccl, world, uid, rank, &cfg);
    fq_status st = FQ_OK;
    if (r != ncclSuccess && r != ncclInProgress) {
        st = nccl_fail(r, "ncclCommInitRankConfig");
        if (c->nccl) (void)ncclCommAbort(c->nccl);
        c->nccl = nullptr;
    } else {
        // every rank must arrive: a peer that never does fails this one at the deadline
        st = comm_wait(c, "ncclCommInitRankConfig", [&] {
            ncclResult_t ae = ncclInProgress;
            (void)ncclCommGetAsyncError(c->nccl, &ae);
            return ae == ncclSuccess ? 1 : 0;
        });
    }
    if (st != FQ_OK) {
        const std::string msg = fq_last_error();
        if (c->nccl) (void)ncclCommAbort(c->nccl);
        (void)hipStreamDestroy(c->stream);
        delete c;
        return fqc::fail(st, msg);
    }
    *out = c;
    return FQ_OK;
}

fq_status fq_comm_set_timeout(fq_comm *c, int64_t timeout_ms) {
    if (!c) return fqc::fail(FQ_E_INVALID, "fq_comm_set_timeout: NULL comm");
    if (timeout_ms <= 0) return fqc::fail(FQ_E_INVALID, "fq_comm_set_timeout: the timeout must be positive");
    c->timeout_ms = timeout_ms;
    return FQ_OK;
}

fq_status fq_comm_info(const fq_comm *c, int32_t *rank, int32_t *world) {
    if (!c) return fqc::fail(FQ_E_INVALID, "fq_comm_info: NULL comm");
    if (rank) *rank = c->rank;
    if (world) *world = c->world;
    return FQ_OK;
}

void fq_comm_destroy(fq_comm *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->nccl) {
        // a non-blocking communicator finalizes asynchronously: wait (bounded),
        // else abort -- a peer that is gone must not hold this rank's exit
        ncclResult_t fr = ncclCommFinalize(c->nccl);
        bool ok = fr == ncclSuccess || fr == ncclInProgress;
        const int64_t t0 = now_ns();
        while (ok) {
            ncclResult_t ae = ncclInProgress;
            if (ncclCommGetAsyncError(c->nccl, &ae) != ncclSuccess) ok = false;
            else if (ae == ncclSuccess) break;
            else if (ae != ncclInProgress || now_ns() - t0 > c->timeout_ms * 1000000) ok = false;
            else std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        if (ok) (void)ncclCommDestroy(c->nccl);
        else (void)ncclCommAbort(c->nccl);
    }
    if (c->d_buf) (void)hipFree(c->d_buf);
    if (c->h_buf) (void)hipHostFree(c->h_buf);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

fq_status fq_state_allreduce(fq_comm *c, uint64_t *d_buf, int64_t n_words, void *stream) {
    if (!c || (!d_buf && n_words > 0) || n_words < 0) return fqc::fail(FQ_E_INVALID, "fq_state_allreduce: bad argument");
    if (c->aborted) return fqc::fail(FQ_E_RCCL, c->abort_reason);
    if (n_words == 0) return FQ_OK;
    const ncclResult_t r = ncclAllReduce(d_buf, d_buf, (size_t)n_words, ncclUint64, ncclSum, c->nccl, (hipStream_t)stream);
    if (r == ncclSuccess) return FQ_OK;
    if (r != ncclInProgress) return fq_comm_abort_reason(c, std::string("RCCL error: ncclAllReduce: ") + ncclGetErrorString(r));
    // non-blocking communicator: the enqueue itself completes asynchronously
    return comm_wait(c, "ncclAllReduce (enqueue)", [&] {
        ncclResult_t ae = ncclInProgress;
        (void)ncclCommGetAsyncError(c->nccl, &ae);
        return ae == ncclSuccess ? 1 : 0;
    });
}

fq_status fq_comm_allreduce_u64(uint64_t *buf, int64_t n_words, void *comm) {
    auto *c = (fq_comm *)comm;
    if (!c || (!buf && n_words > 0) || n_words < 0) return fqc::fail(FQ_E_INVALID, "fq_comm_allreduce_u64: bad argument");
    if (c->aborted) return fqc::fail(FQ_E_RCCL, c->abort_reason);
    if (n_words == 0) return FQ_OK;
    FQ_HIP_TRY(hipSetDevice(c->device));
    if (n_words > c->cap_words) {
        if (c->d_buf) FQ_HIP_TRY(hipFree(c->d_buf));
        if (c->h_buf) FQ_HIP_TRY(hipHostFree(c->h_buf));
        c->d_buf = nullptr;
        c->h_buf = nullptr;
        c->cap_words = 0;
        FQ_HIP_TRY(hipMalloc(&c->d_buf, (size_t)n_words * 8));
        FQ_HIP_TRY(hipHostMalloc(&c->h_buf, (size_t)n_words * 8, hipHostMallocDefault));
        c->cap_words = n_words;
    }
    const size_t bytes = (size_t)n_words * 8;
    memcpy(c->h_buf, buf, bytes);
    FQ_HIP_TRY(hipMemcpyAsync(c->d_buf, c->h_buf, bytes, hipMemcpyHostToDevice, c->stream));
    fq_status st = fq_state_allreduce(c, c->d_buf, n_words, c->stream);
    if (st != FQ_OK) return st;
    FQ_HIP_TRY(hipMemcpyAsync(c->h_buf, c->d_buf, bytes, hipMemcpyDeviceToHost, c->stream));
    // the collective waits for every peer: bounded by the deadline
    st = comm_wait(c, "the state all-reduce", [&] {
        const hipError_t q = hipStreamQuery(c->stream);
        if (q == hipSuccess) return 1;
        if (q == hipErrorNotReady) return 0;
        (void)fqc::hip_fail(q, "hipStreamQuery(exchange)");
        return -1;
    });
    if (st != FQ_OK) return st;
    memcpy(buf, c->h_buf, bytes);
    return FQ_OK;
}

fq_status fq_engine_execute_rccl(fq_engine *e, const char *sql, fq_comm *c, fq_result **out) {
    if (!c) return fqc::fail(FQ_E_INVALID, "fq_engine_execute_rccl: NULL comm");
    return fq_engine_execute_exchange(e, sql, c->rank, c->world, fq_comm_allreduce_u64, c, out);
}

fq_status fq_engine_execute_exchange_row(fq_engine *e, const char *sql, int32_t rank, int32_t world,
                                         fq_allreduce_fn allreduce, void *user, fq_value *row, int32_t cap,
                                         int32_t *ncols) {
    if (!ncols || cap < 0 || (cap > 0 && !row))
        return fqc::fail(FQ_E_INVALID, "fq_engine_execute_exchange_row: NULL argument");
    fq_result *r = nullptr;
    const fq_status s = fq_engine_execute_exchange(e, sql, rank, world, allreduce, user, &r);
    if (s != FQ_OK) return s;
    return fq_result_take_row(r, row, cap, ncols, "fq_engine_execute_exchange_row");
}

fq_status fq_engine_execute_rccl_row(fq_engine *e, const char *sql, fq_comm *c, fq_value *row, int32_t cap,
                                     int32_t *ncols) {
    if (!c) return fqc::fail(FQ_E_INVALID, "fq_engine_execute_rccl_row: NULL comm");
    return fq_engine_execute_exchange_row(e, sql, c->rank, c->world, fq_comm_allreduce_u64, c, row, cap, ncols);
}

}  // extern "C"
