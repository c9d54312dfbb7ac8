// Cross-GPU AggregateFinal exchange (include/fq_comm.h): the state
// all-gather-by-all-reduce protocol over a caller-supplied collective, and the
// RCCL communicator that supplies it natively (one process per GPU, xGMI).
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
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
};

// engine/capi_engine.cpp
void fq_engine_note_exchange(fq_engine *e, int64_t ns, uint64_t rounds, uint64_t bytes);

namespace {

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
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
    if (!id || !out) return fqc::fail(FQ_E_INVALID, "fq_comm_init: NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return fqc::fail(FQ_E_INVALID, "bad rank/world");
    *out = nullptr;
    FQ_HIP_TRY(hipSetDevice(device));
    auto *c = new fq_comm();
    c->device = device;
    c->rank = rank;
    c->world = world;
    hipError_t he = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
        delete c;
        return fqc::hip_fail(he, "hipStreamCreateWithFlags");
    }
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclResult_t r = ncclCommInitRank(&c->nccl, world, uid, rank);
    if (r != ncclSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return nccl_fail(r, "ncclCommInitRank");
    }
    *out = c;
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
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    if (c->d_buf) (void)hipFree(c->d_buf);
    if (c->h_buf) (void)hipHostFree(c->h_buf);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

fq_status fq_state_allreduce(fq_comm *c, uint64_t *d_buf, int64_t n_words, void *stream) {
    if (!c || (!d_buf && n_words > 0) || n_words < 0) return fqc::fail(FQ_E_INVALID, "fq_state_allreduce: bad argument");
    if (n_words == 0) return FQ_OK;
    FQ_NCCL_TRY(ncclAllReduce(d_buf, d_buf, (size_t)n_words, ncclUint64, ncclSum, c->nccl, (hipStream_t)stream));
    return FQ_OK;
}

fq_status fq_comm_allreduce_u64(uint64_t *buf, int64_t n_words, void *comm) {
    auto *c = (fq_comm *)comm;
    if (!c || (!buf && n_words > 0) || n_words < 0) return fqc::fail(FQ_E_INVALID, "fq_comm_allreduce_u64: bad argument");
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
    FQ_HIP_TRY(hipStreamSynchronize(c->stream));
    memcpy(buf, c->h_buf, bytes);
    return FQ_OK;
}

fq_status fq_engine_execute_rccl(fq_engine *e, const char *sql, fq_comm *c, fq_result **out) {
    if (!c) return fqc::fail(FQ_E_INVALID, "fq_engine_execute_rccl: NULL comm");
    return fq_engine_execute_exchange(e, sql, c->rank, c->world, fq_comm_allreduce_u64, c, out);
}

}  // extern "C"
