// C++ restatement of the reference's data layer for the device engine:
//   FuseQueryError / FuseQueryResult        src/error.rs:10-28
//   DataValue + scalar ops                  src/datavalues/data_value.rs:20-239,
//                                           data_value_arithmetic.rs:10-27,
//                                           data_value_aggregate.rs:8-101
//   DataField / DataSchema                  src/datavalues/data_field.rs, data_schema.rs
//   DataBlock (schema + columns)            src/datablocks/data_block.rs:10-62
//   DataColumnarValue                       src/datavalues/data_columnar_value.rs:8-31
// Columns live in HBM (Arrow layout) or, for small results and aggregate
// states, on the host.  Errors are C++ exceptions carrying the reference's
// display text; the C ABI turns them back into fq_status + fq_last_error().
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fq_gpu.h"

namespace fq {

// steady-clock nanoseconds (host phase timers in RuntimeStats)
inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}


using DataType = int32_t;  // FQ_DT_*
class AggFusion;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
struct FQException : std::exception {
    fq_status status;
    std::string msg;
    FQException(fq_status s, std::string m) : status(s), msg(std::move(m)) {}
    const char *what() const noexcept override { return msg.c_str(); }
};
[[noreturn]] void throw_internal(const std::string &m);  // "Internal Error: " + m
[[noreturn]] void throw_plan(const std::string &m);      // "Error during plan: " + m
[[noreturn]] void throw_status(fq_status st, const std::string &m);
void check_fq(fq_status st);  // rethrows fq_last_error() of a C-ABI call
void check_hip(hipError_t e, const char *what);

const char *dtype_name(DataType dt);
int dtype_size(DataType dt);
bool dtype_is_numeric(DataType dt);
bool dtype_is_float(DataType dt);
bool dtype_is_signed(DataType dt);

// ---------------------------------------------------------------------------
// DataValue
// ---------------------------------------------------------------------------
struct DataValue {
    enum Kind : int32_t { kNull = 0, kNone = 1, kSome = 2, kStruct = 3 };
    int32_t kind = kNull;
    DataType dtype = FQ_DT_NULL;
    uint64_t bits = 0;              // fq_value encoding
    std::string str;                // Utf8 payload
    std::vector<DataValue> fields;  // Struct payload

    static DataValue null() { return DataValue(); }
    static DataValue none(DataType dt) {
        DataValue v;
        v.kind = kNone;
        v.dtype = dt;
        return v;
    }
    static DataValue some(DataType dt, uint64_t b) {
        DataValue v;
        v.kind = kSome;
        v.dtype = dt;
        v.bits = b;
        return v;
    }
    static DataValue u64(uint64_t x) { return some(FQ_DT_UINT64, x); }
    static DataValue string(const std::string &s) {
        DataValue v = some(FQ_DT_UTF8, 0);
        v.str = s;
        return v;
    }
    static DataValue make_struct(std::vector<DataValue> f) {
        DataValue v;
        v.kind = kStruct;
        v.fields = std::move(f);
        return v;
    }
    bool is_untyped_null() const { return kind == kNull; }
    bool is_none() const { return kind == kNone; }  // DataValue::is_null (data_value.rs:40-56)
    DataType data_type() const;                     // data_value.rs:58-75
    std::string debug() const;                      // fmt::Debug (data_value.rs:220-239)
    fq_value to_abi() const;
    static DataValue from_abi(const fq_value &v);
    bool operator==(const DataValue &o) const;
};

std::string format_f64(double d);  // Rust `{}` formatting of an f64

DataValue data_value_arithmetic_op(int32_t op, const DataValue &l, const DataValue &r);
DataValue data_value_aggregate_op(uint32_t agg, const DataValue &l, const DataValue &r);
const char *agg_op_name(uint32_t agg);        // Display: "min", "max", "sum", "count"
const char *agg_op_debug_name(uint32_t agg);  // Debug: "Min", "Max", "Sum", "Count"

// ---------------------------------------------------------------------------
// schema
// ---------------------------------------------------------------------------
struct DataField {
    std::string name;
    DataType dtype = FQ_DT_NULL;
    bool nullable = false;
};

struct DataSchema {
    std::vector<DataField> fields;
    int index_of(const std::string &name) const;  // throws the arrow error text
    const DataField &field_with_name(const std::string &name) const;
};
using SchemaRef = std::shared_ptr<const DataSchema>;

// ---------------------------------------------------------------------------
// device runtime: one per engine; a WorkerRes per executing pipe thread
// ---------------------------------------------------------------------------
struct EngineStats {
    std::atomic<uint64_t> scan_launches{0}, scan_rows{0}, scan_bytes{0}, queries{0};
    std::atomic<uint64_t> scan_ns{0};
    std::atomic<uint64_t> plan_ns{0}, exec_ns{0}, first_launch_ns{0};
    // the distributed split: partial, the exchange (fq_comm.cpp), final
    std::atomic<uint64_t> partial_ns{0}, exchange_ns{0}, final_ns{0};
    std::atomic<uint64_t> exchanges{0}, exchange_rounds{0}, exchange_bytes{0};
    // FilterTransform -> ProjectionTransform over block streams (fq_filter_project_blocks)
    std::atomic<uint64_t> project_launches{0}, project_rows{0}, project_kept{0}, project_bytes{0}, project_ns{0};
    // query start (steady_clock ns) while a query runs; the first scan launch
    // of the query adds (launch - start) to first_launch_ns and clears it
    std::atomic<int64_t> query_t0{0};
    // FQ_OPT_PROFILE 2: when the query's scan group saw its end event
    // (ScanGroup::wait_end); fq_engine_execute adds (exec end - it) to tail_ns
    std::atomic<int64_t> scan_end_seen{0};
    std::atomic<uint64_t> tail_ns{0};
    std::atomic<uint64_t> complete_ns{0};  // of tail_ns: the partitions' states read (DataBlock::complete)
};

struct WorkerRes {
    hipStream_t stream = nullptr;
    hipStream_t own = nullptr;  // private queue for row pipelines (created on first use)
    std::mutex *launch_mu = nullptr;  // serialises multi-call enqueues on a shared queue
    void *ws = nullptr;               // fq_aggregate workspace
    size_t ws_bytes = 0;
    size_t queue_index = 0;           // which shared queue (Runtime::shared_)
    std::vector<hipEvent_t> events;   // reusable events (timing pairs, completion)
    // Pinned, device-visible result slots: the scan's finalize kernel writes
    // its fq_agg_state straight to host memory, so no copy is queued behind
    // the next partition's scan.  Chunks of kSlotChunk, reused across queries.
    static constexpr size_t kSlotChunk = 64;
    std::vector<fq_agg_state *> slot_chunks;
    // this worker's block-stream projection launch (fqk::filter_project_blocks_
    // enqueue; one in flight per worker): {kept rows, flag words} in pinned,
    // device-mapped host memory (project_res, its device address project_dres)
    // and a workspace kept zeroed between launches (project_ws)
    uint64_t *project_res = nullptr, *project_dres = nullptr;
    void *project_ws = nullptr;
    // makes the three on first use; the workspace is zeroed on `st`, the
    // queue of the launch that follows (a non-blocking queue does not wait
    // for a memset on the null stream)
    void project_resident(hipStream_t st);
    hipEvent_t take_event();
    void give_event(hipEvent_t e) { events.push_back(e); }
    // completion-only events (hipEventDisableTiming: no timestamp to write)
    std::vector<hipEvent_t> sync_events;
    hipEvent_t take_sync_event();
    void give_sync_event(hipEvent_t e) { sync_events.push_back(e); }
};

// Persistent host threads for the pipes (the reference spawns tokio tasks per
// query, processor_merge.rs:49); a submitted task never waits for a thread.
// A thread that finished a task polls the queue for FQ_TUNE_POOL_SPIN_US
// before it sleeps: the next query's pipes usually arrive within ~0.1 ms, and
// waking a sleeping thread is tens of microseconds at the head of every query.
class ThreadPool {
   public:
    ~ThreadPool();
    void submit(std::function<void()> task);

   private:
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<std::thread> threads_;
    std::deque<std::function<void()>> queue_;
    std::atomic<size_t> pending_{0};  // queue_.size(), readable without mu_
    std::atomic<bool> stopping_{false};
    size_t idle_ = 0;                 // threads sleeping or polling for a task
    bool stop_ = false;
    void run();
};

class Runtime {
   public:
    static constexpr int kHostOnly = -1;  // no GPU: planning and AggregateFinal merges only
    explicit Runtime(int device);
    bool has_device() const { return device_ != kHostOnly; }
    static constexpr uint64_t kPoolKeepBytes = 8ull << 30;  // default mem pool release threshold
    ~Runtime();
    int device() const { return device_; }
    WorkerRes *acquire();
    void release(WorkerRes *w);
    void set_streams(int n);
    int active_streams() const { return active_streams_; }
    // block-stream row pipelines' queues (QueueKind::kRow): two, measured
    // against one in one process, ms per p1 query (profiles/r06_f_p1_streams_ab.json):
    // 1 queue 23.80, 2 queues 23.07, 4 queues unstable (their cached blocks
    // outgrow the large class); aggregates stay on one (2: C3 11.10 -> 11.71,
    // profiles/r06_g_c3_streams_ab.json)
    static constexpr size_t kRowQueues = 2;
    hipStream_t row_queue(size_t lane, std::mutex **mu);
    // timing-capable events shared across pipe threads (ScanGroup)
    hipEvent_t take_event();
    void give_event(hipEvent_t e);
    EngineStats stats;
    std::atomic<int> profile{0};  // FQ_OPT_PROFILE: 1 event pairs per launch, 2 one span per query
    // GROUP BY table slots for the next query (grows x16 when a query fills
    // its table; the query is then re-run)
    std::atomic<int64_t> group_capacity{4096};
    // slots of the last GROUP BY table sized (a TABLE_FULL re-run grows from it)
    std::atomic<int64_t> group_used_capacity{0};
    // rows per radix-partitioned GROUP BY launch (FQ_OPT_GROUP_CHUNK_ROWS)
    std::atomic<int64_t> group_chunk_rows{500000000};
    // FQ_OPT_FAULT_PIPE (testing): merged pipe k (1-based) fails its context setup
    std::atomic<int64_t> fault_pipe{0};
    ThreadPool pool;

   private:
    int device_;
    std::mutex mu_;
    std::vector<std::unique_ptr<WorkerRes>> all_;
    std::vector<WorkerRes *> free_;
    std::vector<hipStream_t> shared_;  // FQ_OPT_STREAMS queues shared by the pipes
    std::vector<std::unique_ptr<std::mutex>> shared_mu_;
    hipStream_t row_[kRowQueues] = {};
    std::mutex row_mu_[kRowQueues];
    size_t next_shared_ = 0;
    std::atomic<int> active_streams_{1};
    std::vector<hipEvent_t> events_;  // take_event / give_event (under mu_)
};

// Device memory released with hipFreeAsync on the stream that owns it (or
// kept in the engine's stream-ordered block cache, core.cpp, for the next
// allocation of its size class on that stream).
//
// Invariant: a stream-ordered buffer may be read on another queue than its
// allocation queue `stream` only by work queued BEFORE the buffer is dropped
// by a thread whose ExecCtx is bound to that reading queue.  The destructor
// then records an event on the dropping thread's queue and makes `stream`
// wait for it, so the allocation queue's next user of the block (cache reuse
// or pool reuse after hipFreeAsync) is ordered after those reads.  A buffer
// read on a queue that is neither `stream` nor the dropping thread's queue
// must be synchronised by its reader before the last reference goes.
struct DeviceBuffer {
    void *ptr = nullptr;
    size_t bytes = 0;
    hipStream_t stream = nullptr;
    bool async = true;
    bool workspace = false;  // alloc_workspace: kept per queue across queries
    DeviceBuffer() = default;
    DeviceBuffer(const DeviceBuffer &) = delete;
    DeviceBuffer &operator=(const DeviceBuffer &) = delete;
    ~DeviceBuffer();
    static std::shared_ptr<DeviceBuffer> alloc(size_t bytes, hipStream_t st);
    static std::shared_ptr<DeviceBuffer> alloc_sync(size_t bytes);  // long-lived tables
    // A large per-launch workspace: the block cache keeps ONE per queue across
    // queries (outside its block caps; flushed by reclaim_device_memory), so
    // the next query on the queue reuses it (>= bytes; ->bytes is its size)
    static std::shared_ptr<DeviceBuffer> alloc_workspace(size_t bytes, hipStream_t st);
};

// Allocation size class: 256 B minimum, then 4 classes per power of two.
size_t size_class(size_t bytes);
// Flush the block cache, wait for the device, trim the default pool to 0:
// every allocation failure calls it before its one retry; also before large
// long-lived allocations and through fq_engine_trim_memory.
void reclaim_device_memory();
size_t block_cache_bytes();            // cached small blocks
size_t block_cache_workspace_bytes();  // kept per-queue workspaces (counted apart)

// Execution context of the thread running a pipe (tokio task in the
// reference, processor_merge.rs:45-63): its device queue and workspaces.
// Which device queue a context's work goes to:
//   kShared  the worker's shared queue (FQ_OPT_STREAMS of them; aggregates:
//            their HBM-bound scans run back to back)
//   kOwn     the worker's private queue (LIMIT row pipelines synchronise per
//            morsel; a shared queue would make every pipe wait for the others)
//   kRow     row queue `lane % Runtime::kRowQueues` (block-stream row
//            pipelines: one projection launch's tail overlaps the next one's
//            ramp on the other queue)
enum class QueueKind { kShared, kOwn, kRow };

class ExecCtx {
   public:
    explicit ExecCtx(Runtime *rt, QueueKind kind = QueueKind::kShared, size_t lane = 0);
    ~ExecCtx();
    ExecCtx(const ExecCtx &) = delete;
    ExecCtx &operator=(const ExecCtx &) = delete;
    static ExecCtx &current();  // throws when no context is bound on this thread
    static ExecCtx *current_or_null();
    Runtime *rt;
    WorkerRes *res;
    AggFusion *fusion = nullptr;  // set while an AggregatePartial drains its input
    hipStream_t stream() const { return stream_; }
    // serialises multi-call enqueues on this context's queue
    std::mutex *launch_mu() const { return launch_mu_; }
    void sync();
    // hands this context's WorkerRes (queue, workspace, pinned result slots)
    // to a shared owner that releases it to the runtime: work this context
    // enqueued may then be finished on another thread after it is gone
    std::shared_ptr<WorkerRes> lease();

   private:
    ExecCtx *prev_;
    hipStream_t stream_ = nullptr;
    std::mutex *launch_mu_ = nullptr;
    bool leased_ = false;
};

// ---------------------------------------------------------------------------
// columns and blocks
// ---------------------------------------------------------------------------
struct Column {
    DataType dtype = FQ_DT_NULL;
    int64_t len = 0;
    std::shared_ptr<DeviceBuffer> dev;  // device values (or Boolean bitmap words)
    size_t offset = 0;                  // byte offset into dev
    std::shared_ptr<std::vector<DataValue>> host;  // host rows (results, states)
    // host values that are all Some of dtype, as their 64-bit fq_value words
    // (GROUP BY results: 100,000 groups x 4 columns as DataValues cost ~15 ms
    // to build, copy and free); to_host() expands them
    std::shared_ptr<std::vector<uint64_t>> flat;
    // consecutive integers v[0], v[0] + 1, ... (a numbers_mt block; slices keep it)
    bool iota = false;

    bool on_device() const { return (bool)dev; }
    void *dptr() const { return dev ? (char *)dev->ptr + offset : nullptr; }
    fq_col abi() const;
    static Column device(DataType dt, int64_t len, hipStream_t st);  // uninitialised
    static Column host_values(DataType dt, std::vector<DataValue> rows);
    static Column host_flat(DataType dt, std::vector<uint64_t> bits);
    Column slice(int64_t start, int64_t n) const;
    std::vector<DataValue> to_host(hipStream_t st) const;  // synchronous copy
};

class Function;

// Block-stream geometry of a ProjectionTransform output over a numbers stream
// (fq_filter_project_blocks): the columns span n_blocks reference blocks of
// block_rows rows, and block b's rows are the first counts[b] of its range --
// the reference's per-block filtered + projected DataBlocks
// (stream_expression.rs:38-50, transform_projection.rs:45-56) kept where they
// were produced.  materialize() compacts them for consumers that need one
// array (host results, LIMIT); fq_engine_execute_blocks hands them over as is.
struct BlockLayout {
    int64_t block_rows = 0, n_blocks = 0;
    int64_t rows = 0;                     // valid rows over all blocks
    std::shared_ptr<DeviceBuffer> counts;  // int64 per block, HBM
};

struct DataBlock {
    SchemaRef schema;
    std::vector<Column> columns;
    // Reference block granularity this device block stands for: the rows are
    // a run of ceil(n / sub_block_rows) blocks of sub_block_rows rows
    // (NumbersStream 10,000-row blocks kept as one partition-sized device
    // block).  0 = one block.
    int64_t sub_block_rows = 0;
    // FilterTransform output not yet compacted: rows where this predicate is
    // true (the aggregate scan fuses it; other consumers call materialize()).
    std::shared_ptr<Function> filter;
    // set: the columns hold a block stream (see BlockLayout), not one array
    std::shared_ptr<const BlockLayout> layout;
    // the MergeProcessor input (partition pipe) the block came from; -1 unknown
    int32_t pipe = -1;
    // the device work that produced this block has completed (its producer
    // waited for it): the merge need not wait again before handing it over
    bool ready = false;
    // set: the block's columns are not final yet -- the consumer runs this
    // (once, on its own thread) before reading them: AggregatePartial's states
    // once the query's scans have ended (complete_block)
    std::function<void(DataBlock &)> complete;

    int64_t num_rows() const;  // columns[0].len (data_block.rs:46-48); needs no pending filter
    int num_columns() const { return (int)columns.size(); }
    const Column &column_by_name(const std::string &name) const;
    uint64_t sub_blocks() const;  // reference blocks represented (>= 1 if rows > 0)
};

// Compact a block with a pending filter (fq_compare/eval + fq_filter_compact)
// or a block-stream layout (fq_blocks_compact) into plain columns.
DataBlock materialize(const DataBlock &b, ExecCtx &ctx);
// runs and clears b.complete, if set
void complete_block(DataBlock &b);
inline bool needs_materialize(const DataBlock &b) { return b.filter || b.layout; }

// DataColumnarValue
struct ColumnarValue {
    bool is_array = false;
    Column array;
    DataValue scalar;
    DataType data_type() const { return is_array ? array.dtype : scalar.data_type(); }
    Column to_array(int64_t size, ExecCtx &ctx) const;  // data_columnar_value.rs:24-30
};

// DataValue::to_array(size) on the device (fq_fill_value)
Column value_to_array(const DataValue &v, int64_t size, ExecCtx &ctx);

}  // namespace fq
