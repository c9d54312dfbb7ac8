// DataValue semantics, schema, device runtime and columns of the engine.
#include "core.h"

#include <math.h>
#include <stdio.h>
#include <string.h>

#include <map>
#include <unordered_map>

#include "../fq_common.h"

namespace fq {

// ---------------------------------------------------------------------------
// errors / dtypes
// ---------------------------------------------------------------------------
void throw_internal(const std::string &m) { throw FQException(FQ_E_INTERNAL, "Internal Error: " + m); }
void throw_plan(const std::string &m) { throw FQException(FQ_E_PLAN, "Error during plan: " + m); }
void throw_status(fq_status st, const std::string &m) { throw FQException(st, m); }
void check_fq(fq_status st) {
    if (st != FQ_OK) throw FQException(st, fq_last_error());
}
void check_hip(hipError_t e, const char *what) {
    if (e != hipSuccess) {
        (void)hipGetLastError();
        throw FQException(FQ_E_HIP, std::string("HIP error ") + hipGetErrorName(e) + " (" +
                                        hipGetErrorString(e) + ") in " + what);
    }
}

const char *dtype_name(DataType dt) { return fqc::dtype_name(dt); }
int dtype_size(DataType dt) { return fqc::dtype_size(dt); }
bool dtype_is_numeric(DataType dt) { return fqc::dtype_is_numeric(dt); }
bool dtype_is_float(DataType dt) { return fqc::dtype_is_float(dt); }
bool dtype_is_signed(DataType dt) { return fqc::dtype_is_signed_int(dt); }

// ---------------------------------------------------------------------------
// DataValue
// ---------------------------------------------------------------------------
DataType DataValue::data_type() const {
    switch (kind) {
        case kNull: return FQ_DT_NULL;
        case kStruct: throw_internal("not implemented: DataValue::Struct data_type");
        default: return dtype;
    }
}

static double bits_f64(uint64_t b) {
    double d;
    memcpy(&d, &b, 8);
    return d;
}
static uint64_t f64_bits(double d) {
    uint64_t b;
    memcpy(&b, &d, 8);
    return b;
}

// Shortest round-trip digits, then positional notation as Rust's Display.
static std::string format_float(double d, bool is_f32) {
    if (d != d) return "NaN";
    if (isinf(d)) return d > 0 ? "inf" : "-inf";
    if (d == 0) return signbit(d) ? "-0" : "0";
    char buf[64];
    int prec = 1;
    for (; prec <= 17; ++prec) {
        snprintf(buf, sizeof buf, "%.*e", prec - 1, d);
        if (is_f32 ? (float)strtod(buf, nullptr) == (float)d : strtod(buf, nullptr) == d) break;
    }
    // buf = [-]D.DDDDe[+-]XX
    std::string s(buf);
    bool neg = s[0] == '-';
    if (neg) s = s.substr(1);
    const size_t epos = s.find('e');
    std::string mant = s.substr(0, epos);
    const int exp = atoi(s.c_str() + epos + 1);
    std::string digits;
    for (char c : mant)
        if (c != '.') digits += c;
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    std::string out;
    const int n = (int)digits.size();
    if (exp < 0) {
        out = "0." + std::string(-exp - 1, '0') + digits;
    } else if (exp >= n - 1) {
        out = digits + std::string(exp - (n - 1), '0');
    } else {
        out = digits.substr(0, exp + 1) + "." + digits.substr(exp + 1);
    }
    return neg ? "-" + out : out;
}

std::string format_f64(double d) { return format_float(d, false); }

std::string DataValue::debug() const {
    switch (kind) {
        case kNull: return "Null";
        case kNone: return "NULL";
        case kStruct: {
            std::string s = "[";
            for (size_t i = 0; i < fields.size(); ++i) {
                if (i) s += ", ";
                s += fields[i].debug();
            }
            return s + "]";
        }
        default: break;
    }
    if (dtype == FQ_DT_UTF8) return str;
    if (dtype == FQ_DT_BOOLEAN) return bits ? "true" : "false";
    if (dtype == FQ_DT_FLOAT64) return format_float(bits_f64(bits), false);
    if (dtype == FQ_DT_FLOAT32) return format_float(bits_f64(bits), true);
    if (dtype_is_signed(dtype)) return std::to_string((long long)(int64_t)bits);
    return std::to_string((unsigned long long)bits);
}

fq_value DataValue::to_abi() const {
    fq_value v;
    v.dtype = kind == kNull ? FQ_DT_NULL : dtype;
    v.is_some = kind == kSome ? 1 : 0;
    v.bits = kind == kSome ? bits : 0;
    return v;
}

DataValue DataValue::from_abi(const fq_value &v) {
    if (v.dtype == FQ_DT_NULL) return null();
    return v.is_some ? some(v.dtype, v.bits) : none(v.dtype);
}

bool DataValue::operator==(const DataValue &o) const {
    if (kind != o.kind) return false;
    if (kind == kNull) return true;
    if (kind == kStruct) return fields == o.fields;
    if (dtype != o.dtype) return false;
    if (kind == kNone) return true;
    return dtype == FQ_DT_UTF8 ? str == o.str : bits == o.bits;
}

const char *agg_op_name(uint32_t agg) {
    switch (agg) {
        case FQ_AGG_MIN: return "min";
        case FQ_AGG_MAX: return "max";
        case FQ_AGG_SUM: return "sum";
        default: return "count";
    }
}
const char *agg_op_debug_name(uint32_t agg) {
    switch (agg) {
        case FQ_AGG_MIN: return "Min";
        case FQ_AGG_MAX: return "Max";
        case FQ_AGG_SUM: return "Sum";
        default: return "Count";
    }
}

// wrap an integer result into the width of dt (release-build arithmetic)
static uint64_t wrap_int(uint64_t v, DataType dt) {
    const int bits = 8 * dtype_size(dt);
    if (bits >= 64) return v;
    const uint64_t m = (1ull << bits) - 1;
    v &= m;
    if (dtype_is_signed(dt) && (v >> (bits - 1))) v |= ~m;
    return v;
}

static void to_array_check(const DataValue &v) {
    if (v.kind == DataValue::kNone) throw_internal("DataValue to array cannot be NONE NULL");
    if (v.kind == DataValue::kStruct) throw_internal("DataValue to array cannot be NONE " + v.debug());
}

// data_value_arithmetic_op (data_value_arithmetic.rs:10-27): Null absorbs,
// otherwise both scalars go through to_array(1) + data_array_arithmetic_op.
DataValue data_value_arithmetic_op(int32_t op, const DataValue &l, const DataValue &r) {
    if (l.kind == DataValue::kNull) return r;
    if (r.kind == DataValue::kNull) return l;
    to_array_check(l);
    to_array_check(r);
    int32_t ct = 0;
    if (fqc::numerical_coercion(fqc::arith_op_str(op), l.dtype, r.dtype, &ct) != FQ_OK)
        throw FQException(FQ_E_INTERNAL, fq_last_error());
    uint64_t a = 0, b = 0;
    if (!fqc::cast_scalar(l.bits, l.dtype, ct, &a) || !fqc::cast_scalar(r.bits, r.dtype, ct, &b))
        return DataValue::none(ct);  // arrow cast -> null -> op -> null
    if (dtype_is_float(ct)) {
        double x = bits_f64(a), y = bits_f64(b), z = 0;
        if ((op == FQ_OP_DIV || op == FQ_OP_MOD) && y == 0.0)
            throw FQException(FQ_E_DIVIDE_BY_ZERO, "Internal Error: Divide by zero error");
        if (ct == FQ_DT_FLOAT32) {
            const float fx = (float)x, fy = (float)y;
            float fz = op == FQ_OP_ADD ? fx + fy : op == FQ_OP_SUB ? fx - fy : op == FQ_OP_MUL ? fx * fy
                       : op == FQ_OP_DIV ? fx / fy : fmodf(fx, fy);
            z = fz;
        } else {
            z = op == FQ_OP_ADD ? x + y : op == FQ_OP_SUB ? x - y : op == FQ_OP_MUL ? x * y
                : op == FQ_OP_DIV ? x / y : fmod(x, y);
        }
        return DataValue::some(ct, f64_bits(z));
    }
    uint64_t z = 0;
    switch (op) {
        case FQ_OP_ADD: z = a + b; break;
        case FQ_OP_SUB: z = a - b; break;
        case FQ_OP_MUL: z = a * b; break;
        default:
            if (b == 0) throw FQException(FQ_E_DIVIDE_BY_ZERO, "Internal Error: Divide by zero error");
            if (dtype_is_signed(ct)) {
                const int64_t sa = (int64_t)a, sb = (int64_t)b;
                if (sb == -1) z = op == FQ_OP_DIV ? (uint64_t)0 - a : 0;  // overflow wraps (unpinned)
                else z = (uint64_t)(op == FQ_OP_DIV ? sa / sb : sa % sb);
            } else {
                z = op == FQ_OP_DIV ? a / b : a % b;
            }
    }
    return DataValue::some(ct, wrap_int(z, ct));
}

static bool lt_bits(DataType dt, uint64_t a, uint64_t b) {
    if (dtype_is_float(dt)) return bits_f64(a) < bits_f64(b);
    if (dtype_is_signed(dt)) return (int64_t)a < (int64_t)b;
    return a < b;
}

// data_value_aggregate_op (data_value_aggregate.rs:8-101 + macros.rs:168-200)
DataValue data_value_aggregate_op(uint32_t agg, const DataValue &l, const DataValue &r) {
    if (l.kind == DataValue::kNull) return r;
    if (r.kind == DataValue::kNull) return l;
    auto unsupported = [&]() {
        throw_internal(std::string("Unsupported data_value_") + agg_op_name(agg) + " for data type: left:" +
                       dtype_name(l.kind == DataValue::kStruct ? FQ_DT_NULL : l.dtype) + ", right:" +
                       dtype_name(r.kind == DataValue::kStruct ? FQ_DT_NULL : r.dtype));
    };
    if (l.kind == DataValue::kStruct || r.kind == DataValue::kStruct || l.dtype != r.dtype) unsupported();
    const DataType dt = l.dtype;
    if (dt == FQ_DT_UTF8) {
        if (agg != FQ_AGG_MIN && agg != FQ_AGG_MAX) unsupported();
        if (l.kind == DataValue::kNone) return r;
        if (r.kind == DataValue::kNone) return l;
        const bool take_r = agg == FQ_AGG_MAX ? r.str > l.str : r.str < l.str;
        return take_r ? r : l;
    }
    if (!dtype_is_numeric(dt)) unsupported();
    if (agg == FQ_AGG_COUNT) return DataValue::u64(1);
    if (l.kind == DataValue::kNone && r.kind == DataValue::kNone) return DataValue::none(dt);
    if (r.kind == DataValue::kNone) return l;
    if (l.kind == DataValue::kNone) return r;
    if (agg == FQ_AGG_SUM) {
        if (dtype_is_float(dt)) {
            double z = bits_f64(l.bits) + bits_f64(r.bits);
            if (dt == FQ_DT_FLOAT32) z = (float)bits_f64(l.bits) + (float)bits_f64(r.bits);
            return DataValue::some(dt, f64_bits(z));
        }
        return DataValue::some(dt, wrap_int(l.bits + r.bits, dt));
    }
    // f64::min / f64::max ignore NaN; Ord::min/max for integers
    if (dtype_is_float(dt)) {
        const double a = bits_f64(l.bits), b = bits_f64(r.bits);
        if (a != a) return r;
        if (b != b) return l;
    }
    const bool take_r = agg == FQ_AGG_MAX ? lt_bits(dt, l.bits, r.bits) : lt_bits(dt, r.bits, l.bits);
    return take_r ? r : l;
}

// ---------------------------------------------------------------------------
// schema
// ---------------------------------------------------------------------------
int DataSchema::index_of(const std::string &name) const {
    for (size_t i = 0; i < fields.size(); ++i)
        if (fields[i].name == name) return (int)i;
    std::string valid = "[";
    for (size_t i = 0; i < fields.size(); ++i) {
        if (i) valid += ", ";
        valid += "\"" + fields[i].name + "\"";
    }
    valid += "]";
    throw_internal("Invalid argument error: Unable to get field named \"" + name + "\". Valid fields: " + valid);
}

const DataField &DataSchema::field_with_name(const std::string &name) const { return fields[index_of(name)]; }

// ---------------------------------------------------------------------------
// runtime
// ---------------------------------------------------------------------------
// Stream-ordered block cache in front of hipMallocAsync / hipFreeAsync.
// Measured on the README LIMIT query (tools/readme_window.py under rocprofv3
// --hip-runtime-trace): 20-80 us per hipMallocAsync and up to 2.5 ms per
// hipFreeAsync of a morsel buffer -- 5.4 of its 6.6 ms.  A block freed on
// queue S goes to S's free list instead; an allocation on S takes a cached
// block of S of the same size class.  Reuse stays in S's order: the block is
// only handed out again to work queued on S after everything S already holds.
// That is the guarantee hipFreeAsync(ptr, S) + hipMallocAsync(S) give PROVIDED
// every reader of the block ran on S -- DeviceBuffer's destructor makes S wait
// for the dropping thread's queue when that is a different one (a block built
// on a pipe's private queue and read on the consumer's after MergeProcessor);
// see the invariant at DeviceBuffer in core.h.
//
// Sizes are rounded up to classes (4 per power of two, <= 25 % slack) so that
// blocks of one class are interchangeable; blocks above kMaxBlock are never
// cached among them (they would crowd out the frequent small ones), each
// queue keeps at most kStreamBytes and the whole cache kCacheBytes.  Blocks
// above kMaxBlock -- morsels past ~8M rows, a row pipeline's projected
// columns (up to 2.5 GB each, a few dozen per query) -- are kept apart
// (large_cached_, large_cap_ over all queues): mapping them afresh from the
// pool cost ~150 ms per 2.5 GB block on the box
// (profiles/r04_c_prof_p1_timeline.txt), and 0.8 GB blocks that missed the
// small class's 2 GB per-queue cap ran a p1 step at 900 ms instead of 28.  The one
// large workspace a queue may keep is counted apart (ws_cached_, capped at
// ws_cap_ over all queues), so a kept GROUP BY workspace never takes
// the small blocks' room.  Every
// allocation failure -- stream-ordered, hipMalloc or the workspace -- calls
// reclaim_device_memory(): the cache is flushed and the default pool trimmed
// to 0, then the allocation is retried once.
namespace {
class BlockCache {
   public:
    static constexpr size_t kCacheBytes = 6ull << 30;
    static constexpr size_t kStreamBytes = 2ull << 30;
    static constexpr size_t kMaxBlock = 64ull << 20;  // above: the large-block class
    // The two big classes are sized to the device (add_stream reads its HBM):
    // kept blocks above kMaxBlock at most 3/10 of it (96 GB on a 288 GB
    // MI355X), the kept workspaces at most 1/10 (32 GB cap), and a large block
    // is only kept while the device still has max(8 GB, 1/16) of its HBM free,
    // so another allocator in the process (torch, RCCL) keeps room.
    static constexpr size_t kLargeMaxBytes = 96ull << 30;
    static constexpr size_t kWorkspaceMaxBytes = 32ull << 30;
    static BlockCache &get() {
        static BlockCache *c = new BlockCache();  // never destroyed: buffers may outlive statics
        return *c;
    }
    void add_stream(hipStream_t s) {
        if (!fqc::knob(FQ_TUNE_BLOCK_CACHE)) return;  // A/B switch: plain stream-ordered pool
        size_t free_b = 0, total = 0;
        const bool sized = hipMemGetInfo(&free_b, &total) == hipSuccess && total > 0;
        (void)hipGetLastError();
        std::lock_guard<std::mutex> lk(mu_);
        if (sized && !device_total_) {
            device_total_ = total;
            large_cap_ = std::min(kLargeMaxBytes, total / 10 * 3);
            ws_cap_ = std::min(kWorkspaceMaxBytes, total / 10);
            reserve_ = std::max<size_t>(8ull << 30, total / 16);
        }
        free_.emplace(s, Queue());
    }
    // a cached block of s of exactly `bytes` (a size class), or nullptr
    void *take(hipStream_t s, size_t bytes) {
        std::lock_guard<std::mutex> lk(mu_);
        auto f = free_.find(s);
        if (f == free_.end()) return nullptr;
        auto it = f->second.blocks.find(bytes);
        if (it == f->second.blocks.end()) return nullptr;
        void *p = it->second;
        if (bytes > kMaxBlock) {
            large_cached_ -= bytes;
        } else {
            cached_ -= bytes;
            f->second.bytes -= bytes;
        }
        f->second.blocks.erase(it);
        return p;
    }
    // false: not cached (unregistered queue, oversized block or a cap
    // reached), the caller frees
    bool put(hipStream_t s, void *p, size_t bytes) {
        if (bytes > kMaxBlock) {
            // the device's free HBM, read before the lock (a driver call)
            size_t free_b = 0, total = 0;
            const bool known = hipMemGetInfo(&free_b, &total) == hipSuccess;
            (void)hipGetLastError();
            std::lock_guard<std::mutex> lk(mu_);
            auto f = free_.find(s);
            if (f == free_.end() || large_cached_ + bytes > large_cap_ || (known && free_b < reserve_)) return false;
            f->second.blocks.emplace(bytes, p);
            large_cached_ += bytes;
            return true;
        }
        std::lock_guard<std::mutex> lk(mu_);
        auto f = free_.find(s);
        if (f == free_.end() || cached_ + bytes > kCacheBytes || f->second.bytes + bytes > kStreamBytes) return false;
        f->second.blocks.emplace(bytes, p);
        f->second.bytes += bytes;
        cached_ += bytes;
        return true;
    }
    // The queue's one kept workspace (the partitioned GROUP BY's ~4 GB, above
    // kMaxBlock and the queue cap): the next query's launches on the queue take
    // it back instead of mapping it afresh (hipMallocAsync of GBs: up to 540 ms)
    void *take_workspace(hipStream_t s, size_t min_bytes, size_t *bytes) {
        std::lock_guard<std::mutex> lk(mu_);
        auto f = free_.find(s);
        if (f == free_.end() || !f->second.ws || f->second.ws_bytes < min_bytes) return nullptr;
        void *p = f->second.ws;
        *bytes = f->second.ws_bytes;
        ws_cached_ -= f->second.ws_bytes;
        f->second.ws = nullptr;
        f->second.ws_bytes = 0;
        return p;
    }
    bool put_workspace(hipStream_t s, void *p, size_t bytes) {
        std::lock_guard<std::mutex> lk(mu_);
        auto f = free_.find(s);
        if (f == free_.end() || f->second.ws || ws_cached_ + bytes > ws_cap_) return false;
        f->second.ws = p;
        f->second.ws_bytes = bytes;
        ws_cached_ += bytes;
        return true;
    }
    // s is idle and about to be destroyed: free its blocks, stop caching on it
    void drop_stream(hipStream_t s) {
        std::lock_guard<std::mutex> lk(mu_);
        auto f = free_.find(s);
        if (f == free_.end()) return;
        for (auto &b : f->second.blocks) {
            (void)hipFree(b.second);
            (b.first > kMaxBlock ? large_cached_ : cached_) -= b.first;
        }
        if (f->second.ws) {
            (void)hipFree(f->second.ws);
            ws_cached_ -= f->second.ws_bytes;
        }
        free_.erase(f);
    }
    // hand every cached block back to the device pool (in its queue's order)
    void flush() {
        std::lock_guard<std::mutex> lk(mu_);
        for (auto &f : free_) {
            if (f.second.blocks.empty() && !f.second.ws) continue;
            for (auto &b : f.second.blocks) (void)hipFreeAsync(b.second, f.first);
            if (f.second.ws) (void)hipFreeAsync(f.second.ws, f.first);
            f.second.blocks.clear();
            f.second.bytes = 0;
            f.second.ws = nullptr;
            f.second.ws_bytes = 0;
            (void)hipStreamSynchronize(f.first);
        }
        cached_ = 0;
        ws_cached_ = 0;
        large_cached_ = 0;
    }
    size_t cached_bytes() {
        std::lock_guard<std::mutex> lk(mu_);
        return cached_ + large_cached_;
    }
    size_t cached_workspace_bytes() {
        std::lock_guard<std::mutex> lk(mu_);
        return ws_cached_;
    }

   private:
    struct Queue {
        std::multimap<size_t, void *> blocks;
        size_t bytes = 0;
        void *ws = nullptr;  // take_workspace / put_workspace
        size_t ws_bytes = 0;
    };
    std::mutex mu_;
    std::unordered_map<hipStream_t, Queue> free_;
    size_t cached_ = 0;     // small blocks (kCacheBytes / kStreamBytes caps)
    size_t ws_cached_ = 0;  // kept workspaces (ws_cap_)
    size_t large_cached_ = 0;  // blocks above kMaxBlock (large_cap_)
    size_t device_total_ = 0;  // HBM of the device the first queue belongs to
    size_t large_cap_ = 24ull << 30, ws_cap_ = 8ull << 30, reserve_ = 8ull << 30;  // until add_stream sizes them
};

// One reusable ordering event per (thread, device) for cross-queue drops.
hipEvent_t drop_event(int device) {
    thread_local std::unordered_map<int, hipEvent_t> ev;  // leaked at thread exit (HIP may be gone by then)
    auto it = ev.find(device);
    if (it != ev.end()) return it->second;
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    ev.emplace(device, e);
    return e;
}

// hipMalloc-family call with one reclaim-and-retry on failure
template <class F> hipError_t alloc_with_reclaim(F f) {
    hipError_t e = f();
    if (e == hipSuccess) return e;
    (void)hipGetLastError();
    reclaim_device_memory();
    e = f();
    if (e != hipSuccess) (void)hipGetLastError();
    return e;
}
}  // namespace

size_t size_class(size_t bytes) {
    if (bytes <= 256) return 256;
    const int k = 63 - __builtin_clzll((unsigned long long)(bytes - 1));  // 2^k < bytes <= 2^(k+1)
    const size_t step = ((size_t)1 << k) / 4;
    return (bytes + step - 1) / step * step;
}

void reclaim_device_memory() {
    BlockCache::get().flush();
    // every stream-ordered free has to land in the pool before the trim
    (void)hipDeviceSynchronize();
    int dev = 0;
    hipMemPool_t pool;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess)
        (void)hipMemPoolTrimTo(pool, 0);
    (void)hipGetLastError();
}

size_t block_cache_bytes() { return BlockCache::get().cached_bytes(); }
size_t block_cache_workspace_bytes() { return BlockCache::get().cached_workspace_bytes(); }

Runtime::Runtime(int device) : device_(device) {
    if (device == kHostOnly) return;  // planning / AggregateFinal merges only
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= device || device < 0)
        throw FQException(FQ_E_HIP, "fq_engine: no HIP device " + std::to_string(device) +
                                        " (the device path has no CPU fallback)");
    check_hip(hipSetDevice(device), "hipSetDevice");
    // Stream-ordered allocations (columns, workspaces) come from the device's
    // default pool; with its default release threshold of 0 every
    // synchronisation hands the freed memory back to the driver and the next
    // morsel maps it again.  Keep up to kPoolKeepBytes cached.
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
        uint64_t keep = kPoolKeepBytes;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
    (void)hipGetLastError();
    set_streams(1);
}

void Runtime::set_streams(int n) {
    std::lock_guard<std::mutex> lk(mu_);
    if (device_ == kHostOnly) return;
    if (n < 1) n = 1;
    while ((int)shared_.size() < n) {
        hipStream_t s;
        check_hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreateWithFlags");
        BlockCache::get().add_stream(s);
        shared_.push_back(s);
        shared_mu_.push_back(std::make_unique<std::mutex>());
    }
    // new workers pick round-robin among the first n; idle ones are dealt
    // again once every queue has drained (a worker's resident projection
    // workspace is re-zeroed by work on its old queue), so the next query's
    // pipes spread over exactly n queues -- workers in use keep theirs
    (void)hipDeviceSynchronize();
    (void)hipGetLastError();
    // blocks cached on the queues the pipes leave would hold the large
    // class's cap while the new queues map every block afresh
    if (n != active_streams_.load()) reclaim_device_memory();
    next_shared_ = 0;
    active_streams_ = n;
    for (WorkerRes *w : free_) {
        const size_t q = next_shared_++ % (size_t)n;
        w->stream = shared_[q];
        w->launch_mu = shared_mu_[q].get();
        w->queue_index = q;
    }
}

hipStream_t Runtime::row_queue(size_t lane, std::mutex **mu) {
    const size_t q = lane % kRowQueues;
    std::lock_guard<std::mutex> lk(mu_);
    if (!row_[q]) {
        check_hip(hipStreamCreateWithFlags(&row_[q], hipStreamNonBlocking), "hipStreamCreateWithFlags");
        BlockCache::get().add_stream(row_[q]);
    }
    *mu = &row_mu_[q];
    return row_[q];
}

WorkerRes *Runtime::acquire() {
    std::lock_guard<std::mutex> lk(mu_);
    if (!free_.empty()) {
        WorkerRes *w = free_.back();
        free_.pop_back();
        return w;
    }
    auto w = std::make_unique<WorkerRes>();
    if (device_ == kHostOnly) {
        all_.push_back(std::move(w));
        return all_.back().get();
    }
    const size_t q = next_shared_++ % (size_t)active_streams_;
    w->stream = shared_[q];
    w->launch_mu = shared_mu_[q].get();
    w->queue_index = q;
    w->ws_bytes = fq_aggregate_workspace_bytes(0);
    check_hip(alloc_with_reclaim([&] { return hipMalloc(&w->ws, w->ws_bytes); }), "hipMalloc(workspace)");
    all_.push_back(std::move(w));
    return all_.back().get();
}

void Runtime::release(WorkerRes *w) {
    std::lock_guard<std::mutex> lk(mu_);
    free_.push_back(w);
}

hipEvent_t Runtime::take_event() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (!events_.empty()) {
            hipEvent_t e = events_.back();
            events_.pop_back();
            return e;
        }
    }
    hipEvent_t e;
    check_hip(hipEventCreate(&e), "hipEventCreate");
    return e;
}

void Runtime::give_event(hipEvent_t e) {
    if (!e) return;
    std::lock_guard<std::mutex> lk(mu_);
    events_.push_back(e);
}

Runtime::~Runtime() {
    if (device_ == kHostOnly) return;
    (void)hipSetDevice(device_);
    for (auto &s : shared_) (void)hipStreamSynchronize(s);
    for (auto &s : row_)
        if (s) (void)hipStreamSynchronize(s);
    for (auto &w : all_) {
        if (w->own) {
            (void)hipStreamSynchronize(w->own);
            BlockCache::get().drop_stream(w->own);
            (void)hipStreamDestroy(w->own);
        }
        if (w->ws) (void)hipFree(w->ws);
        for (auto ev : w->events) (void)hipEventDestroy(ev);
        for (auto ev : w->sync_events) (void)hipEventDestroy(ev);
        for (auto *c : w->slot_chunks) (void)hipHostFree(c);
        if (w->project_res) (void)hipHostFree(w->project_res);
        if (w->project_ws) (void)hipFree(w->project_ws);
    }
    for (auto ev : events_) (void)hipEventDestroy(ev);
    for (auto &s : shared_) {
        BlockCache::get().drop_stream(s);
        (void)hipStreamDestroy(s);
    }
    for (auto &s : row_)
        if (s) {
            BlockCache::get().drop_stream(s);
            (void)hipStreamDestroy(s);
        }
}

void WorkerRes::project_resident(hipStream_t st) {
    if (project_ws) return;
    void *h = nullptr, *d = nullptr, *ws = nullptr;
    check_hip(hipHostMalloc(&h, 4 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent),
              "hipHostMalloc(projection result)");
    project_res = (uint64_t *)h;
    check_hip(hipHostGetDevicePointer(&d, h, 0), "hipHostGetDevicePointer");
    project_dres = (uint64_t *)d;
    const size_t bytes = fq_filter_project_blocks_workspace_bytes();
    check_hip(alloc_with_reclaim([&] { return hipMalloc(&ws, bytes); }), "hipMalloc(projection workspace)");
    // ordered before this worker's first projection launch on st; the hand-off
    // kernel after every launch keeps it zeroed from then on
    check_hip(hipMemsetAsync(ws, 0, bytes, st), "hipMemsetAsync(projection workspace)");
    project_ws = ws;
}

hipEvent_t WorkerRes::take_sync_event() {
    if (!sync_events.empty()) {
        hipEvent_t e = sync_events.back();
        sync_events.pop_back();
        return e;
    }
    hipEvent_t e;
    check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreateWithFlags");
    return e;
}

hipEvent_t WorkerRes::take_event() {
    if (!events.empty()) {
        hipEvent_t e = events.back();
        events.pop_back();
        return e;
    }
    hipEvent_t e;
    check_hip(hipEventCreate(&e), "hipEventCreate");
    return e;
}

// ---------------------------------------------------------------------------
// thread pool
// ---------------------------------------------------------------------------
void ThreadPool::submit(std::function<void()> task) {
    std::unique_lock<std::mutex> lk(mu_);
    queue_.push_back(std::move(task));
    pending_.store(queue_.size(), std::memory_order_release);
    if (idle_ < queue_.size()) threads_.emplace_back([this] { run(); });  // never wait for a thread
    else cv_.notify_one();
}

void ThreadPool::run() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
        ++idle_;  // polling counts as idle: submit() hands the task to this thread
        const int64_t spin_ns = fqc::knob(FQ_TUNE_POOL_SPIN_US) * 1000;
        if (queue_.empty() && !stop_ && spin_ns > 0) {
            lk.unlock();
            const int64_t until = now_ns() + spin_ns;
            while (pending_.load(std::memory_order_acquire) == 0 && !stopping_.load(std::memory_order_relaxed) &&
                   now_ns() < until) {
                for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
            }
            lk.lock();
        }
        cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
        --idle_;
        if (queue_.empty()) return;  // stop_
        std::function<void()> t = std::move(queue_.front());
        queue_.pop_front();
        pending_.store(queue_.size(), std::memory_order_release);
        lk.unlock();
        t();
        lk.lock();
    }
}

ThreadPool::~ThreadPool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
        stopping_ = true;
    }
    cv_.notify_all();
    for (auto &t : threads_)
        if (t.joinable()) t.join();
}

static thread_local ExecCtx *g_current = nullptr;

DeviceBuffer::~DeviceBuffer() {
    if (!ptr) return;
    if (!async) {
        (void)hipFree(ptr);
        return;
    }
    // Dropped on another queue than the one it was allocated on (a merged
    // block read by the consumer): the allocating queue waits for the
    // dropping thread's queue before the block can be reused or freed there.
    ExecCtx *c = ExecCtx::current_or_null();
    if (c && c->rt->has_device() && c->stream() != stream) {
        hipEvent_t ev = drop_event(c->rt->device());
        if (ev && hipEventRecord(ev, c->stream()) == hipSuccess) (void)hipStreamWaitEvent(stream, ev, 0);
        (void)hipGetLastError();
    }
    const bool kept = workspace ? BlockCache::get().put_workspace(stream, ptr, bytes)
                                : BlockCache::get().put(stream, ptr, bytes);
    if (!kept) (void)hipFreeAsync(ptr, stream);
}

static void require_device() {
    ExecCtx *c = ExecCtx::current_or_null();
    if (c && !c->rt->has_device())
        throw FQException(FQ_E_HIP, "fq_engine: this engine has no device (created with device -1); "
                                    "the hot path has no CPU fallback");
}

std::shared_ptr<DeviceBuffer> DeviceBuffer::alloc(size_t bytes, hipStream_t st) {
    require_device();
    auto b = std::make_shared<DeviceBuffer>();
    b->bytes = size_class(bytes);
    b->stream = st;
    if ((b->ptr = BlockCache::get().take(st, b->bytes))) return b;
    if (alloc_with_reclaim([&] { return hipMallocAsync(&b->ptr, b->bytes, st); }) != hipSuccess) {
        b->ptr = nullptr;
        b->async = false;
        check_hip(alloc_with_reclaim([&] { return hipMalloc(&b->ptr, b->bytes); }), "hipMalloc");
    }
    return b;
}

std::shared_ptr<DeviceBuffer> DeviceBuffer::alloc_workspace(size_t bytes, hipStream_t st) {
    require_device();
    auto b = std::make_shared<DeviceBuffer>();
    b->stream = st;
    b->workspace = true;
    size_t got = 0;
    if ((b->ptr = BlockCache::get().take_workspace(st, bytes, &got))) {
        b->bytes = got;
        return b;
    }
    b->bytes = size_class(bytes);
    if (alloc_with_reclaim([&] { return hipMallocAsync(&b->ptr, b->bytes, st); }) != hipSuccess) {
        b->ptr = nullptr;
        b->async = false;
        check_hip(alloc_with_reclaim([&] { return hipMalloc(&b->ptr, b->bytes); }), "hipMalloc(workspace)");
    }
    return b;
}

std::shared_ptr<DeviceBuffer> DeviceBuffer::alloc_sync(size_t bytes) {
    require_device();
    auto b = std::make_shared<DeviceBuffer>();
    b->bytes = bytes < 256 ? 256 : bytes;
    b->async = false;
    check_hip(alloc_with_reclaim([&] { return hipMalloc(&b->ptr, b->bytes); }), "hipMalloc(table)");
    return b;
}

ExecCtx::ExecCtx(Runtime *r, QueueKind kind, size_t lane) : rt(r), res(nullptr), prev_(g_current) {
    if (rt->has_device()) check_hip(hipSetDevice(rt->device()), "hipSetDevice");
    res = rt->acquire();
    stream_ = res->stream;
    launch_mu_ = res->launch_mu;
    if (kind == QueueKind::kOwn && rt->has_device()) {
        if (!res->own) {
            check_hip(hipStreamCreateWithFlags(&res->own, hipStreamNonBlocking), "hipStreamCreateWithFlags");
            BlockCache::get().add_stream(res->own);
        }
        stream_ = res->own;
    } else if (kind == QueueKind::kRow && rt->has_device()) {
        stream_ = rt->row_queue(lane, &launch_mu_);
    }
    g_current = this;
}

ExecCtx::~ExecCtx() {
    g_current = prev_;
    if (!leased_) rt->release(res);
}

std::shared_ptr<WorkerRes> ExecCtx::lease() {
    if (leased_) throw_internal("ExecCtx::lease: already leased");
    leased_ = true;
    Runtime *r = rt;
    return std::shared_ptr<WorkerRes>(res, [r](WorkerRes *w) { r->release(w); });
}

void complete_block(DataBlock &b) {
    if (!b.complete) return;
    std::function<void(DataBlock &)> f = std::move(b.complete);
    b.complete = nullptr;
    f(b);
}

ExecCtx *ExecCtx::current_or_null() { return g_current; }

ExecCtx &ExecCtx::current() {
    if (!g_current) throw_internal("no device execution context on this thread");
    return *g_current;
}

// Waits for the work enqueued on this context's queue so far.  An event, not
// hipStreamSynchronize: on a queue shared by several pipes the wait must not
// extend to launches other pipes enqueue meanwhile.
void ExecCtx::sync() {
    if (!rt->has_device()) return;
    hipEvent_t ev = res->take_sync_event();
    hipError_t e;
    {
        std::lock_guard<std::mutex> lk(*launch_mu_);
        e = hipEventRecord(ev, stream());
    }
    if (e == hipSuccess) e = hipEventSynchronize(ev);
    res->give_sync_event(ev);
    check_hip(e, "hipEventSynchronize");
}

// ---------------------------------------------------------------------------
// columns / blocks
// ---------------------------------------------------------------------------
static size_t col_bytes(DataType dt, int64_t len) {
    if (dt == FQ_DT_BOOLEAN) return (size_t)((len + 63) / 64) * 8;
    return (size_t)len * (size_t)dtype_size(dt);
}

fq_col Column::abi() const {
    fq_col c;
    c.data = dptr();
    c.len = len;
    c.dtype = dtype;
    c.reserved = 0;
    return c;
}

Column Column::device(DataType dt, int64_t len, hipStream_t st) {
    Column c;
    c.dtype = dt;
    c.len = len;
    c.dev = DeviceBuffer::alloc(col_bytes(dt, len), st);
    return c;
}

Column Column::host_values(DataType dt, std::vector<DataValue> rows) {
    Column c;
    c.dtype = dt;
    c.len = (int64_t)rows.size();
    c.host = std::make_shared<std::vector<DataValue>>(std::move(rows));
    return c;
}

Column Column::host_flat(DataType dt, std::vector<uint64_t> bits) {
    Column c;
    c.dtype = dt;
    c.len = (int64_t)bits.size();
    c.flat = std::make_shared<std::vector<uint64_t>>(std::move(bits));
    return c;
}

Column Column::slice(int64_t start, int64_t n) const {
    Column c = *this;
    if (start < 0) start = 0;
    if (start > len) start = len;
    if (n > len - start) n = len - start;
    c.len = n;
    if (host) {
        c.host = std::make_shared<std::vector<DataValue>>(host->begin() + start, host->begin() + start + n);
    } else if (flat) {
        c.flat = std::make_shared<std::vector<uint64_t>>(flat->begin() + start, flat->begin() + start + n);
    } else if (dev) {
        if (dtype == FQ_DT_BOOLEAN) {
            if (start % 64) throw_internal("bitmap slices must start on a 64-row boundary");
            c.offset = offset + (size_t)(start / 64) * 8;
        } else {
            c.offset = offset + (size_t)start * dtype_size(dtype);
        }
    }
    return c;
}

std::vector<DataValue> Column::to_host(hipStream_t st) const {
    if (host) return *host;
    if (flat) {
        std::vector<DataValue> out;
        out.reserve(flat->size());
        for (uint64_t b : *flat) out.push_back(DataValue::some(dtype, b));
        return out;
    }
    std::vector<DataValue> out;
    if (!dev || len == 0) {
        if (dtype == FQ_DT_NULL) out.assign((size_t)len, DataValue::null());
        return out;
    }
    const size_t nb = col_bytes(dtype, len);
    std::vector<uint8_t> h(nb);
    check_hip(hipMemcpyAsync(h.data(), dptr(), nb, hipMemcpyDeviceToHost, st), "hipMemcpyAsync(D2H)");
    check_hip(hipStreamSynchronize(st), "hipStreamSynchronize");
    out.reserve((size_t)len);
    for (int64_t i = 0; i < len; ++i) {
        uint64_t bits = 0;
        switch (dtype) {
            case FQ_DT_BOOLEAN: bits = (h[(size_t)i / 8] >> (i % 8)) & 1; break;
            case FQ_DT_INT8: bits = (uint64_t)(int64_t)((int8_t *)h.data())[i]; break;
            case FQ_DT_INT16: bits = (uint64_t)(int64_t)((int16_t *)h.data())[i]; break;
            case FQ_DT_INT32: bits = (uint64_t)(int64_t)((int32_t *)h.data())[i]; break;
            case FQ_DT_INT64: bits = (uint64_t)((int64_t *)h.data())[i]; break;
            case FQ_DT_UINT8: bits = ((uint8_t *)h.data())[i]; break;
            case FQ_DT_UINT16: bits = ((uint16_t *)h.data())[i]; break;
            case FQ_DT_UINT32: bits = ((uint32_t *)h.data())[i]; break;
            case FQ_DT_UINT64: bits = ((uint64_t *)h.data())[i]; break;
            case FQ_DT_FLOAT32: bits = f64_bits((double)((float *)h.data())[i]); break;
            case FQ_DT_FLOAT64: bits = ((uint64_t *)h.data())[i]; break;
            default: throw_internal("to_host: unsupported column type");
        }
        out.push_back(DataValue::some(dtype, bits));
    }
    return out;
}

int64_t DataBlock::num_rows() const {
    if (filter) throw_internal("num_rows() of a block with a pending filter");
    if (layout) return layout->rows;
    return columns.empty() ? 0 : columns[0].len;
}

const Column &DataBlock::column_by_name(const std::string &name) const {
    return columns[(size_t)schema->index_of(name)];
}

uint64_t DataBlock::sub_blocks() const {
    const int64_t rows = columns.empty() ? 0 : columns[0].len;
    if (rows == 0 || sub_block_rows <= 0) return 1;
    return (uint64_t)((rows + sub_block_rows - 1) / sub_block_rows);
}

Column value_to_array(const DataValue &v, int64_t size, ExecCtx &ctx) {
    if (v.kind == DataValue::kNull) {  // NullArray::new(size)
        Column c;
        c.dtype = FQ_DT_NULL;
        c.len = size;
        return c;
    }
    to_array_check(v);
    if (v.dtype == FQ_DT_UTF8)
        throw_status(FQ_E_UNSUPPORTED, "Utf8 columns are not supported on the device path");
    Column c = Column::device(v.dtype, size, ctx.stream());
    check_fq(fq_fill_value(c.dptr(), size, v.dtype, v.bits, ctx.stream()));
    return c;
}

Column ColumnarValue::to_array(int64_t size, ExecCtx &ctx) const {
    if (is_array) return array;
    return value_to_array(scalar, size, ctx);
}

}  // namespace fq
