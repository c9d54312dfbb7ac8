// C ABI of the engine (include/fq_engine.h).
#include <string.h>

#include <functional>
#include <iterator>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../fq_common.h"
#include "core.h"
#include "fq_engine.h"
#include "pipeline.h"
#include "planner.h"

// One result column: DataValues, or (flat) the 64-bit words of values that
// are all Some of one type -- GROUP BY results, kept flat from the final to
// fq_result_values
struct ResultCol {
    std::vector<fq::DataValue> v;
    std::vector<uint64_t> flat;
    int32_t flat_dtype = -1;  // >= 0: the column is flat
    bool is_flat() const { return flat_dtype >= 0; }
    size_t size() const { return is_flat() ? flat.size() : v.size(); }
    bool empty() const { return size() == 0; }
    fq::DataValue value(size_t i) const {
        return is_flat() ? fq::DataValue::some((fq::DataType)flat_dtype, flat[i]) : v[i];
    }
    fq_value abi(size_t i) const { return is_flat() ? value(i).to_abi() : v[i].to_abi(); }
    void to_values() {  // a DataValue block joins a flat column
        if (!is_flat()) return;
        v.reserve(flat.size());
        for (uint64_t b : flat) v.push_back(fq::DataValue::some((fq::DataType)flat_dtype, b));
        flat.clear();
        flat_dtype = -1;
    }
    void push_back(fq::DataValue x) {
        to_values();
        v.push_back(std::move(x));
    }
};

struct fq_result {
    std::vector<std::string> names;
    std::vector<int32_t> types;
    std::vector<ResultCol> cols;
    int64_t rows = 0;
    mutable std::vector<std::string> text;  // fq_result_text storage
};

struct fq_block_stream {
    fq_engine *e = nullptr;
    fq::QueryContextRef qctx;
    fq::Pipeline pipeline;
    fq::StreamRef s;
    fq::DataBlock cur;  // the block the caller holds
    std::vector<std::string> names;
    std::vector<const char *> name_ptrs;
    std::vector<fq_col> cols;
};

struct fq_engine {
    std::unique_ptr<fq::Runtime> rt;
    std::shared_ptr<fq::DataSource> ds;
    size_t worker_threads = 8;
    bool modulo = true;
    // Plans of recently seen statements (the reference re-parses every query;
    // a plan is a pure function of the text and the planner options, so a
    // repeated statement skips the parser and PlanBuilder).
    std::mutex plan_mu;
    std::unordered_map<std::string, fq::QueryPlan> plans;
    // Open block streams: their pipes run on this engine's pool, queues and
    // workspaces, so fq_engine_destroy closes them first (see fq_engine.h).
    std::mutex streams_mu;
    std::unordered_set<fq_block_stream *> streams;
};

namespace {
// Stop a block stream's pipes (the merge channel closes, every pipe is joined)
// and drop its device blocks; the stream object stays for fq_block_stream_free.
void close_stream(fq_block_stream *bs) {
    if (!bs->e) return;
    fq::ExecCtx ctx(bs->e->rt.get());
    bs->cur = fq::DataBlock{};
    bs->cols.clear();
    bs->s.reset();
    bs->pipeline = fq::Pipeline{};
    bs->qctx.reset();
}
}  // namespace

// the Function-handle ABI (capi_function.cpp) runs its device calls here
fq::Runtime *fq_engine_runtime(fq_engine *e) { return e->rt.get(); }

// the exchange (fq_comm.cpp) accounts its wall time, rounds and bytes here
void fq_engine_note_exchange(fq_engine *e, int64_t ns, uint64_t rounds, uint64_t bytes) {
    e->rt->stats.exchange_ns += (uint64_t)ns;
    e->rt->stats.exchanges++;
    e->rt->stats.exchange_rounds += rounds;
    e->rt->stats.exchange_bytes += bytes;
}

namespace {

template <typename F>
fq_status guard(F &&f) {
    try {
        f();
        return FQ_OK;
    } catch (const fq::FQException &e) {
        return fqc::fail(e.status, e.msg);
    } catch (const std::exception &e) {
        return fqc::internal(e.what());
    } catch (...) {
        return fqc::internal("unknown exception");
    }
}

// A GROUP BY table ran out of slots: the next attempt gets 16x the slots of
// the table that filled (plan_group_by's sample-based size is the floor).
bool grow_group_table(fq_engine *e, const fq::FQException &ex, int attempt) {
    if (ex.status != FQ_E_TABLE_FULL || attempt >= 4) return false;
    const int64_t used = std::max(e->rt->group_capacity.load(), e->rt->group_used_capacity.load());
    if (used >= ((int64_t)1 << 30)) return false;
    e->rt->group_capacity.store(used * 16);
    return true;
}

// the grown floor lasts for one statement's re-runs only
struct GroupCapacityReset {
    fq_engine *e;
    ~GroupCapacityReset() { e->rt->group_capacity.store(4096); }
};

// host wall time of one call into a stats counter (failed calls count too)
struct PhaseTimer {
    std::atomic<uint64_t> &acc;
    int64_t t0 = fq::now_ns();
    ~PhaseTimer() { acc += (uint64_t)(fq::now_ns() - t0); }
};

fq::QueryContextRef make_ctx(fq_engine *e, int rank, int world) {
    auto c = std::make_shared<fq::QueryContext>();
    c->worker_threads = e->worker_threads;
    c->datasource = e->ds;
    c->factory.modulo = e->modulo;
    c->rt = e->rt.get();
    c->rank = rank;
    c->world = world;
    return c;
}

fq::QueryPlan plan_for(fq_engine *e, const char *sql, const fq::QueryContext &qctx) {
    std::string key(sql);
    key += '\0';
    key += std::to_string(qctx.factory.modulo) + "/" + std::to_string(qctx.worker_threads);
    {
        std::lock_guard<std::mutex> lk(e->plan_mu);
        auto it = e->plans.find(key);
        if (it != e->plans.end()) return it->second;
    }
    fq::QueryPlan plan = fq::build_from_sql(sql, qctx);  // errors are not cached
    fq::optimize(plan);  // mysql_handler.rs:58: every statement is optimised before execution
    std::lock_guard<std::mutex> lk(e->plan_mu);
    if (e->plans.size() >= 256) e->plans.clear();
    e->plans.emplace(std::move(key), plan);
    return plan;
}

// Host rows of the block are moved in when the block holds the only
// reference to them (streams hand their blocks over), else copied.
void append_block(fq_result *r, fq::DataBlock b0, fq::ExecCtx &ctx) {
    fq::DataBlock b = fq::needs_materialize(b0) ? fq::materialize(b0, ctx) : std::move(b0);
    if (r->names.empty()) {
        for (const auto &f : b.schema->fields) {
            r->names.push_back(f.name);
            r->types.push_back(f.dtype);
        }
        r->cols.resize(b.columns.size());
    }
    int64_t n = 0;
    for (size_t c = 0; c < b.columns.size() && c < r->cols.size(); ++c) {
        fq::Column &col = b.columns[c];
        ResultCol &rc = r->cols[c];
        if (col.flat && (rc.empty() || (rc.is_flat() && rc.flat_dtype == col.dtype))) {
            std::vector<uint64_t> f = col.flat.use_count() == 1 ? std::move(*col.flat) : *col.flat;
            n = std::max<int64_t>(n, (int64_t)f.size());
            if (rc.empty()) {
                rc.v.clear();
                rc.flat = std::move(f);
                rc.flat_dtype = col.dtype;
            } else {
                rc.flat.insert(rc.flat.end(), f.begin(), f.end());
            }
            continue;
        }
        std::vector<fq::DataValue> v =
            col.host && col.host.use_count() == 1 ? std::move(*col.host) : col.to_host(ctx.stream());
        if (col.dtype == FQ_DT_NULL && v.empty()) v.assign((size_t)col.len, fq::DataValue::null());
        n = std::max<int64_t>(n, (int64_t)v.size());
        rc.to_values();
        if (rc.v.empty()) rc.v = std::move(v);
        else rc.v.insert(rc.v.end(), std::make_move_iterator(v.begin()), std::make_move_iterator(v.end()));
    }
    r->rows += n;
}

const fq::PlanNode *aggregate_node(const fq::QueryPlan &p) {
    for (const auto &n : p.nodes)
        if (n.kind == fq::PlanNode::kAggregate) return &n;
    return nullptr;
}

}  // namespace

extern "C" {

fq_status fq_engine_create(int32_t device, fq_engine **out) {
    if (!out) return fqc::fail(FQ_E_INVALID, "fq_engine_create: out is NULL");
    *out = nullptr;
    return guard([&] {
        auto e = std::make_unique<fq_engine>();
        e->rt = std::make_unique<fq::Runtime>(device);
        e->ds = std::make_shared<fq::DataSource>();
        *out = e.release();
    });
}

void fq_engine_destroy(fq_engine *e) {
    if (!e) return;
    {
        // streams still open: joined here, while the pool and queues they use
        // exist; they become orphans that only fq_block_stream_free accepts
        std::lock_guard<std::mutex> lk(e->streams_mu);
        for (fq_block_stream *bs : e->streams) {
            try {
                close_stream(bs);
            } catch (...) {
            }
            bs->e = nullptr;
        }
        e->streams.clear();
    }
    if (e->ds) e->ds->numbers()->unpin_all();
    delete e;
}

fq_status fq_engine_set_option(fq_engine *e, int32_t option, int64_t value) {
    if (!e) return fqc::fail(FQ_E_INVALID, "fq_engine_set_option: NULL engine");
    return guard([&] {
        switch (option) {
            case FQ_OPT_WORKER_THREADS: e->worker_threads = (size_t)(value < 0 ? 0 : value); break;
            case FQ_OPT_MODULO: e->modulo = value != 0; break;
            case FQ_OPT_PROFILE:
                if (value < 0 || value > 2) throw fq::FQException(FQ_E_INVALID, "FQ_OPT_PROFILE is 0, 1 or 2");
                e->rt->profile = (int)value;
                break;
            case FQ_OPT_STREAMS: e->rt->set_streams((int)value); break;
            case FQ_OPT_CHUNK_ROWS:
                if (value < 10000 || value % 10000)
                    throw fq::FQException(FQ_E_INVALID, "FQ_OPT_CHUNK_ROWS must be a positive multiple of 10000");
                e->ds->numbers()->set_chunk_rows((uint64_t)value);
                break;
            case FQ_OPT_GROUP_CHUNK_ROWS:
                if (value < 64 || value % 64)
                    throw fq::FQException(FQ_E_INVALID, "FQ_OPT_GROUP_CHUNK_ROWS must be a positive multiple of 64");
                e->rt->group_chunk_rows.store(value);
                break;
            case FQ_OPT_FAULT_PIPE:
                if (value < 0) throw fq::FQException(FQ_E_INVALID, "FQ_OPT_FAULT_PIPE is 0 or a pipe number");
                e->rt->fault_pipe.store(value);
                break;
            default: throw fq::FQException(FQ_E_INVALID, "fq_engine_set_option: unknown option");
        }
    });
}

fq_status fq_engine_materialize_numbers(fq_engine *e, uint64_t total, int32_t rank, int32_t world) {
    if (!e) return fqc::fail(FQ_E_INVALID, "NULL engine");
    if (world < 1 || rank < 0 || rank >= world) return fqc::fail(FQ_E_INVALID, "bad rank/world");
    return guard([&] {
        fq::ExecCtx ctx(e->rt.get());
        // long-lived columns of up to 10 GB each: give the idle cached blocks back first
        fq::reclaim_device_memory();
        auto parts = fq::NumbersTable::generate_parts(total);
        const size_t np = parts.size();
        const size_t lo = np * (size_t)rank / (size_t)world, hi = np * (size_t)(rank + 1) / (size_t)world;
        for (size_t i = lo; i < hi; ++i) {
            uint64_t t, b, en;
            fq::NumbersTable::parse_part(parts[i].name, t, b, en);
            if (en < b) throw fq::FQException(FQ_E_UNSUPPORTED, "numbers_mt(0) is not supported");
            const uint64_t rows = fq::NumbersTable::stream_rows(b, en);
            fq::Column c;
            c.dtype = FQ_DT_UINT64;
            c.len = (int64_t)rows;
            c.dev = fq::DeviceBuffer::alloc_sync(rows * 8);
            fq::check_fq(fq_fill_numbers_u64((uint64_t *)c.dptr(), b, rows, ctx.stream()));
            c.iota = true;
            ctx.sync();
            e->ds->numbers()->pin(parts[i].name, c);
        }
    });
}

fq_status fq_engine_release_numbers(fq_engine *e) {
    if (!e) return fqc::fail(FQ_E_INVALID, "NULL engine");
    return guard([&] { e->ds->numbers()->unpin_all(); });
}

fq_status fq_engine_trim_memory(fq_engine *e) {
    if (!e) return fqc::fail(FQ_E_INVALID, "NULL engine");
    return guard([&] {
        if (!e->rt->has_device()) return;
        fq::check_hip(hipSetDevice(e->rt->device()), "hipSetDevice");
        fq::reclaim_device_memory();
    });
}

fq_status fq_engine_execute(fq_engine *e, const char *sql, fq_result **out) {
    if (!e || !sql || !out) return fqc::fail(FQ_E_INVALID, "fq_engine_execute: NULL argument");
    *out = nullptr;
    return guard([&] {
        fq::ExecCtx ctx(e->rt.get());
        const int64_t t0 = fq::now_ns();
        e->rt->stats.query_t0 = t0;
        auto qctx = make_ctx(e, 0, 1);
        fq::QueryPlan plan = plan_for(e, sql, *qctx);
        auto r = std::make_unique<fq_result>();
        if (plan.explain) {  // ExplainExecutor (executor_explain.rs:38-59)
            fq::Pipeline p = fq::build_pipeline(plan, qctx);
            r->names = {"explain"};
            r->types = {FQ_DT_UTF8};
            r->cols.resize(1);
            r->cols[0].push_back(fq::DataValue::string(plan.display()));
            r->cols[0].push_back(fq::DataValue::string(p.display()));
            r->rows = 2;
        } else {
            GroupCapacityReset reset{e};
            for (int attempt = 0;; ++attempt) {
                fq::Pipeline p = fq::build_pipeline(plan, qctx);
                const int64_t t1 = fq::now_ns();
                e->rt->stats.plan_ns += (uint64_t)(t1 - t0);
                try {
                    fq::StreamRef s = p.execute();
                    fq::DataBlock b;
                    while (s->next(b)) append_block(r.get(), std::move(b), ctx);
                } catch (const fq::FQException &ex) {
                    // a GROUP BY table ran out of slots: re-run with 16x the slots
                    if (!grow_group_table(e, ex, attempt)) throw;
                    r = std::make_unique<fq_result>();
                    continue;
                }
                const int64_t t2 = fq::now_ns();
                e->rt->stats.exec_ns += (uint64_t)(t2 - t1);
                const int64_t seen = e->rt->stats.scan_end_seen.exchange(0);
                if (seen) e->rt->stats.tail_ns += (uint64_t)(t2 - seen);
                break;
            }
            if (r->names.empty())
                for (const auto &f : plan.nodes.back().schema->fields) {
                    r->names.push_back(f.name);
                    r->types.push_back(f.dtype);
                    r->cols.emplace_back();
                }
        }
        e->rt->stats.queries++;
        *out = r.release();
    });
}

fq_status fq_engine_explain(fq_engine *e, const char *sql, char *buf, size_t cap, size_t *len) {
    if (!e || !sql) return fqc::fail(FQ_E_INVALID, "fq_engine_explain: NULL argument");
    return guard([&] {
        fq::ExecCtx ctx(e->rt.get());
        auto qctx = make_ctx(e, 0, 1);
        fq::QueryPlan plan = plan_for(e, sql, *qctx);
        fq::Pipeline p = fq::build_pipeline(plan, qctx);
        const std::string s = plan.display() + "\n" + p.display();
        if (len) *len = s.size();
        if (buf && cap) {
            const size_t n = std::min(cap - 1, s.size());
            memcpy(buf, s.data(), n);
            buf[n] = 0;
        }
    });
}

fq_status fq_engine_execute_partial(fq_engine *e, const char *sql, int32_t rank, int32_t world, void *buf,
                                    size_t cap, size_t *len) {
    if (!e || !sql || !len) return fqc::fail(FQ_E_INVALID, "fq_engine_execute_partial: NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return fqc::fail(FQ_E_INVALID, "bad rank/world");
    PhaseTimer timer{e->rt->stats.partial_ns};
    return guard([&] {
        fq::ExecCtx ctx(e->rt.get());
        auto qctx = make_ctx(e, rank, world);
        fq::QueryPlan plan = plan_for(e, sql, *qctx);
        if (plan.explain || !aggregate_node(plan))
            throw fq::FQException(FQ_E_UNSUPPORTED, "distributed execution covers aggregate queries only");
        fq::QueryPlan partial = plan;
        while (!partial.nodes.empty() && partial.nodes.back().kind == fq::PlanNode::kLimit) partial.nodes.pop_back();
        std::vector<std::vector<fq::DataValue>> per_func;
        GroupCapacityReset reset{e};
        for (int attempt = 0;; ++attempt) {
            per_func.clear();
            try {
                fq::Pipeline p = fq::build_pipeline(partial, qctx, /*emit_states=*/true);
                fq::StreamRef s = p.execute();
                fq::DataBlock b;
                while (s->next(b)) {
                    auto &rows = *b.columns.at(0).host;  // this block is ours: move the rows out
                    per_func.reserve(per_func.size() + rows.size());
                    for (auto &v : rows) per_func.push_back(std::move(v.fields));
                }
            } catch (const fq::FQException &ex) {  // GROUP BY table full: 16x the slots
                if (!grow_group_table(e, ex, attempt)) throw;
                continue;
            }
            break;
        }
        // GROUP BY rows travel as flat arrays when they can (fq::encode_group_rows)
        std::vector<uint8_t> enc;
        if (!aggregate_node(partial)->groups.empty()) enc = fq::encode_group_rows(per_func);
        if (enc.empty()) enc = fq::encode_states(per_func);
        *len = enc.size();
        if (!buf || cap < enc.size())
            throw fq::FQException(FQ_E_INVALID, "fq_engine_execute_partial: buffer too small (need " +
                                                    std::to_string(enc.size()) + " bytes)");
        memcpy(buf, enc.data(), enc.size());
        e->rt->stats.queries++;
    });
}

fq_status fq_engine_execute_blocks(fq_engine *e, const char *sql, int32_t rank, int32_t world, fq_block_stream **out) {
    if (!e || !sql || !out) return fqc::fail(FQ_E_INVALID, "fq_engine_execute_blocks: NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return fqc::fail(FQ_E_INVALID, "bad rank/world");
    *out = nullptr;
    return guard([&] {
        fq::ExecCtx ctx(e->rt.get());
        auto bs = std::make_unique<fq_block_stream>();
        bs->e = e;
        bs->qctx = make_ctx(e, rank, world);
        fq::QueryPlan plan = plan_for(e, sql, *bs->qctx);
        if (plan.explain || aggregate_node(plan))
            throw fq::FQException(FQ_E_UNSUPPORTED, "fq_engine_execute_blocks covers row pipelines (Filter / Projection "
                                                    "/ Limit); aggregates return host rows through fq_engine_execute");
        for (const auto &f : plan.nodes.back().schema->fields) bs->names.push_back(f.name);
        for (const auto &n : bs->names) bs->name_ptrs.push_back(n.c_str());
        bs->pipeline = fq::build_pipeline(plan, bs->qctx);
        bs->s = bs->pipeline.execute();
        e->rt->stats.queries++;
        std::lock_guard<std::mutex> lk(e->streams_mu);
        e->streams.insert(bs.get());
        *out = bs.release();
    });
}

fq_status fq_block_stream_next(fq_block_stream *bs, fq_device_block *out, int32_t *has_block) {
    if (!bs || !out || !has_block) return fqc::fail(FQ_E_INVALID, "fq_block_stream_next: NULL argument");
    *has_block = 0;
    *out = fq_device_block{};
    out->pipe = -1;
    if (!bs->e)
        return fqc::fail(FQ_E_INVALID, "fq_block_stream_next: the stream's engine was destroyed (fq_engine_destroy "
                                       "closes the streams still open)");
    return guard([&] {
        fq::ExecCtx ctx(bs->e->rt.get());
        bs->cur = fq::DataBlock{};  // the caller is done with the previous block
        bs->cols.clear();
        if (!bs->s) return;
        fq::DataBlock b;
        if (!bs->s->next(b)) {
            bs->s.reset();  // the pipes are joined: nothing runs after the end
            return;
        }
        if (b.filter) b = fq::materialize(b, ctx);  // a Filter with no Projection above it
        for (const auto &c : b.columns)
            if (!c.on_device() && c.len > 0)
                throw fq::FQException(FQ_E_UNSUPPORTED, "fq_block_stream_next: a host block in a row pipeline");
        ctx.sync();  // the consumer-side transforms (a LIMIT's compaction) are done too
        bs->cur = std::move(b);
        for (const auto &c : bs->cur.columns) bs->cols.push_back(c.abi());
        out->n_columns = (int32_t)bs->cols.size();
        out->pipe = bs->cur.pipe < 0 ? 0 : bs->cur.pipe;  // no merge channel: the one source pipe
        out->names = bs->name_ptrs.data();
        out->columns = bs->cols.data();
        out->rows = bs->cur.num_rows();
        if (bs->cur.layout) {
            out->block_rows = bs->cur.layout->block_rows;
            out->n_blocks = bs->cur.layout->n_blocks;
            out->d_counts = (const int64_t *)bs->cur.layout->counts->ptr;
        }
        *has_block = 1;
    });
}

void fq_block_stream_free(fq_block_stream *bs) {
    if (!bs) return;
    if (fq_engine *e = bs->e) {
        {
            std::lock_guard<std::mutex> lk(e->streams_mu);
            e->streams.erase(bs);
        }
        try {
            close_stream(bs);  // closes the merge channel and joins the pipes
        } catch (...) {
        }
    }
    delete bs;
}

fq_status fq_engine_partial_state_bytes(fq_engine *e, const char *sql, size_t *bytes) {
    if (!e || !sql || !bytes) return fqc::fail(FQ_E_INVALID, "fq_engine_partial_state_bytes: NULL argument");
    *bytes = 0;
    return guard([&] {
        auto qctx = make_ctx(e, 0, 1);
        fq::QueryPlan plan = plan_for(e, sql, *qctx);
        const fq::PlanNode *agg = aggregate_node(plan);
        if (plan.explain || !agg) throw fq::FQException(FQ_E_UNSUPPORTED, "distributed execution covers aggregate queries only");
        if (!agg->groups.empty()) return;  // one row per group: known only after the scan
        // fresh functions have the state vectors' final shape (Null records are
        // 16 bytes like Some ones), so this is exactly encode_states' length
        std::vector<std::vector<fq::DataValue>> per_func;
        for (const auto &x : agg->exprs) per_func.push_back(x.to_function(qctx->factory)->accumulate_result());
        *bytes = fq::encode_states(per_func).size();
    });
}

}  // extern "C"

namespace {

// The cross-GPU GROUP BY final: every rank's flat rows into one fresh device
// table (sized for all of them), ready for GroupByFinalTransform's extract.
// Empty when there are no rows at all (the host path makes the empty result).
std::shared_ptr<fq::GroupByShared> merge_group_rows_on_device(
    fq_engine *e, const fq::PlanNode &agg, const fq::QueryContext &qctx, int32_t world,
    const std::function<const uint8_t *(int32_t)> &row_ptr, size_t stride, fq::ExecCtx &ctx) {
    (void)e;
    std::vector<fq::AggregatorFunction *> leaves;
    std::vector<fq::FunctionRef> fs;
    for (const auto &x : agg.exprs) fs.push_back(x.to_function(qctx.factory));
    for (auto &f : fs) f->collect_aggregators(leaves);
    const size_t nl = leaves.size();
    std::vector<fq::GroupRows> parts;
    size_t total = 0;
    fq::DataType kdt = FQ_DT_NULL;
    std::vector<fq::DataType> dts(nl, FQ_DT_NULL);
    for (int32_t r = 0; r < world; ++r) {
        parts.push_back(fq::decode_group_rows(row_ptr(r), stride));
        const fq::GroupRows &g = parts.back();
        if (g.keys.empty()) continue;
        if (g.st.size() != nl) throw fq::FQException(FQ_E_INVALID, "GROUP BY: malformed partial state row");
        kdt = g.key_dtype;
        dts = g.dtypes;
        total += g.keys.size();
    }
    if (total == 0) return nullptr;
    if (kdt != FQ_DT_UINT64 && kdt != FQ_DT_INT64) return nullptr;  // the host path reports it
    auto shared = std::make_shared<fq::GroupByShared>();
    fq_group_table &d = shared->desc;
    d = fq_group_table{};
    d.key_dtype = kdt;
    if (nl == 0) {  // keys only: a dummy Count keeps the table valid
        d.n_aggs = 1;
        d.kinds[0] = FQ_AGG_COUNT;
        d.dtypes[0] = FQ_DT_UINT64;
        shared->dummy_count = true;
    } else {
        d.n_aggs = (int32_t)nl;
        for (size_t a = 0; a < nl; ++a) {
            d.kinds[a] = (int32_t)leaves[a]->op();
            d.dtypes[a] = leaves[a]->op() == FQ_AGG_COUNT ? FQ_DT_UINT64 : dts[a];
            shared->leaf_ops.push_back(leaves[a]->op());
        }
    }
    int64_t cap = 64;
    while (cap < (int64_t)(2 * total)) cap <<= 1;
    d.capacity = cap;
    shared->mem = fq::DeviceBuffer::alloc(fq_group_table_bytes(cap, d.n_aggs), ctx.stream());
    d.d_mem = shared->mem->ptr;
    fq::check_fq(fq_group_table_init(&d, ctx.stream()));
    // all ranks' rows back to back: keys[total], then each state array
    const size_t na = (size_t)d.n_aggs;
    std::vector<uint64_t> host(total * (1 + na), 0);
    size_t at = 0;
    for (const fq::GroupRows &g : parts) {
        const size_t n = g.keys.size();
        std::copy(g.keys.begin(), g.keys.end(), host.begin() + (long)at);
        for (size_t a = 0; a < nl; ++a) std::copy(g.st[a].begin(), g.st[a].end(), host.begin() + (long)((1 + a) * total + at));
        at += n;
    }
    auto stage = fq::DeviceBuffer::alloc(host.size() * 8, ctx.stream());
    fq::check_hip(hipMemcpyAsync(stage->ptr, host.data(), host.size() * 8, hipMemcpyHostToDevice, ctx.stream()),
                  "hipMemcpyAsync");
    const uint64_t *dk = (const uint64_t *)stage->ptr;
    const uint64_t *ds[FQ_MAX_GROUP_AGGS] = {};
    for (size_t a = 0; a < na; ++a) ds[a] = dk + (1 + a) * total;
    fq::check_fq(fq_group_table_merge(&d, dk, ds, (int64_t)total, ctx.stream()));
    ctx.sync();  // the staging copy's host vector and the stage buffer go out of scope
    shared->ready = true;
    return shared;
}

}  // namespace

extern "C" {

fq_status fq_engine_execute_final(fq_engine *e, const char *sql, const void *states, size_t stride, int32_t world,
                                  fq_result **out) {
    if (!e || !sql || !states || !out || world < 1) return fqc::fail(FQ_E_INVALID, "fq_engine_execute_final: bad argument");
    *out = nullptr;
    PhaseTimer timer{e->rt->stats.final_ns};
    return guard([&] {
        fq::ExecCtx ctx(e->rt.get());
        auto qctx = make_ctx(e, 0, 1);
        fq::QueryPlan plan = plan_for(e, sql, *qctx);
        const fq::PlanNode *agg = aggregate_node(plan);
        if (plan.explain || !agg) throw fq::FQException(FQ_E_UNSUPPORTED, "distributed execution covers aggregate queries only");
        const bool grouped = !agg->groups.empty();
        auto row_ptr = [&](int32_t r) { return (const uint8_t *)states + (size_t)r * stride; };
        // GROUP BY with every rank's rows as flat arrays and a GPU here: the
        // rows are merged into one device table (fq_group_table_merge) that
        // the final transform then extracts, as after a local GROUP BY
        std::shared_ptr<fq::GroupByShared> merged;
        if (grouped && e->rt->has_device()) {
            bool flat = true;
            for (int32_t r = 0; r < world && flat; ++r) flat = fq::is_group_rows(row_ptr(r), stride);
            if (flat) merged = merge_group_rows_on_device(e, *agg, *qctx, world, row_ptr, stride, ctx);
        }
        std::vector<fq::DataBlock> blocks;
        for (int32_t r = 0; r < world && !merged; ++r) {
            std::vector<fq::DataValue> rows;
            if (fq::is_group_rows(row_ptr(r), stride)) {
                const fq::GroupRows g = fq::decode_group_rows(row_ptr(r), stride);
                for (size_t i = 0; i < g.keys.size(); ++i) {
                    std::vector<fq::DataValue> row;
                    row.push_back(fq::DataValue::some(g.key_dtype, g.keys[i]));
                    for (size_t a = 0; a < g.st.size(); ++a) row.push_back(fq::DataValue::some(g.dtypes[a], g.st[a][i]));
                    rows.push_back(fq::DataValue::make_struct(std::move(row)));
                }
            } else {
                auto per_func = fq::decode_states(row_ptr(r), stride);
                for (auto &v : per_func) rows.push_back(fq::DataValue::make_struct(std::move(v)));
            }
            fq::DataBlock b;
            b.schema = agg->schema;
            b.columns.push_back(fq::Column::host_values(FQ_DT_NULL, std::move(rows)));
            blocks.push_back(std::move(b));
        }
        fq::Pipeline p;
        p.add_source(std::make_shared<fq::BlocksProcessor>(blocks));
        p.add_simple_transform([&]() -> fq::ProcessorRef {
            std::vector<fq::FunctionRef> fs;
            for (const auto &x : agg->exprs) fs.push_back(x.to_function(qctx->factory));
            if (grouped)  // merged on the device, or exchanged groups merged by key on the host
                return std::make_shared<fq::GroupByFinalTransform>(
                    agg->schema, fs, merged ? merged : std::make_shared<fq::GroupByShared>(), false);
            return std::make_shared<fq::AggregateFinalTransform>(agg->schema, fs);
        });
        for (const auto &n : plan.nodes)
            if (n.kind == fq::PlanNode::kLimit) {
                const size_t lim = n.limit;
                p.add_simple_transform([lim]() { return std::make_shared<fq::LimitTransform>(lim); });
            }
        auto r = std::make_unique<fq_result>();
        fq::StreamRef s = p.execute();
        fq::DataBlock b;
        while (s->next(b)) append_block(r.get(), std::move(b), ctx);
        *out = r.release();
    });
}

fq_status fq_engine_get_stats(fq_engine *e, fq_engine_stats *out) {
    if (!e || !out) return fqc::fail(FQ_E_INVALID, "NULL argument");
    out->scan_launches = e->rt->stats.scan_launches.load();
    out->scan_rows = e->rt->stats.scan_rows.load();
    out->scan_bytes = e->rt->stats.scan_bytes.load();
    out->scan_ms = (double)e->rt->stats.scan_ns.load() * 1e-6;
    out->queries = e->rt->stats.queries.load();
    out->plan_ms = (double)e->rt->stats.plan_ns.load() * 1e-6;
    out->exec_ms = (double)e->rt->stats.exec_ns.load() * 1e-6;
    out->first_launch_ms = (double)e->rt->stats.first_launch_ns.load() * 1e-6;
    out->tail_ms = (double)e->rt->stats.tail_ns.load() * 1e-6;
    out->complete_ms = (double)e->rt->stats.complete_ns.load() * 1e-6;
    out->partial_ms = (double)e->rt->stats.partial_ns.load() * 1e-6;
    out->exchange_ms = (double)e->rt->stats.exchange_ns.load() * 1e-6;
    out->final_ms = (double)e->rt->stats.final_ns.load() * 1e-6;
    out->exchanges = e->rt->stats.exchanges.load();
    out->exchange_rounds = e->rt->stats.exchange_rounds.load();
    out->exchange_bytes = e->rt->stats.exchange_bytes.load();
    out->cached_block_bytes = fq::block_cache_bytes();
    out->cached_workspace_bytes = fq::block_cache_workspace_bytes();
    out->project_launches = e->rt->stats.project_launches.load();
    out->project_rows = e->rt->stats.project_rows.load();
    out->project_kept = e->rt->stats.project_kept.load();
    out->project_bytes = e->rt->stats.project_bytes.load();
    out->project_ms = (double)e->rt->stats.project_ns.load() * 1e-6;
    return FQ_OK;
}

fq_status fq_engine_reset_stats(fq_engine *e) {
    if (!e) return fqc::fail(FQ_E_INVALID, "NULL engine");
    e->rt->stats.scan_launches = 0;
    e->rt->stats.scan_rows = 0;
    e->rt->stats.scan_bytes = 0;
    e->rt->stats.scan_ns = 0;
    e->rt->stats.queries = 0;
    e->rt->stats.plan_ns = 0;
    e->rt->stats.exec_ns = 0;
    e->rt->stats.first_launch_ns = 0;
    e->rt->stats.tail_ns = 0;
    e->rt->stats.complete_ns = 0;
    e->rt->stats.partial_ns = 0;
    e->rt->stats.exchange_ns = 0;
    e->rt->stats.final_ns = 0;
    e->rt->stats.exchanges = 0;
    e->rt->stats.exchange_rounds = 0;
    e->rt->stats.exchange_bytes = 0;
    e->rt->stats.project_launches = 0;
    e->rt->stats.project_rows = 0;
    e->rt->stats.project_kept = 0;
    e->rt->stats.project_bytes = 0;
    e->rt->stats.project_ns = 0;
    return FQ_OK;
}

int64_t fq_result_num_rows(const fq_result *r) { return r ? r->rows : 0; }
int32_t fq_result_num_columns(const fq_result *r) { return r ? (int32_t)r->names.size() : 0; }
const char *fq_result_column_name(const fq_result *r, int32_t col) {
    if (!r || col < 0 || col >= (int32_t)r->names.size()) return nullptr;
    return r->names[(size_t)col].c_str();
}
int32_t fq_result_column_type(const fq_result *r, int32_t col) {
    if (!r || col < 0 || col >= (int32_t)r->types.size()) return -1;
    return r->types[(size_t)col];
}
fq_status fq_result_mysql_type(const fq_result *r, int32_t col, int32_t *out) {
    if (!r || !out || col < 0 || col >= (int32_t)r->types.size())
        return fqc::fail(FQ_E_INVALID, "fq_result_mysql_type: out of range");
    // MySQLStream::execute (servers/mysql/mysql_stream.rs:30-62)
    switch (r->types[(size_t)col]) {
        case FQ_DT_INT8:
        case FQ_DT_INT16:
        case FQ_DT_INT32:
        case FQ_DT_INT64:
        case FQ_DT_UINT8:
        case FQ_DT_UINT16:
        case FQ_DT_UINT32:
        case FQ_DT_UINT64: *out = FQ_MYSQL_TYPE_LONG; return FQ_OK;
        case FQ_DT_FLOAT32:
        case FQ_DT_FLOAT64: *out = FQ_MYSQL_TYPE_FLOAT; return FQ_OK;
        case FQ_DT_UTF8: *out = FQ_MYSQL_TYPE_VARCHAR; return FQ_OK;
        default:
            return fqc::internal(std::string("Unsupported column type:") + fqc::dtype_name(r->types[(size_t)col]));
    }
}

fq_status fq_result_value(const fq_result *r, int64_t row, int32_t col, fq_value *out) {
    if (!r || !out || col < 0 || col >= (int32_t)r->cols.size() || row < 0 ||
        row >= (int64_t)r->cols[(size_t)col].size())
        return fqc::fail(FQ_E_INVALID, "fq_result_value: out of range");
    *out = r->cols[(size_t)col].abi((size_t)row);
    return FQ_OK;
}
fq_status fq_result_values(const fq_result *r, int32_t col, fq_value *out, int64_t n) {
    if (!r || (!out && n > 0) || col < 0 || col >= (int32_t)r->cols.size() || n < 0 ||
        n > (int64_t)r->cols[(size_t)col].size())
        return fqc::fail(FQ_E_INVALID, "fq_result_values: out of range");
    const ResultCol &c = r->cols[(size_t)col];
    if (c.is_flat()) {
        const fq_value proto = fq::DataValue::some((fq::DataType)c.flat_dtype, 0).to_abi();
        for (int64_t i = 0; i < n; ++i) {
            out[i] = proto;
            out[i].bits = c.flat[(size_t)i];
        }
        return FQ_OK;
    }
    for (int64_t i = 0; i < n; ++i) out[i] = c.v[(size_t)i].to_abi();
    return FQ_OK;
}
const char *fq_result_text(const fq_result *r, int64_t row, int32_t col) {
    if (!r || col < 0 || col >= (int32_t)r->cols.size() || row < 0 || row >= (int64_t)r->cols[(size_t)col].size())
        return nullptr;
    r->text.push_back(r->cols[(size_t)col].value((size_t)row).debug());
    return r->text.back().c_str();
}
void fq_result_free(fq_result *r) { delete r; }

// a one-row result's values into row[] (the first min(cap, columns)), the
// result freed: fq_engine_execute_row and the exchange _row calls (fq_comm.cpp)
fq_status fq_result_take_row(fq_result *r, fq_value *row, int32_t cap, int32_t *ncols, const char *what) {
    std::unique_ptr<fq_result> hold(r);
    const int64_t rows = fq_result_num_rows(r);
    if (rows != 1)
        return fqc::fail(FQ_E_INVALID,
                         std::string(what) + ": the statement returned " + std::to_string(rows) + " rows, not one");
    *ncols = (int32_t)r->cols.size();
    for (int32_t c = 0; c < *ncols && c < cap; ++c) row[c] = r->cols[(size_t)c].abi(0);
    return FQ_OK;
}

fq_status fq_engine_execute_row(fq_engine *e, const char *sql, fq_value *row, int32_t cap, int32_t *ncols) {
    if (!e || !sql || !ncols || cap < 0 || (cap > 0 && !row))
        return fqc::fail(FQ_E_INVALID, "fq_engine_execute_row: NULL argument");
    fq_result *r = nullptr;
    const fq_status s = fq_engine_execute(e, sql, &r);
    if (s != FQ_OK) return s;
    return fq_result_take_row(r, row, cap, ncols, "fq_engine_execute_row");
}

}  // extern "C"
