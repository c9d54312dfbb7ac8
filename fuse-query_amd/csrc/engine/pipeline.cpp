// Data sources, processors, streams and the pipeline.
#include "pipeline.h"

#include <string.h>

#include <exception>
#include <algorithm>
#include <map>

namespace fq {

// ---------------------------------------------------------------------------
// system.numbers_mt
// ---------------------------------------------------------------------------
static constexpr uint64_t kBlockSize = 10000;  // numbers_stream.rs:29

NumbersTable::NumbersTable() {
    auto s = std::make_shared<DataSchema>();
    s->fields.push_back(DataField{"number", FQ_DT_UINT64, false});  // numbers_table.rs:21-25
    schema_ = s;
}

// NumbersTable::generate_parts (numbers_table.rs:29-55)
std::vector<Partition> NumbersTable::generate_parts(uint64_t total) {
    const uint64_t workers = 8, chunk = total / workers;
    std::vector<Partition> parts;
    auto name = [&](uint64_t a, uint64_t b) {
        return std::to_string(total) + "-" + std::to_string(a) + "-" + std::to_string(b);
    };
    if (chunk == 0) {
        parts.push_back(Partition{name(0, total - 1), 0});  // total - 1 wraps at 0 (release build)
        return parts;
    }
    const uint64_t remain = total % workers;
    for (uint64_t p = 0; p < workers; ++p) {
        const uint64_t start = p * chunk;
        uint64_t end = (p + 1) * chunk - 1;
        if (p == workers - 1 && remain > 0) end += remain;
        parts.push_back(Partition{name(start, end), 0});
    }
    return parts;
}

void NumbersTable::parse_part(const std::string &n, uint64_t &total, uint64_t &begin, uint64_t &end) {
    const size_t a = n.find('-'), b = n.find('-', a == std::string::npos ? a : a + 1);
    if (a == std::string::npos || b == std::string::npos) throw_internal("bad numbers_mt partition name: " + n);
    total = std::stoull(n.substr(0, a));
    begin = std::stoull(n.substr(a + 1, b - a - 1));
    end = std::stoull(n.substr(b + 1));
}

// NumbersStream::create (numbers_stream.rs:27-62): the partition's blocks are
// one contiguous run; the last block ends at block_begin + remain.
uint64_t NumbersTable::stream_rows(uint64_t begin, uint64_t end) {
    const uint64_t count = end - begin + 1;
    const uint64_t nblocks = count / kBlockSize, remain = count % kBlockSize;
    if (nblocks == 0 || remain == 0) return count;
    return kBlockSize * (nblocks - 1) + remain + 1;
}

ReadDataSourcePlan NumbersTable::read_plan(const DataValue *arg) const {
    uint64_t total = 10000;  // numbers_table.rs:69
    if (arg && arg->kind == DataValue::kSome && (arg->dtype == FQ_DT_UINT64 || arg->dtype == FQ_DT_INT64))
        total = arg->bits;
    ReadDataSourcePlan p;
    p.db = "system";
    p.table = name();
    p.table_type = "System";
    p.schema = schema_;
    p.partitions = generate_parts(total);
    p.description = "(Read from system.numbers_mt table)";
    return p;
}

void NumbersTable::pin(const std::string &part, Column col) {
    std::lock_guard<std::mutex> lk(mu_);
    resident_[part] = std::move(col);
}
void NumbersTable::unpin_all() {
    std::lock_guard<std::mutex> lk(mu_);
    resident_.clear();
}
bool NumbersTable::pinned(const std::string &part, Column &out) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = resident_.find(part);
    if (it == resident_.end()) return false;
    out = it->second;
    return true;
}

// NumbersStream::poll_next (numbers_stream.rs:65-83): one device block per
// partition (its 10,000-row blocks are kept as sub_block_rows), or -- for a
// row pipeline -- the partition's rows as consecutive morsels of growing size
// (the same rows in the same order; a LIMIT that is satisfied stops pulling
// after the first few instead of after a whole partition).
class NumbersStream : public BlockStream {
   public:
    NumbersStream(NumbersTable *t, SchemaRef s, std::vector<Partition> parts, ReadMode mode)
        : t_(t), schema_(std::move(s)), parts_(std::move(parts)), mode_(mode) {}
    bool next(DataBlock &out) override {
        if (off_ >= rows_) {  // next partition
            if (i_ >= parts_.size()) return false;
            const Partition &p = parts_[i_++];
            uint64_t total, end;
            NumbersTable::parse_part(p.name, total, begin_, end);
            if (end - begin_ + 1 == 0 || end < begin_)
                throw_status(FQ_E_UNSUPPORTED, "numbers_mt partition " + p.name +
                                                   " materialises 2^64 rows in the reference (total - 1 wraps)");
            rows_ = NumbersTable::stream_rows(begin_, end);
            off_ = 0;
            morsel_ = NumbersTable::kMorselFirst;
            has_pinned_ = t_->pinned(p.name, pinned_) && (uint64_t)pinned_.len == rows_;
            // kChunks: equal pieces of whole 10,000-row blocks, at most chunk_rows() each
            const uint64_t blocks = (rows_ + kBlockSize - 1) / kBlockSize;
            const uint64_t per = std::max<uint64_t>(1, t_->chunk_rows() / kBlockSize);
            const uint64_t pieces = (blocks + per - 1) / per;
            piece_ = pieces ? (blocks + pieces - 1) / pieces * kBlockSize : rows_;
            if (rows_ == 0) {  // an empty partition still yields its (empty) block
                emit(Column::device(FQ_DT_UINT64, 0, ExecCtx::current().stream()), out);
                return true;
            }
        }
        // row pipelines: growing morsels; aggregates: the resident partition
        // whole, a generated one in chunk_rows() pieces (bounded HBM; whole
        // 10,000-row blocks, so the per-block state replay is unchanged)
        const uint64_t n = mode_ == ReadMode::kMorsels ? std::min(morsel_, rows_ - off_)
                           : mode_ == ReadMode::kChunks ? std::min(piece_, rows_ - off_)
                           : has_pinned_                ? rows_ - off_
                                                        : std::min(t_->chunk_rows(), rows_ - off_);
        Column col;
        if (has_pinned_) {
            col = pinned_.slice((int64_t)off_, (int64_t)n);
        } else {
            ExecCtx &ctx = ExecCtx::current();
            col = Column::device(FQ_DT_UINT64, (int64_t)n, ctx.stream());
            check_fq(fq_fill_numbers_u64((uint64_t *)col.dptr(), begin_ + off_, n, ctx.stream()));
            col.iota = true;
        }
        off_ += n;
        morsel_ = std::min(morsel_ * 2, NumbersTable::kMorselMax);
        emit(col, out);
        return true;
    }

   private:
    void emit(const Column &col, DataBlock &out) {
        out = DataBlock{};
        out.schema = schema_;
        out.columns.push_back(col);
        out.sub_block_rows = (int64_t)kBlockSize;
    }
    NumbersTable *t_;
    SchemaRef schema_;
    std::vector<Partition> parts_;
    ReadMode mode_;
    size_t i_ = 0;
    uint64_t begin_ = 0, rows_ = 0, off_ = 0, morsel_ = 0, piece_ = 0;
    bool has_pinned_ = false;
    Column pinned_;
};

StreamRef NumbersTable::read(const std::vector<Partition> &parts, ReadMode mode) {
    return std::make_unique<NumbersStream>(this, schema_, parts, mode);
}

DataSource::DataSource() : numbers_(std::make_shared<NumbersTable>()) {
    dbs_["system"]["numbers_mt"] = numbers_;  // datasource.rs:22-33
}

TableRef DataSource::get_table(const std::string &db, const std::string &table) const {
    auto d = dbs_.find(db);
    if (d == dbs_.end()) throw_internal("Cannot find the database: " + db);
    auto t = d->second.find(table);
    if (t == d->second.end()) throw_internal("Cannot find the table: " + table);
    return t->second;
}

// ---------------------------------------------------------------------------
// processors
// ---------------------------------------------------------------------------
std::string IProcessor::format(FormatterSettings &s) const {
    std::string out;
    if (s.indent > 0) {
        out += "\n";
        for (size_t i = 0; i < s.indent; ++i) out += s.indent_char;
    }
    out += s.prefix + " " + name() + " \xc3\x97 " + std::to_string(s.ways) + " " +
           (s.ways == 1 ? "processor" : "processors");
    return out;
}

std::string MergeProcessor::format(FormatterSettings &s) const {
    std::string out;
    if (s.indent > 0) {
        out += "\n";
        for (size_t i = 0; i < s.indent; ++i) out += s.indent_char;
    }
    out += s.prefix + " Merge (" + s.prev_name + " \xc3\x97 " + std::to_string(s.prev_ways) + " " +
           (s.prev_ways == 1 ? "processor" : "processors") + ") to (" + name() + " \xc3\x97 " +
           std::to_string(s.ways) + ")";
    return out;
}

// tokio mpsc::channel(partitions) + ChannelStream (stream_channel.rs:14-28)
struct Channel {
    std::mutex mu;
    std::condition_variable cv_send, cv_recv;
    struct Item {
        bool is_err = false;
        size_t pipe = 0;  // input index (partition order)
        DataBlock block;
        FQException err{0, ""};
    };
    std::deque<Item> q;
    size_t cap = 1;
    int live = 0;
    bool closed = false;

    bool send(Item it) {
        std::unique_lock<std::mutex> lk(mu);
        cv_send.wait(lk, [&] { return q.size() < cap || closed; });
        if (closed) return false;
        q.push_back(std::move(it));
        cv_recv.notify_one();
        return true;
    }
    // errors are queued even after close() (the consumer drains them to pick
    // the earliest partition's) and never wait for room
    void send_error(Item it) {
        std::lock_guard<std::mutex> lk(mu);
        q.push_back(std::move(it));
        cv_recv.notify_one();
    }
    void done() {
        std::lock_guard<std::mutex> lk(mu);
        --live;
        cv_recv.notify_all();
    }
    bool recv(Item &it) {
        std::unique_lock<std::mutex> lk(mu);
        cv_recv.wait(lk, [&] { return !q.empty() || live == 0; });
        if (q.empty()) return false;
        it = std::move(q.front());
        q.pop_front();
        cv_send.notify_one();
        return true;
    }
    void close() {
        std::lock_guard<std::mutex> lk(mu);
        closed = true;
        cv_send.notify_all();
    }
    bool is_closed() {
        std::lock_guard<std::mutex> lk(mu);
        return closed;
    }
    void wait_all_done() {
        std::unique_lock<std::mutex> lk(mu);
        cv_recv.wait(lk, [&] { return live == 0; });
    }
};

class ChannelStream : public BlockStream {
   public:
    std::shared_ptr<Channel> ch;
    ~ChannelStream() override {
        ch->close();
        ch->wait_all_done();  // every pipe task has released its device context
    }
    bool next(DataBlock &out) override {
        Channel::Item it;
        if (!ch->recv(it)) return false;
        settle(it);
        if (it.is_err) {
            // Several pipes may fail; the reference surfaces whichever error
            // reaches its channel first (processor_merge.rs:45-63).  Report
            // the one of the earliest partition instead -- deterministic, and
            // what a sequential run of the partitions raises first.
            ch->close();
            Channel::Item e = std::move(it);
            while (ch->recv(it)) {
                settle(it);
                if (it.is_err && it.pipe < e.pipe) e = std::move(it);
            }
            throw e.err;
        }
        out = std::move(it.block);
        return true;
    }

   private:
    // a block whose states are finished here (DataBlock::complete): its
    // failure is its pipe's error, ordered like one the pipe sent itself
    static void settle(Channel::Item &it) {
        if (it.is_err || !it.block.complete) return;
        try {
            complete_block(it.block);
        } catch (const FQException &e) {
            it.is_err = true;
            it.err = e;
        } catch (const std::exception &e) {
            it.is_err = true;
            it.err = FQException(FQ_E_INTERNAL, std::string("Internal Error: ") + e.what());
        }
    }
};

// A pipe's task failed: its error goes to the channel the way the reference's
// task sends its Err (processor_merge.rs:50-54), and the pipe's processor
// releases what the other pipes wait on.
static void pipe_failed(const ProcessorRef &in, const std::shared_ptr<Channel> &ch, size_t pipe, const FQException &e) {
    in->abandon();
    Channel::Item it;
    it.is_err = true;
    it.pipe = pipe;
    it.err = e;
    ch->send_error(std::move(it));
}

// MergeProcessor::execute (processor_merge.rs:37-66): one host thread per
// input pipe (the tokio::spawn), each with its own device context.
StreamRef MergeProcessor::execute() {
    if (list_.empty()) throw_internal("Merge processor cannot be zero");
    if (list_.size() == 1) return list_[0]->execute();
    Runtime *rt = ExecCtx::current().rt;
    auto cs = std::make_unique<ChannelStream>();
    cs->ch = std::make_shared<Channel>();
    cs->ch->cap = list_.size();
    cs->ch->live = (int)list_.size();
    auto task = [&](size_t pipe) {
        std::shared_ptr<Channel> ch = cs->ch;
        ProcessorRef in = list_[pipe];
        const QueueKind queues = queues_;
        return [in, ch, rt, pipe, queues]() {
            try {
                if (rt->fault_pipe.load(std::memory_order_relaxed) == (int64_t)pipe + 1)
                    throw FQException(FQ_E_HIP, "hipMalloc(workspace): out of memory (FQ_OPT_FAULT_PIPE)");
                ExecCtx ctx(rt, queues, pipe);
                StreamRef s = in->execute();
                DataBlock b;
                // the consumer gone (a satisfied LIMIT dropped the merged
                // stream): stop pulling instead of scanning the rest
                while (!ch->is_closed() && s->next(b)) {
                    // device work of this block done before another thread reads
                    // it; a host block (AggregatePartial's states) has none left
                    bool device = (bool)b.layout || (bool)b.filter;
                    for (const Column &c : b.columns) device |= c.on_device();
                    if (device && !b.ready) ctx.sync();
                    Channel::Item it;
                    b.pipe = (int32_t)pipe;
                    it.pipe = pipe;
                    it.block = std::move(b);
                    if (!ch->send(std::move(it))) break;
                }
            } catch (const FQException &e) {
                pipe_failed(in, ch, pipe, e);
            } catch (const std::exception &e) {
                pipe_failed(in, ch, pipe, FQException(FQ_E_INTERNAL, std::string("Internal Error: ") + e.what()));
            } catch (...) {  // every pipe reports done, or the consumer waits for it forever
                pipe_failed(in, ch, pipe, FQException(FQ_E_INTERNAL, "Internal Error: unknown exception in a pipe"));
            }
            ch->done();
        };
    };
    // Pipes whose output is one block (AggregatePartial: it enqueues its scans
    // and hands over a deferred block without waiting) can run on this thread:
    // pipe 0 runs first and enqueues its scan without waiting for a pool thread
    // to wake (nor for the other pipes' submissions); the others' scans queue
    // behind that ~1.4 ms scan anyway.  The channel holds every pipe's block,
    // so nothing here waits for the consumer.
    if (inline_first_) task(0)();
    for (size_t pipe = inline_first_ ? 1 : 0; pipe < list_.size(); ++pipe) {
        try {
            rt->pool.submit(task(pipe));
        } catch (const std::exception &e) {
            // this pipe and the ones after it never run: each reports its
            // failure and is done, so the consumer and the scan group do not
            // wait for them
            for (size_t p = pipe; p < list_.size(); ++p) {
                pipe_failed(list_[p], cs->ch, p, FQException(FQ_E_INTERNAL, std::string("Internal Error: ") + e.what()));
                cs->ch->done();
            }
            break;
        }
    }
    return cs;
}

StreamRef SourceTransform::execute() {
    TableRef t = ctx_->get_table(db_, table_);  // transform_source.rs:49-52
    return t->read(parts_, mode_);
}

namespace {
class MapStream : public BlockStream {
   public:
    MapStream(StreamRef in, std::function<DataBlock(DataBlock)> f) : in_(std::move(in)), f_(std::move(f)) {}
    bool next(DataBlock &out) override {
        DataBlock b;
        if (!in_->next(b)) return false;
        out = f_(std::move(b));
        return true;
    }

   private:
    StreamRef in_;
    std::function<DataBlock(DataBlock)> f_;
};

struct FusionGuard {
    ExecCtx &ctx;
    AggFusion *prev;
    FusionGuard(ExecCtx &c, AggFusion *f) : ctx(c), prev(c.fusion) { ctx.fusion = f; }
    ~FusionGuard() { ctx.fusion = prev; }
};
}  // namespace

// FilterTransform: the block keeps its columns and carries the predicate;
// the aggregate scan fuses it, every other consumer compacts (materialize).
StreamRef FilterTransform::execute() {
    FunctionRef pred = func_->clone();
    return std::make_unique<MapStream>(input_->execute(), [pred](DataBlock b) {
        if (needs_materialize(b)) b = materialize(b, ExecCtx::current());
        b.filter = pred;
        return b;
    });
}

namespace {
// a pipe's stream that reports its end (or its destruction, a pipe that
// failed or was stopped) to the query's LaunchSpan, once
class SpanStream : public BlockStream {
   public:
    SpanStream(StreamRef in, LaunchSpanRef span) : in_(std::move(in)), span_(std::move(span)) {}
    ~SpanStream() override { end(); }
    bool next(DataBlock &out) override {
        if (in_->next(out)) return true;
        end();
        return false;
    }

   private:
    void end() {
        if (span_) span_->arrive();
        span_.reset();
    }
    StreamRef in_;
    LaunchSpanRef span_;
};
}  // namespace

void ProjectionTransform::abandon() {
    if (!entered_.exchange(true) && span_) span_->arrive();
    input_->abandon();
}

StreamRef ProjectionTransform::execute() {
    SchemaRef schema = schema_;
    std::vector<FunctionRef> funcs;
    for (auto &f : funcs_) funcs.push_back(f->clone());
    const bool blocks = block_stream_;
    LaunchSpanRef span = entered_.exchange(true) ? nullptr : span_;
    // the span's arrival is owned by the SpanStream from here on
    struct Arrive {
        LaunchSpanRef s;
        ~Arrive() {
            if (s) s->arrive();
        }
    } arrive_on_throw{span};
    StreamRef in = input_->execute();
    LaunchSpan *sp = span.get();
    StreamRef mapped = std::make_unique<MapStream>(std::move(in), [schema, funcs, blocks, sp](DataBlock b) {
        ExecCtx &ctx = ExecCtx::current();
        DataBlock out;
        if (b.layout) b = materialize(b, ctx);  // a block stream in: one array first
        if (project_fused(b, funcs, schema, ctx, out, blocks, sp)) return out;  // filter + expressions in one pass
        b = materialize(b, ctx);
        const int64_t rows = b.num_rows();
        out.schema = schema;
        for (auto &f : funcs) out.columns.push_back(f->eval(b, ctx).to_array(rows, ctx));
        return out;
    });
    arrive_on_throw.s.reset();
    if (!span) return mapped;
    return std::make_unique<SpanStream>(std::move(mapped), std::move(span));
}

namespace {
// one partition's partial states still on the device: what the consumer needs
// to finish them once the query's scans have ended (members in destruction
// order: the fusion, which may still wait for its scans, before the lease)
struct PendingPartial {
    Runtime *rt = nullptr;
    std::shared_ptr<WorkerRes> res;  // the pipe's result slots and queue
    ScanGroupRef group;
    std::vector<FunctionRef> funcs;
    std::unique_ptr<AggFusion> fusion;
};

// the partial states block's one column (transform_aggregate_partial.rs:64-78)
Column partial_states(const std::vector<FunctionRef> &funcs) {
    std::vector<DataValue> rows;
    for (auto &f : funcs) rows.push_back(DataValue::make_struct(f->accumulate_result()));
    return Column::host_values(FQ_DT_NULL, std::move(rows));
}
}  // namespace

void AggregatePartialTransform::abandon() {
    if (!entered_.exchange(true) && group_) group_->arrive(false);
    input_->abandon();
}

StreamRef AggregatePartialTransform::execute() {
    // this pipe's place in the query's ScanGroup: arrives once, also when it fails
    ScanTicket ticket(entered_.exchange(true) ? nullptr : group_.get());
    std::vector<FunctionRef> funcs;
    for (auto &f : funcs_) funcs.push_back(f->clone());
    ExecCtx &ctx = ExecCtx::current();
    StreamRef in = input_->execute();
    auto fusion = std::make_unique<AggFusion>(ctx, &ticket);
    {
        FusionGuard guard(ctx, fusion.get());
        DataBlock b;
        while (in->next(b)) {
            if (b.layout) b = materialize(b, ctx);
            for (auto &f : funcs) f->accumulate(b, ctx);
            fusion->end_block();
        }
    }
    DataBlock out;
    out.schema = schema_;
    if (fusion->finish_deferred()) {
        // The pipe does not wait: its block carries the states' completion,
        // which the consumer runs (ChannelStream::next / AggregateFinal) once
        // the query's scans have ended -- one thread waits on the group's end
        // event and reads every partition's states, none is woken per pipe.
        auto p = std::make_shared<PendingPartial>();
        p->rt = ctx.rt;
        p->res = ctx.lease();
        p->group = group_;
        p->funcs = std::move(funcs);
        p->fusion = std::move(fusion);
        out.complete = [p](DataBlock &blk) {
            p->group->wait_end();
            const int64_t t0 = now_ns();
            p->group->account();
            p->fusion->replay();
            p->fusion.reset();
            blk.columns.push_back(partial_states(p->funcs));
            if (p->rt->profile.load(std::memory_order_relaxed) == 2)
                p->rt->stats.complete_ns += (uint64_t)(now_ns() - t0);
        };
    } else {
        fusion->finish();
        fusion.reset();
        out.columns.push_back(partial_states(funcs));
    }
    return std::make_unique<DataBlockStream>(std::vector<DataBlock>{out});
}

StreamRef AggregateFinalTransform::execute() {
    std::vector<FunctionRef> funcs;
    for (auto &f : funcs_) funcs.push_back(f->clone());
    StreamRef in = input_->execute();
    // Every partial first, then the merge: an error of any partition (the
    // earliest partition's, see ChannelStream) wins over an error of the
    // merge itself (e.g. two None sums), as in a run where each partition's
    // error surfaces before the final sees the other partitions' states.
    std::vector<DataBlock> partials;
    DataBlock b;
    while (in->next(b)) partials.push_back(std::move(b));
    for (DataBlock &pb : partials) complete_block(pb);  // one pipe: no channel ran it
    for (const DataBlock &pb : partials) {
        if (pb.columns.empty() || !pb.columns[0].host) continue;
        const std::vector<DataValue> &rows = *pb.columns[0].host;
        for (size_t i = 0; i < funcs.size() && i < rows.size(); ++i)
            if (rows[i].kind == DataValue::kStruct) funcs[i]->merge_state(rows[i].fields);
    }
    DataBlock out;
    out.schema = schema_;
    if (emit_states_) {
        std::vector<DataValue> rows;
        for (auto &f : funcs) rows.push_back(DataValue::make_struct(f->accumulate_result()));
        out.columns.push_back(Column::host_values(FQ_DT_NULL, std::move(rows)));
    } else {
        for (auto &f : funcs) {
            const DataValue v = f->merge_result();
            if (v.kind == DataValue::kNone) throw_internal("DataValue to array cannot be NONE NULL");
            if (v.kind == DataValue::kStruct) throw_internal("DataValue to array cannot be NONE " + v.debug());
            out.columns.push_back(Column::host_values(v.kind == DataValue::kNull ? FQ_DT_NULL : v.dtype, {v}));
        }
    }
    return std::make_unique<DataBlockStream>(std::vector<DataBlock>{out});
}

// ---------------------------------------------------------------------------
// GROUP BY
// ---------------------------------------------------------------------------
namespace {

// (key, row) pairs by key, ties by row: std::sort below 4,096 pairs, else a
// stable LSD radix sort on 16-bit digits of the key (skipping digits that are
// equal in every key) -- 100,000 groups sorted in ~1 ms instead of ~6 ms
void sort_key_index(std::vector<std::pair<uint64_t, uint32_t>> &v) {
    const size_t n = v.size();
    if (n < 4096) {
        std::sort(v.begin(), v.end());
        return;
    }
    uint64_t all_or = 0, all_and = ~0ull;
    for (const auto &p : v) {
        all_or |= p.first;
        all_and &= p.first;
    }
    std::vector<std::pair<uint64_t, uint32_t>> tmp(n);
    std::vector<uint32_t> cnt(1u << 16);
    for (int shift = 0; shift < 64; shift += 16) {
        if ((((all_or ^ all_and) >> shift) & 0xffffull) == 0) continue;  // this digit is the same everywhere
        std::fill(cnt.begin(), cnt.end(), 0u);
        for (const auto &p : v) ++cnt[(p.first >> shift) & 0xffff];
        uint32_t run = 0;
        for (auto &c : cnt) {
            const uint32_t x = c;
            c = run;
            run += x;
        }
        for (const auto &p : v) tmp[cnt[(p.first >> shift) & 0xffff]++] = p;
        v.swap(tmp);
    }
}

std::vector<AggregatorFunction *> leaves_of(const std::vector<FunctionRef> &funcs) {
    std::vector<AggregatorFunction *> v;
    for (auto &f : funcs) f->collect_aggregators(v);
    return v;
}

// one leaf's state from its 64-bit device word
DataValue leaf_value(uint32_t op, DataType dt, uint64_t bits) {
    return DataValue::some(op == FQ_AGG_COUNT ? FQ_DT_UINT64 : dt, bits);
}

// the atomics' fold, on host values of one leaf (exchange merge)
DataValue fold_leaf(uint32_t op, const DataValue &a, const DataValue &b) {
    if (a.kind != DataValue::kSome) return b;
    if (b.kind != DataValue::kSome) return a;
    const DataType dt = a.dtype;
    if (op == FQ_AGG_COUNT || op == FQ_AGG_SUM) {
        if (dt == FQ_DT_FLOAT64) {
            const double r = __builtin_bit_cast(double, a.bits) + __builtin_bit_cast(double, b.bits);
            return DataValue::some(dt, __builtin_bit_cast(uint64_t, r));
        }
        return DataValue::some(dt, a.bits + b.bits);
    }
    bool b_better;
    if (dt == FQ_DT_FLOAT64) {
        const double x = __builtin_bit_cast(double, a.bits), y = __builtin_bit_cast(double, b.bits);
        b_better = op == FQ_AGG_MAX ? y > x : y < x;
    } else if (dt == FQ_DT_INT64) {
        const int64_t x = (int64_t)a.bits, y = (int64_t)b.bits;
        b_better = op == FQ_AGG_MAX ? y > x : y < x;
    } else {
        b_better = op == FQ_AGG_MAX ? b.bits > a.bits : b.bits < a.bits;
    }
    return b_better ? b : a;
}

// One leaf's states over the rows of a GROUP BY final: 64-bit words plus a
// Some/None flag per row (exchanged states may be None; device ones never)
struct FlatLeaf {
    DataType dtype = FQ_DT_NULL;
    std::vector<uint64_t> bits;
    std::vector<uint8_t> some;
    DataValue value(uint32_t r) const {
        return some[r] ? DataValue::some(dtype, bits[r]) : DataValue::none(dtype);
    }
    // row `to` = fold_leaf(row `to`, row `from`)
    void fold_into(uint32_t op, uint32_t to, uint32_t from) {
        if (!some[from]) return;
        if (!some[to]) {
            bits[to] = bits[from];
            some[to] = 1;
            return;
        }
        const DataValue v = fold_leaf(op, DataValue::some(dtype, bits[to]), DataValue::some(dtype, bits[from]));
        bits[to] = v.bits;
    }
};

}  // namespace

// GROUP BY sizing from a sample of the first block: the distinct keys among
// its first kGroupSampleRows passing rows (a count-only table).  A sample
// whose keys repeat (distinct <= half the rows) has seen about all the groups
// of a block; one that is still mostly distinct grows with the rows.  Beyond
// 3,072 groups per launch (3/4 of an LDS table) the launches go through the
// radix-partitioned kernels with about 1,024 groups per bin; the table gets
// twice the expected groups in slots (a TABLE_FULL re-run grows it 16x).
namespace {
constexpr int64_t kGroupSampleRows = 1 << 21;
constexpr int64_t kGroupMinSlots = 1 << 16;

struct GroupPlan {
    int64_t capacity = 4096;
    int log2_parts = 0;
};

int64_t next_pow2(int64_t v) {
    int64_t p = 64;
    while (p < v && p < ((int64_t)1 << 30)) p <<= 1;
    return p;
}

GroupPlan plan_group_by(const fq_group_table &d, const fq_col &c, const fq_pred *pred, const fq_expr *key,
                        int64_t blocks, ExecCtx &ctx) {
    // dense keys (`key % d` that the kernel's LDS table indexes directly):
    // at most d groups, never the partitioned path, no sample needed
    if (const int64_t dk = key ? fq_group_dense_keys(c.dtype, key, d.n_aggs) : 0) {
        GroupPlan p;
        p.capacity = next_pow2(std::max<int64_t>(4096, 2 * dk));
        return p;
    }
    const int64_t rows = std::min<int64_t>(c.len, kGroupSampleRows);
    fq_group_table t{};
    t.capacity = next_pow2(2 * rows);
    t.key_dtype = d.key_dtype;
    t.n_aggs = 1;
    t.kinds[0] = FQ_AGG_COUNT;
    t.dtypes[0] = FQ_DT_UINT64;
    auto mem = DeviceBuffer::alloc(fq_group_table_bytes(t.capacity, 1), ctx.stream());
    t.d_mem = mem->ptr;
    fq_col sample = c;
    sample.len = rows;
    {
        std::lock_guard<std::mutex> lk(*ctx.launch_mu());
        check_fq(fq_group_table_init(&t, ctx.stream()));
        check_fq(fq_group_aggregate(&t, &sample, pred, key, nullptr, ctx.stream()));
    }
    int64_t g = 0;
    check_fq(fq_group_table_count(&t, &g, ctx.stream()));  // synchronises
    const bool repeats = 2 * g <= rows;
    const int64_t per_launch =
        repeats ? 2 * g : (int64_t)((double)g * (double)c.len / (double)std::max<int64_t>(rows, 1));
    GroupPlan p;
    // at least 2^16 slots (~32 MB with 3 states and 16 replicas; init and
    // extract stay in the tens of microseconds): clustered keys -- each
    // partition its own key range, number / 1000000 -- show few groups in
    // the sample but many per query, and a full table costs a re-run
    // keys that keep coming (mostly distinct in the sample, GROUP BY number)
    // differ from block to block as well: the table holds every block's
    p.capacity = next_pow2(std::max<int64_t>(kGroupMinSlots, 2 * per_launch * (repeats ? 1 : blocks)));
    if (per_launch > 3072) {  // ~1,024 groups per bin (tools/groupby_sweep.py: 100,000 groups x 3
        p.log2_parts = 1;       // aggregates, P = 64/128/256: 13.3/12.4/13.8 ms per 10 GB)
        while (p.log2_parts < 8 && (per_launch >> p.log2_parts) > 1024) ++p.log2_parts;
    }
    return p;
}
}  // namespace

StreamRef GroupByPartialTransform::execute() {
    ExecCtx &ctx = ExecCtx::current();
    std::vector<FunctionRef> funcs;
    for (auto &f : funcs_) funcs.push_back(f->clone());
    const std::vector<AggregatorFunction *> leaves = leaves_of(funcs);
    if (leaves.size() > FQ_MAX_GROUP_AGGS)
        throw_status(FQ_E_UNSUPPORTED, "GROUP BY supports at most " + std::to_string(FQ_MAX_GROUP_AGGS) +
                                           " aggregate functions on the device path");
    StreamRef in = input_->execute();
    DataBlock b;
    bool launched = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timed;
    while (in->next(b)) {
        const DataSchema &s = *b.schema;
        FusedChain kc;
        if (!key_->to_chain(s, kc))
            throw_status(FQ_E_UNSUPPORTED, "GROUP BY key " + key_->display() +
                                               " must be an arithmetic expression over one column on the device path");
        if (kc.out_dtype != FQ_DT_UINT64 && kc.out_dtype != FQ_DT_INT64)
            throw_status(FQ_E_UNSUPPORTED, std::string("GROUP BY key must be UInt64 or Int64, not ") +
                                               dtype_name(kc.out_dtype));
        std::vector<FusedChain> args(leaves.size());
        for (size_t i = 0; i < leaves.size(); ++i) {
            if (leaves[i]->op() == FQ_AGG_COUNT) {
                args[i].column = kc.column;
                args[i].out_dtype = FQ_DT_UINT64;
                continue;
            }
            if (!leaves[i]->arg().to_chain(s, args[i]) || args[i].column != kc.column)
                throw_status(FQ_E_UNSUPPORTED, "GROUP BY aggregate " + leaves[i]->display() +
                                                   " must be over the key's column on the device path");
            const DataType dt = args[i].out_dtype;
            if (dt != FQ_DT_UINT64 && dt != FQ_DT_INT64 && dt != FQ_DT_FLOAT64)
                throw_status(FQ_E_UNSUPPORTED, std::string("GROUP BY state type ") + dtype_name(dt) +
                                                   " is not supported on the device path");
        }
        // the pending filter: fused when it is a predicate over the same column
        FusedPred fp;
        bool has_pred = false;
        if (b.filter) {
            if (b.filter->to_pred(s, fp) && fp.column == kc.column) has_pred = true;
            else b = materialize(b, ctx);
        }
        const Column &col = b.column_by_name(kc.column);
        if (col.len == 0) continue;
        fq_col c = col.abi();
        {
            std::lock_guard<std::mutex> lk(shared_->mu);
            if (!shared_->ready) {
                fq_group_table &d = shared_->desc;
                d = fq_group_table{};
                d.key_dtype = kc.out_dtype;
                d.n_aggs = (int32_t)leaves.size();
                shared_->leaf_ops.clear();
                for (size_t i = 0; i < leaves.size(); ++i) {
                    d.kinds[i] = (int32_t)leaves[i]->op();
                    d.dtypes[i] = args[i].out_dtype;
                    shared_->leaf_ops.push_back(leaves[i]->op());
                }
                if (leaves.empty()) {  // keys only (SELECT k ... GROUP BY k)
                    d.n_aggs = 1;
                    d.kinds[0] = FQ_AGG_COUNT;
                    d.dtypes[0] = FQ_DT_UINT64;
                    shared_->dummy_count = true;
                }
                const GroupPlan gp = plan_group_by(d, c, has_pred ? fp.get() : nullptr,
                                                   kc.expr.n_steps ? &kc.expr : nullptr, shared_->blocks_hint, ctx);
                d.capacity = std::max<int64_t>(ctx.rt->group_capacity.load(), gp.capacity);
                ctx.rt->group_used_capacity.store(d.capacity);
                shared_->log2_parts = gp.log2_parts;
                shared_->mem = DeviceBuffer::alloc(fq_group_table_bytes(d.capacity, d.n_aggs), ctx.stream());
                d.d_mem = shared_->mem->ptr;
                {
                    std::lock_guard<std::mutex> lk2(*ctx.launch_mu());
                    check_fq(fq_group_table_init(&d, ctx.stream()));
                }
                ctx.sync();  // other pipes may use other queues
                shared_->ready = true;
            }
        }
        fq_expr vals[FQ_MAX_GROUP_AGGS];
        for (size_t i = 0; i < leaves.size(); ++i) vals[i] = args[i].expr;
        const bool prof = ctx.rt->profile.load();
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (prof) {
            e0 = ctx.res->take_event();
            e1 = ctx.res->take_event();
            // compile the shape's kernel (first use) outside the timed pair
            fq_group_table probe = shared_->desc;
            fq_col empty = c;
            empty.len = 0;
            check_fq(fq_group_aggregate(&probe, &empty, has_pred ? fp.get() : nullptr,
                                        kc.expr.n_steps ? &kc.expr : nullptr, vals, ctx.stream()));
        }
        const int lp = shared_->log2_parts;
        // radix-partitioned launches go over the block in chunks of
        // FQ_OPT_GROUP_CHUNK_ROWS rows (a multiple of 64: bitmap predicates
        // are offset by whole words): the partition workspace (~8.6 B per row,
        // ~4.3 GB at the default 5e8) is the queue's kept workspace in the
        // device block cache (DeviceBuffer::alloc_workspace), so the next
        // query on this queue reuses it (mapping GBs afresh per query cost up
        // to 540 ms of hipMallocAsync)
        // (split evenly, no short tail chunk: a 1.25e9-row partition as 3 x
        // 4.17e8 ran 5.32 ms per 10 GB, as 5e8 + 5e8 + 2.5e8 5.72-5.76 on
        // another box -- profiles/r02_s4_g2_chunks.txt)
        int64_t chunk = c.len;
        if (lp > 0) {
            const int64_t cap = std::max<int64_t>(64, ctx.rt->group_chunk_rows.load());
            const int64_t pieces = (c.len + cap - 1) / cap;
            chunk = std::min<int64_t>(cap, ((c.len + pieces - 1) / pieces + 63) / 64 * 64);
            if (chunk < 1) chunk = 1;
        }
        std::shared_ptr<DeviceBuffer> ws;
        if (lp > 0) {
            const size_t need = fq_group_partition_workspace_bytes(chunk, lp);
            std::lock_guard<std::mutex> lk(shared_->mu);
            auto &slot = shared_->part_ws[ctx.stream()];
            if (!slot || slot->bytes < need) slot = DeviceBuffer::alloc_workspace(need, ctx.stream());
            ws = slot;
        }
        {
            std::lock_guard<std::mutex> lk(*ctx.launch_mu());
            if (prof) check_hip(hipEventRecord(e0, ctx.stream()), "hipEventRecord");
            if (lp > 0) {
                fq_pred pc{};
                if (has_pred) pc = *fp.get();
                for (int64_t off = 0; off < c.len; off += chunk) {
                    fq_col cc = c;
                    cc.data = (char *)c.data + off * 8;
                    cc.len = std::min(chunk, c.len - off);
                    if (has_pred && pc.kind == FQ_PRED_BITMAP) pc.bitmap = fp.get()->bitmap + off / 64;
                    // a numbers_mt chunk's values lie within 2^31 of its first: 4-byte partition rows
                    const int32_t lpf = lp | (col.iota && cc.len <= ((int64_t)1 << 31) ? FQ_GROUP_NARROW_ROWS : 0);
                    check_fq(fq_group_aggregate_partitioned(&shared_->desc, &cc, has_pred ? &pc : nullptr,
                                                            kc.expr.n_steps ? &kc.expr : nullptr, vals, lpf, ws->ptr,
                                                            ws->bytes, ctx.stream()));
                }
            } else
                check_fq(fq_group_aggregate(&shared_->desc, &c, has_pred ? fp.get() : nullptr,
                                            kc.expr.n_steps ? &kc.expr : nullptr, vals, ctx.stream()));
            if (prof) check_hip(hipEventRecord(e1, ctx.stream()), "hipEventRecord");
        }
        if (prof) timed.push_back({e0, e1});
        launched = true;
        ctx.rt->stats.scan_launches++;
        ctx.rt->stats.scan_rows += (uint64_t)c.len;
        ctx.rt->stats.scan_bytes += (uint64_t)c.len * 8u;
        if (const int64_t q0 = ctx.rt->stats.query_t0.exchange(0))
            ctx.rt->stats.first_launch_ns += (uint64_t)(now_ns() - q0);
    }
    if (launched) ctx.sync();  // the final transform reads the table from another pipe
    for (auto &p : timed) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess)
            ctx.rt->stats.scan_ns += (uint64_t)((double)ms * 1e6);
        ctx.res->give_event(p.first);
        ctx.res->give_event(p.second);
    }
    return std::make_unique<DataBlockStream>(std::vector<DataBlock>{});
}

StreamRef GroupByFinalTransform::execute() {
    ExecCtx &ctx = ExecCtx::current();
    std::vector<FunctionRef> funcs;
    for (auto &f : funcs_) funcs.push_back(f->clone());
    const std::vector<AggregatorFunction *> leaves = leaves_of(funcs);
    StreamRef in = input_->execute();
    // Groups as flat arrays: one row per (key, leaf states) from the device
    // table and from exchanged partial rows (Struct rows [key, leaf states...],
    // fq_engine_execute_final); sorted by key, equal keys folded.
    const size_t nl = leaves.size();
    DataType kdt = FQ_DT_NULL;
    std::vector<uint64_t> keys;
    std::vector<FlatLeaf> ls(nl);
    DataBlock b;
    std::vector<const std::vector<DataValue> *> exchanged;
    std::vector<DataBlock> held;  // keeps the exchanged rows alive
    while (in->next(b)) {
        if (b.columns.empty() || !b.columns[0].host) continue;
        for (const auto &row : *b.columns[0].host)
            if (row.kind == DataValue::kStruct && !row.fields.empty()) exchanged.push_back(&row.fields);
        held.push_back(b);
    }
    if (shared_->ready) kdt = shared_->desc.key_dtype;
    else if (!exchanged.empty()) kdt = (*exchanged[0])[0].dtype;
    for (const std::vector<DataValue> *rp : exchanged) {
        const std::vector<DataValue> &row = *rp;
        if (row.size() != 1 + nl) throw_status(FQ_E_INVALID, "GROUP BY: malformed partial state row");
        keys.push_back(row[0].bits);
        for (size_t a = 0; a < nl; ++a) {
            const DataValue &v = row[a + 1];
            if (ls[a].dtype == FQ_DT_NULL && v.kind == DataValue::kSome) ls[a].dtype = v.dtype;
            ls[a].bits.push_back(v.bits);
            ls[a].some.push_back(v.kind == DataValue::kSome ? 1 : 0);
        }
    }
    if (shared_->ready) {
        const fq_group_table &d = shared_->desc;
        int64_t groups = 0;
        check_fq(fq_group_table_count(&d, &groups, ctx.stream()));
        const int64_t n = groups > 0 ? groups : 1;
        auto kbuf = DeviceBuffer::alloc((size_t)n * 8, ctx.stream());
        std::vector<std::shared_ptr<DeviceBuffer>> st;
        uint64_t *ptrs[FQ_MAX_GROUP_AGGS] = {};
        for (int a = 0; a < d.n_aggs; ++a) {
            st.push_back(DeviceBuffer::alloc((size_t)n * 8, ctx.stream()));
            ptrs[a] = (uint64_t *)st.back()->ptr;
        }
        int64_t got = 0;
        check_fq(fq_group_table_extract(&d, (uint64_t *)kbuf->ptr, ptrs, n, &got, ctx.stream()));
        const size_t at = keys.size();  // after the exchanged rows (the fold order)
        keys.resize(at + (size_t)got);
        for (size_t a = 0; a < nl; ++a) {
            ls[a].dtype = leaves[a]->op() == FQ_AGG_COUNT ? FQ_DT_UINT64 : (DataType)d.dtypes[a];
            ls[a].bits.resize(at + (size_t)got);
            ls[a].some.resize(at + (size_t)got, 1);
        }
        if (got > 0) {
            check_hip(hipMemcpyAsync(keys.data() + at, kbuf->ptr, (size_t)got * 8, hipMemcpyDeviceToHost,
                                     ctx.stream()),
                      "hipMemcpyAsync");
            for (size_t a = 0; a < nl; ++a)
                check_hip(hipMemcpyAsync(ls[a].bits.data() + at, st[a]->ptr, (size_t)got * 8, hipMemcpyDeviceToHost,
                                         ctx.stream()),
                          "hipMemcpyAsync");
            ctx.sync();
        }
    }
    std::vector<uint32_t> rows;  // one source row per group, in key order
    if (emit_states_ && exchanged.empty()) {
        // partial states of this rank's own table: the keys are unique and
        // the receiving final merges and orders them, so no sort here
        rows.resize(keys.size());
        for (size_t i = 0; i < keys.size(); ++i) rows[i] = (uint32_t)i;
    } else {
        // sort by key (Int64 numerically: the sign bit flipped orders it as
        // unsigned), then fold each run of equal keys into its first row
        const uint64_t flip = kdt == FQ_DT_INT64 ? (1ull << 63) : 0ull;
        std::vector<std::pair<uint64_t, uint32_t>> order(keys.size());
        for (size_t i = 0; i < keys.size(); ++i) order[i] = {keys[i] ^ flip, (uint32_t)i};
        sort_key_index(order);
        rows.reserve(order.size());
        for (size_t i = 0; i < order.size();) {
            const uint32_t r0 = order[i].second;
            size_t j = i + 1;
            for (; j < order.size() && order[j].first == order[i].first; ++j)
                for (size_t a = 0; a < nl; ++a) ls[a].fold_into(leaves[a]->op(), r0, order[j].second);
            rows.push_back(r0);
            i = j;
        }
    }
    DataBlock out;
    out.schema = schema_;
    const size_t ng = rows.size();
    if (emit_states_) {
        std::vector<DataValue> srows;
        srows.reserve(ng);
        for (uint32_t r : rows) {
            std::vector<DataValue> row;
            row.reserve(1 + nl);
            row.push_back(DataValue::some(kdt, keys[r]));
            for (size_t a = 0; a < nl; ++a) row.push_back(ls[a].value(r));
            srows.push_back(DataValue::make_struct(std::move(row)));
        }
        out.columns.push_back(Column::host_values(FQ_DT_NULL, std::move(srows)));
        return std::make_unique<DataBlockStream>(std::vector<DataBlock>{out});
    }
    // key column, then each aggregate expression evaluated from its leaves;
    // an expression that IS one leaf (count(x), sum(x) ...) is that leaf's
    // states as they stand (merge_result returns the state).  The key and
    // such leaves are flat host columns (all Some); trees are DataValues.
    std::vector<std::vector<DataValue>> cols(1 + funcs.size());
    std::vector<std::vector<uint64_t>> flat(1 + funcs.size());
    std::vector<DataType> flat_dt(1 + funcs.size(), FQ_DT_NULL);
    flat[0].resize(ng);
    flat_dt[0] = kdt;
    for (size_t i = 0; i < ng; ++i) flat[0][i] = keys[rows[i]];
    std::vector<int> direct(funcs.size(), -1);
    bool any_tree = false;
    for (size_t f = 0; f < funcs.size(); ++f) {
        for (size_t a = 0; a < nl; ++a)
            if (funcs[f].get() == static_cast<Function *>(leaves[a])) direct[f] = (int)a;
        any_tree |= direct[f] < 0;
    }
    for (size_t f = 0; f < funcs.size(); ++f) {
        if (direct[f] < 0) {
            cols[f + 1].reserve(ng);
            continue;
        }
        const FlatLeaf &L = ls[(size_t)direct[f]];
        std::vector<uint64_t> &fc = flat[f + 1];
        fc.resize(ng);
        flat_dt[f + 1] = L.dtype;
        for (size_t i = 0; i < ng; ++i) {
            const uint32_t r = rows[i];
            if (!L.some[r]) throw_internal("DataValue to array cannot be NONE NULL");
            fc[i] = L.bits[r];
        }
    }
    if (any_tree) {
        for (uint32_t r : rows) {
            for (size_t a = 0; a < nl; ++a) leaves[a]->set_state(ls[a].value(r));
            for (size_t f = 0; f < funcs.size(); ++f) {
                if (direct[f] >= 0) continue;
                DataValue v = funcs[f]->merge_result();
                if (v.kind == DataValue::kNone) throw_internal("DataValue to array cannot be NONE NULL");
                cols[f + 1].push_back(std::move(v));
            }
        }
    }
    for (size_t c = 0; c < cols.size(); ++c) {
        DataType dt = c < schema_->fields.size() ? schema_->fields[c].dtype : FQ_DT_NULL;
        if (flat_dt[c] != FQ_DT_NULL && ng > 0) {  // the states' own type, as the DataValue path had it
            out.columns.push_back(Column::host_flat(flat_dt[c], std::move(flat[c])));
            continue;
        }
        if (c == 0 || (c > 0 && direct[c - 1] >= 0)) {  // no groups: an empty column of the schema's type
            out.columns.push_back(Column::host_values(dt, {}));
            continue;
        }
        if (!cols[c].empty() && cols[c][0].kind == DataValue::kSome) dt = cols[c][0].dtype;
        out.columns.push_back(Column::host_values(dt, std::move(cols[c])));
    }
    return std::make_unique<DataBlockStream>(std::vector<DataBlock>{out});
}

// LimitStream (stream_limit.rs:13-60)
namespace {
class LimitStream : public BlockStream {
   public:
    LimitStream(StreamRef in, size_t limit) : in_(std::move(in)), limit_(limit) {}
    bool next(DataBlock &out) override {
        DataBlock b;
        if (!in_->next(b)) return false;
        if (current_ == limit_) return false;
        ExecCtx &ctx = ExecCtx::current();
        b = materialize(b, ctx);
        const size_t rows = (size_t)b.num_rows();
        if (current_ + rows < limit_) {
            current_ += rows;
            out = b;
            return true;
        }
        const size_t keep = limit_ - current_;
        current_ = limit_;
        out = b;
        for (auto &c : out.columns) c = c.slice(0, (int64_t)keep);
        return true;
    }

   private:
    StreamRef in_;
    size_t limit_, current_ = 0;
};
}  // namespace

StreamRef LimitTransform::execute() { return std::make_unique<LimitStream>(input_->execute(), limit_); }

// ---------------------------------------------------------------------------
// Pipeline
// ---------------------------------------------------------------------------
void Pipeline::add_source(ProcessorRef source) {
    if (pipes_.empty()) pipes_.emplace_back();
    pipes_[0].push_back(std::move(source));
}

void Pipeline::add_simple_transform(const std::function<ProcessorRef()> &f) {
    if (pipes_.empty()) throw_internal("Can't add transform to an empty pipe list");
    std::vector<ProcessorRef> items;
    for (auto &x : pipes_.back()) {
        ProcessorRef p = f();
        p->connect_to(x);
        items.push_back(p);
    }
    pipes_.push_back(std::move(items));
}

void Pipeline::merge_processor() {
    if (pipes_.empty()) throw_internal("Can't merge processor when the last pipe is empty");
    if (pipes_.back().size() > 1) {
        // AggregatePartial pipes emit one block each (pipeline_builder.rs:73-95)
        const bool one_block = dynamic_cast<AggregatePartialTransform *>(pipes_.back()[0].get()) != nullptr;
        auto p = std::make_shared<MergeProcessor>(queues_, one_block);
        for (auto &x : pipes_.back()) p->connect_to(x);
        pipes_.push_back({p});
    }
}

StreamRef Pipeline::execute() {
    if (pipes_.empty()) throw_internal("Pipeline is empty");
    if (pipes_.back().size() > 1) merge_processor();
    return pipes_.back()[0]->execute();
}

std::string Pipeline::display() const {
    FormatterSettings s;
    std::string out;
    for (size_t k = pipes_.size(); k-- > 0;) {
        const auto &cur = pipes_[k];
        if (k > 0) {
            s.prev_ways = pipes_[k - 1].size();
            s.prev_name = pipes_[k - 1][0]->name();
        }
        s.ways = cur.size();
        s.indent += 1;
        out += cur[0]->format(s);
    }
    return out;
}

// ---------------------------------------------------------------------------
// partial-state wire format (replaces the reference's serde_json Utf8 rows,
// transform_aggregate_partial.rs:61-72): "FQS1", u32 n_funcs, then per func
// u32 n_values, u32 0, n_values x {i32 kind, i32 dtype, u64 bits}.
// ---------------------------------------------------------------------------
std::vector<uint8_t> encode_states(const std::vector<std::vector<DataValue>> &per_func) {
    std::vector<uint8_t> out(8);
    memcpy(out.data(), "FQS1", 4);
    const uint32_t nf = (uint32_t)per_func.size();
    memcpy(out.data() + 4, &nf, 4);
    for (const auto &vals : per_func) {
        uint32_t hdr[2] = {(uint32_t)vals.size(), 0};
        const size_t o = out.size();
        out.resize(o + 8 + vals.size() * 16);
        memcpy(out.data() + o, hdr, 8);
        for (size_t i = 0; i < vals.size(); ++i) {
            const DataValue &v = vals[i];
            if (v.kind == DataValue::kStruct || (v.kind == DataValue::kSome && v.dtype == FQ_DT_UTF8))
                throw_status(FQ_E_UNSUPPORTED, "partial state " + v.debug() + " has no fixed-size encoding");
            const int32_t kd[2] = {v.kind, v.kind == DataValue::kNull ? FQ_DT_NULL : v.dtype};
            memcpy(out.data() + o + 8 + i * 16, kd, 8);
            memcpy(out.data() + o + 16 + i * 16, &v.bits, 8);
        }
    }
    return out;
}

std::vector<std::vector<DataValue>> decode_states(const uint8_t *p, size_t n) {
    if (n < 8 || memcmp(p, "FQS1", 4) != 0) throw_status(FQ_E_INVALID, "partial states: bad header");
    uint32_t nf;
    memcpy(&nf, p + 4, 4);
    size_t o = 8;
    std::vector<std::vector<DataValue>> out;
    for (uint32_t f = 0; f < nf; ++f) {
        if (o + 8 > n) throw_status(FQ_E_INVALID, "partial states: truncated");
        uint32_t cnt;
        memcpy(&cnt, p + o, 4);
        o += 8;
        if (o + (size_t)cnt * 16 > n) throw_status(FQ_E_INVALID, "partial states: truncated");
        std::vector<DataValue> vals;
        for (uint32_t i = 0; i < cnt; ++i) {
            int32_t kd[2];
            uint64_t bits;
            memcpy(kd, p + o, 8);
            memcpy(&bits, p + o + 8, 8);
            o += 16;
            DataValue v;
            v.kind = kd[0];
            v.dtype = kd[1];
            v.bits = v.kind == DataValue::kSome ? bits : 0;
            vals.push_back(v);
        }
        out.push_back(std::move(vals));
    }
    return out;
}

// "FQG1", u32 n_leaves, u64 n, i32 key dtype, i32 pad, i32 leaf dtypes
// [n_leaves] (padded to 8 B), keys[n], states[leaf][n]
std::vector<uint8_t> encode_group_rows(const std::vector<std::vector<DataValue>> &rows) {
    const size_t nl = rows.empty() ? 0 : rows[0].size() - 1;
    if (!rows.empty() && rows[0].empty()) return {};
    std::vector<DataType> dts(nl, FQ_DT_NULL);
    DataType kdt = FQ_DT_NULL;
    for (const auto &r : rows) {
        if (r.size() != nl + 1) return {};
        for (size_t a = 0; a <= nl; ++a) {
            const DataValue &v = r[a];
            if (v.kind != DataValue::kSome || dtype_size(v.dtype) != 8 || v.dtype == FQ_DT_UTF8) return {};
            DataType &want = a == 0 ? kdt : dts[a - 1];
            if (want == FQ_DT_NULL) want = v.dtype;
            else if (want != v.dtype) return {};
        }
    }
    const size_t n = rows.size(), hdr = 24 + ((nl * 4 + 7) / 8) * 8;
    std::vector<uint8_t> out(hdr + n * 8 * (1 + nl));
    memcpy(out.data(), "FQG1", 4);
    const uint32_t nl32 = (uint32_t)nl;
    const uint64_t n64 = n;
    const int32_t kd[2] = {kdt, 0};
    memcpy(out.data() + 4, &nl32, 4);
    memcpy(out.data() + 8, &n64, 8);
    memcpy(out.data() + 16, kd, 8);
    for (size_t a = 0; a < nl; ++a) memcpy(out.data() + 24 + a * 4, &dts[a], 4);
    uint64_t *k = (uint64_t *)(out.data() + hdr);
    for (size_t i = 0; i < n; ++i) k[i] = rows[i][0].bits;
    for (size_t a = 0; a < nl; ++a) {
        uint64_t *s = k + (1 + a) * n;
        for (size_t i = 0; i < n; ++i) s[i] = rows[i][a + 1].bits;
    }
    return out;
}

bool is_group_rows(const uint8_t *p, size_t n) { return n >= 24 && memcmp(p, "FQG1", 4) == 0; }

GroupRows decode_group_rows(const uint8_t *p, size_t n) {
    if (!is_group_rows(p, n)) throw_status(FQ_E_INVALID, "GROUP BY partial rows: bad header");
    uint32_t nl;
    uint64_t rows;
    int32_t kd[2];
    memcpy(&nl, p + 4, 4);
    memcpy(&rows, p + 8, 8);
    memcpy(kd, p + 16, 8);
    const size_t hdr = 24 + ((size_t)nl * 4 + 7) / 8 * 8;
    // by division: `rows` comes off the wire and a product could wrap
    if (nl > FQ_MAX_GROUP_AGGS || hdr > n || rows > (n - hdr) / (8 * (1 + (uint64_t)nl)))
        throw_status(FQ_E_INVALID, "GROUP BY partial rows: truncated");
    GroupRows g;
    g.key_dtype = kd[0];
    g.dtypes.resize(nl);
    for (uint32_t a = 0; a < nl; ++a) memcpy(&g.dtypes[a], p + 24 + a * 4, 4);
    const uint64_t *k = (const uint64_t *)(p + hdr);
    g.keys.assign(k, k + rows);
    g.st.resize(nl);
    for (uint32_t a = 0; a < nl; ++a) g.st[a].assign(k + (1 + a) * rows, k + (2 + a) * rows);
    return g;
}

}  // namespace fq
