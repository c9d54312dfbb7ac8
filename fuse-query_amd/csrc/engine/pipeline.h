// Processors, streams and pipeline (src/processors/, src/transforms/,
// src/datastreams/, src/datasources/) restated for device DataBlocks.
//
// One host thread per pipe replaces the reference's tokio task per pipe
// (processor_merge.rs:45-63); each thread binds an ExecCtx (device queue +
// scan workspace).  Blocks flow by pull (BlockStream::next) as in the
// reference's Stream::poll_next; errors are exceptions forwarded through the
// MergeProcessor channel like the reference forwards Err items.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "core.h"
#include "functions.h"

namespace fq {

// ---------------------------------------------------------------------------
// streams (SendableDataBlockStream, stream.rs:8-9)
// ---------------------------------------------------------------------------
class BlockStream {
   public:
    virtual ~BlockStream() = default;
    virtual bool next(DataBlock &out) = 0;  // false = end of stream; throws on error
};
using StreamRef = std::unique_ptr<BlockStream>;

// DataBlockStream (stream_datablock.rs:13-60)
class DataBlockStream : public BlockStream {
   public:
    explicit DataBlockStream(std::vector<DataBlock> blocks) : blocks_(std::move(blocks)) {}
    bool next(DataBlock &out) override {
        if (i_ >= blocks_.size()) return false;
        out = std::move(blocks_[i_++]);  // read once: the consumer gets the only reference
        return true;
    }

   private:
    std::vector<DataBlock> blocks_;
    size_t i_ = 0;
};

// ---------------------------------------------------------------------------
// data sources (src/datasources/)
// ---------------------------------------------------------------------------
struct Partition {  // partition.rs:5-11
    std::string name;
    uint64_t version = 0;
};

struct ReadDataSourcePlan {  // plan_read_datasource.rs
    std::string db, table, table_type, description;
    SchemaRef schema;
    std::vector<Partition> partitions;
};

// How a table yields a partition's rows (the same rows, in order, always):
//   kWhole    aggregates: a resident partition as one block, a generated one in
//             chunk_rows() pieces (bounded HBM)
//   kChunks   row pipelines without LIMIT: pieces of at most chunk_rows() rows,
//             resident or not, so the projected blocks in flight stay bounded
//   kMorsels  row pipelines with LIMIT: growing morsels, so a satisfied LIMIT
//             stops the scan early (stream_limit.rs:28-48)
enum class ReadMode { kWhole, kChunks, kMorsels };

class ITable {  // table.rs:13-22
   public:
    virtual ~ITable() = default;
    virtual std::string name() const = 0;
    virtual SchemaRef schema() const = 0;
    virtual ReadDataSourcePlan read_plan(const DataValue *table_arg) const = 0;
    virtual StreamRef read(const std::vector<Partition> &parts, ReadMode mode = ReadMode::kWhole) = 0;
};
using TableRef = std::shared_ptr<ITable>;

// system.numbers_mt (numbers_table.rs:14-97, numbers_stream.rs:20-84) with
// partitions optionally pinned in HBM.
class NumbersTable : public ITable {
   public:
    NumbersTable();
    std::string name() const override { return "numbers_mt"; }
    SchemaRef schema() const override { return schema_; }
    ReadDataSourcePlan read_plan(const DataValue *table_arg) const override;
    StreamRef read(const std::vector<Partition> &parts, ReadMode mode = ReadMode::kWhole) override;
    // morsel sizes: the first is kMorselFirst rows, each next one twice the
    // last up to kMorselMax (multiples of the 10,000-row block)
    static constexpr uint64_t kMorselFirst = 160000;
    static constexpr uint64_t kMorselMax = 327680000;

    static std::vector<Partition> generate_parts(uint64_t total);
    static void parse_part(const std::string &name, uint64_t &total, uint64_t &begin, uint64_t &end);
    static uint64_t stream_rows(uint64_t begin, uint64_t end);  // rows NumbersStream yields
    void pin(const std::string &part, Column col);
    // device block size for partitions that are not resident (FQ_OPT_CHUNK_ROWS)
    void set_chunk_rows(uint64_t r) { chunk_rows_ = r; }
    uint64_t chunk_rows() const { return chunk_rows_; }
    void unpin_all();
    bool pinned(const std::string &part, Column &out);

   private:
    SchemaRef schema_;
    std::mutex mu_;
    std::map<std::string, Column> resident_;
    std::atomic<uint64_t> chunk_rows_{400000000};
};

class DataSource {  // datasource.rs:11-62
   public:
    DataSource();
    TableRef get_table(const std::string &db, const std::string &table) const;
    std::shared_ptr<NumbersTable> numbers() const { return numbers_; }

   private:
    std::map<std::string, std::map<std::string, TableRef>> dbs_;
    std::shared_ptr<NumbersTable> numbers_;
};

// FuseQueryContext (context.rs:10-37) + the engine's execution knobs
struct QueryContext {
    size_t worker_threads = 8;
    std::string default_db = "default";
    std::shared_ptr<DataSource> datasource;
    FactoryOptions factory;
    Runtime *rt = nullptr;
    int rank = 0, world = 1;  // distributed partial: this rank's partition shard
    TableRef get_table(const std::string &db, const std::string &table) const {
        return datasource->get_table(db, table);
    }
};
using QueryContextRef = std::shared_ptr<QueryContext>;

// ---------------------------------------------------------------------------
// processors (processor.rs:22-57)
// ---------------------------------------------------------------------------
struct FormatterSettings {
    size_t ways = 0, indent = 0;
    std::string indent_char = "  ", prefix = "\xe2\x94\x94\xe2\x94\x80";  // "└─"
    size_t prev_ways = 0;
    std::string prev_name;
};

class IProcessor {
   public:
    virtual ~IProcessor() = default;
    virtual std::string name() const = 0;
    virtual void connect_to(std::shared_ptr<IProcessor> input) = 0;
    virtual StreamRef execute() = 0;
    virtual std::string format(FormatterSettings &s) const;
    // the pipe this processor ends failed before (or without) running
    // execute(): release whatever other pipes wait on (MergeProcessor calls it
    // from the failing pipe's task; transforms pass it to their input)
    virtual void abandon() {}
};
using ProcessorRef = std::shared_ptr<IProcessor>;

class EmptyProcessor : public IProcessor {  // processor_empty.rs:14-49
   public:
    std::string name() const override { return "EmptyProcessor"; }
    void connect_to(ProcessorRef) override { throw_internal("Cannot call EmptyProcessor connect_to"); }
    StreamRef execute() override { return std::make_unique<DataBlockStream>(std::vector<DataBlock>{}); }
    std::string format(FormatterSettings &) const override { return ""; }
};

class MergeProcessor : public IProcessor {  // processor_merge.rs:16-94
   public:
    explicit MergeProcessor(QueueKind queues = QueueKind::kShared, bool inline_first = false)
        : queues_(queues), inline_first_(inline_first) {}
    std::string name() const override { return "MergeProcessor"; }
    void connect_to(ProcessorRef input) override { list_.push_back(std::move(input)); }
    StreamRef execute() override;
    std::string format(FormatterSettings &s) const override;

   private:
    std::vector<ProcessorRef> list_;
    QueueKind queues_;    // the input pipes' device queues (kRow: pipe p on row queue p)
    bool inline_first_;   // pipe 0 runs on the calling thread (one-block pipes)
};

class SourceTransform : public IProcessor {  // transform_source.rs:14-53
   public:
    SourceTransform(QueryContextRef ctx, std::string db, std::string table, std::vector<Partition> parts,
                    ReadMode mode = ReadMode::kWhole)
        : ctx_(std::move(ctx)), db_(std::move(db)), table_(std::move(table)), parts_(std::move(parts)), mode_(mode) {}
    std::string name() const override { return "SourceTransform"; }
    void connect_to(ProcessorRef) override { throw_internal("Cannot call SourceTransform connect_to"); }
    StreamRef execute() override;

   private:
    QueryContextRef ctx_;
    std::string db_, table_;
    std::vector<Partition> parts_;
    ReadMode mode_;
};

class FilterTransform : public IProcessor {  // transform_filter.rs:17-77
   public:
    explicit FilterTransform(FunctionRef pred) : func_(std::move(pred)), input_(std::make_shared<EmptyProcessor>()) {}
    std::string name() const override { return "FilterTransform"; }
    void connect_to(ProcessorRef input) override { input_ = std::move(input); }
    StreamRef execute() override;
    void abandon() override { input_->abandon(); }

   private:
    FunctionRef func_;
    ProcessorRef input_;
};

class ProjectionTransform : public IProcessor {  // transform_projection.rs:16-78
   public:
    // block_stream: a filtered numbers stream is projected into the reference's
    // per-block geometry (fq_filter_project_blocks); false -- a LIMIT above
    // compacts every block anyway and wants latency -- one contiguous array
    // per block (fq_filter_project)
    // span: the query's block-stream projections timed together (LaunchSpan)
    ProjectionTransform(SchemaRef schema, std::vector<FunctionRef> funcs, bool block_stream = true,
                        LaunchSpanRef span = nullptr)
        : schema_(std::move(schema)), funcs_(std::move(funcs)), input_(std::make_shared<EmptyProcessor>()),
          block_stream_(block_stream), span_(std::move(span)) {}
    std::string name() const override { return "ProjectionTransform"; }
    void connect_to(ProcessorRef input) override { input_ = std::move(input); }
    StreamRef execute() override;
    void abandon() override;  // a pipe that never ran still counts in the span

   private:
    SchemaRef schema_;
    std::vector<FunctionRef> funcs_;
    ProcessorRef input_;
    bool block_stream_;
    LaunchSpanRef span_;
    std::atomic<bool> entered_{false};
};

class AggregatePartialTransform : public IProcessor {  // transform_aggregate_partial.rs:18-79
   public:
    // group: the query's AggregatePartial pipes (they wait for their scans together)
    AggregatePartialTransform(SchemaRef schema, std::vector<FunctionRef> funcs, ScanGroupRef group = nullptr)
        : schema_(std::move(schema)), funcs_(std::move(funcs)), input_(std::make_shared<EmptyProcessor>()),
          group_(std::move(group)) {}
    std::string name() const override { return "AggregatePartialTransform"; }
    void connect_to(ProcessorRef input) override { input_ = std::move(input); }
    StreamRef execute() override;
    // a pipe whose ExecCtx could not be set up never reaches execute(): its
    // place in the scan group arrives here, so the other pipes' deferred
    // states (ScanGroup::wait_end) do not wait for it
    void abandon() override;

   private:
    SchemaRef schema_;
    std::vector<FunctionRef> funcs_;
    ProcessorRef input_;
    ScanGroupRef group_;
    std::atomic<bool> entered_{false};  // execute() took this pipe's ScanTicket
};

class AggregateFinalTransform : public IProcessor {  // transform_aggregate_final.rs:18-79
   public:
    // emit_states: output the merged accumulate_result() (for a cross-GPU
    // exchange) instead of merge_result() values.
    AggregateFinalTransform(SchemaRef schema, std::vector<FunctionRef> funcs, bool emit_states = false)
        : schema_(std::move(schema)), funcs_(std::move(funcs)), input_(std::make_shared<EmptyProcessor>()),
          emit_states_(emit_states) {}
    std::string name() const override { return "AggregateFinalTransform"; }
    void connect_to(ProcessorRef input) override { input_ = std::move(input); }
    StreamRef execute() override;

   private:
    SchemaRef schema_;
    std::vector<FunctionRef> funcs_;
    ProcessorRef input_;
    bool emit_states_;
};

// GROUP BY.  The reference plans group_expr but has no
// transform for it (pipeline_builder.rs:50-66 builds AggregatePartial/Final
// from aggr_expr only).  Here every pipe streams its blocks into ONE device
// hash table per query (fq_group_aggregate: key = the group expression's
// fused chain, one state per AggregatorFunction leaf of the aggregate
// expressions), and the final transform extracts the groups, sorts them by
// key and evaluates each aggregate expression per group from its leaves'
// states (merge_result over the Function tree).
struct GroupByShared {
    std::mutex mu;
    bool ready = false;
    fq_group_table desc{};
    std::shared_ptr<DeviceBuffer> mem;
    std::vector<uint32_t> leaf_ops;  // per table aggregate
    bool dummy_count = false;        // no aggregate: a Count keeps the table valid
    int log2_parts = 0;              // > 0: radix-partitioned launches (high cardinality)
    int64_t blocks_hint = 1;         // numbers_mt partitions of this rank (planner)
    // their workspace (~8 B per row), one per device queue: the pipes that
    // share a queue run its launches in order, so they share the memory
    // instead of mapping a fresh block per pipe
    std::map<hipStream_t, std::shared_ptr<DeviceBuffer>> part_ws;
};

class GroupByPartialTransform : public IProcessor {
   public:
    GroupByPartialTransform(FunctionRef key, std::vector<FunctionRef> funcs, std::shared_ptr<GroupByShared> shared)
        : key_(std::move(key)), funcs_(std::move(funcs)), shared_(std::move(shared)),
          input_(std::make_shared<EmptyProcessor>()) {}
    // the reference builds AggregatePartial/Final for a grouped plan too
    // (pipeline_builder.rs:50-66), so EXPLAIN shows the same processors
    std::string name() const override { return "AggregatePartialTransform"; }
    void connect_to(ProcessorRef input) override { input_ = std::move(input); }
    StreamRef execute() override;

   private:
    FunctionRef key_;
    std::vector<FunctionRef> funcs_;
    std::shared_ptr<GroupByShared> shared_;
    ProcessorRef input_;
};

class GroupByFinalTransform : public IProcessor {
   public:
    GroupByFinalTransform(SchemaRef schema, std::vector<FunctionRef> funcs, std::shared_ptr<GroupByShared> shared,
                          bool emit_states)
        : schema_(std::move(schema)), funcs_(std::move(funcs)), shared_(std::move(shared)),
          input_(std::make_shared<EmptyProcessor>()), emit_states_(emit_states) {}
    std::string name() const override { return "AggregateFinalTransform"; }
    void connect_to(ProcessorRef input) override { input_ = std::move(input); }
    StreamRef execute() override;

   private:
    SchemaRef schema_;
    std::vector<FunctionRef> funcs_;
    std::shared_ptr<GroupByShared> shared_;
    ProcessorRef input_;
    bool emit_states_;
};

class LimitTransform : public IProcessor {  // transform_limit.rs:12-43
   public:
    explicit LimitTransform(size_t n) : limit_(n), input_(std::make_shared<EmptyProcessor>()) {}
    std::string name() const override { return "LimitTransform"; }
    void connect_to(ProcessorRef input) override { input_ = std::move(input); }
    StreamRef execute() override;
    void abandon() override { input_->abandon(); }

   private:
    size_t limit_;
    ProcessorRef input_;
};

// A processor yielding prepared blocks (AggregateFinal input across GPUs).
class BlocksProcessor : public IProcessor {
   public:
    explicit BlocksProcessor(std::vector<DataBlock> b) : blocks_(std::move(b)) {}
    std::string name() const override { return "ExchangeSource"; }
    void connect_to(ProcessorRef) override { throw_internal("Cannot call ExchangeSource connect_to"); }
    StreamRef execute() override { return std::make_unique<DataBlockStream>(blocks_); }

   private:
    std::vector<DataBlock> blocks_;
};

// ---------------------------------------------------------------------------
// Pipeline (pipeline.rs:15-135)
// ---------------------------------------------------------------------------
class Pipeline {
   public:
    size_t pipe_num() const { return pipes_.empty() ? 0 : pipes_.back().size(); }
    void add_source(ProcessorRef source);
    void add_simple_transform(const std::function<ProcessorRef()> &f);
    void merge_processor();
    StreamRef execute();
    std::string display() const;
    // row pipelines (no aggregate): merged pipes run on private device queues
    void set_queues(QueueKind k) { queues_ = k; }

   private:
    std::vector<std::vector<ProcessorRef>> pipes_;
    QueueKind queues_ = QueueKind::kShared;
};

// serialised partial states (one 16-byte record per DataValue)
std::vector<uint8_t> encode_states(const std::vector<std::vector<DataValue>> &per_func);
std::vector<std::vector<DataValue>> decode_states(const uint8_t *p, size_t n);

// GROUP BY partial states as flat arrays ("FQG1"): rows [key, leaf states...]
// that are all 64-bit Some values -- what a GPU table holds -- travel as
// keys[n] + states[leaf][n] (8 B per value instead of a 16-B DataValue record),
// and the final merges them on the device (fq_group_table_merge).
struct GroupRows {
    DataType key_dtype = FQ_DT_NULL;
    std::vector<DataType> dtypes;           // per leaf
    std::vector<uint64_t> keys;             // n
    std::vector<std::vector<uint64_t>> st;  // [leaf][n]
};
// empty when some row is not encodable (a None state, a Struct, Utf8 ...)
std::vector<uint8_t> encode_group_rows(const std::vector<std::vector<DataValue>> &rows);
bool is_group_rows(const uint8_t *p, size_t n);
GroupRows decode_group_rows(const uint8_t *p, size_t n);

}  // namespace fq
