// The reference's expression tree (src/functions/), restated over device
// columns.  `Function` keeps the reference's method set exactly
// (function.rs:28-131: return_type, nullable, eval, set_depth, accumulate,
// accumulate_result, merge_state, merge_result) with its depth-indexed state
// merging (plan_expression.rs:40-60, function_arithmetic.rs:48-52); two
// extra hooks describe fusable shapes to the device scan (to_chain/to_pred).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "core.h"

namespace fq {

// An ArithmeticFunction tree expressed as fq_expr over one column.
struct FusedChain {
    std::string column;
    DataType col_dtype = FQ_DT_NULL;
    fq_expr expr{};
    DataType out_dtype = FQ_DT_NULL;
    int depth = 0;  // value-stack depth the expression tree needs (FQ_OP_PUSH)
    std::string key() const;
};

// A ComparisonFunction (or an and/or tree of them, FQ_PRED_TREE) expressed
// as fq_pred over one column.
struct FusedPred {
    std::string column;
    DataType col_dtype = FQ_DT_NULL;
    fq_pred pred{};
    fq_pred_tree tree{};  // kind == FQ_PRED_TREE
    std::string key() const;
    // the fq_pred to hand to the ABI (points pred.tree at this object's tree)
    const fq_pred *get() {
        pred.tree = pred.kind == FQ_PRED_TREE ? &tree : nullptr;
        return &pred;
    }
};

class Function;
class AggregatorFunction;
using FunctionRef = std::shared_ptr<Function>;

class Function {
   public:
    virtual ~Function() = default;
    virtual std::string display() const = 0;  // fmt::Debug of Function (function.rs:134-146)
    virtual DataType return_type(const DataSchema &s) const = 0;
    virtual bool nullable(const DataSchema &s) const = 0;
    virtual ColumnarValue eval(const DataBlock &b, ExecCtx &ctx) = 0;
    virtual void set_depth(size_t depth) = 0;
    virtual void accumulate(const DataBlock &b, ExecCtx &ctx) = 0;
    virtual std::vector<DataValue> accumulate_result() const = 0;
    virtual void merge_state(const std::vector<DataValue> &states) = 0;
    virtual DataValue merge_result() const = 0;
    virtual FunctionRef clone() const = 0;

    // fusion hooks (not in the reference: describe the shape, no semantics)
    virtual bool to_chain(const DataSchema &, FusedChain &) const { return false; }
    virtual bool to_pred(const DataSchema &, FusedPred &) const { return false; }
    virtual const DataValue *as_constant() const { return nullptr; }
    virtual const std::string *as_field() const { return nullptr; }
    // the AggregatorFunction leaves of this tree, left to right (GROUP BY
    // evaluates the tree per group from device states)
    virtual void collect_aggregators(std::vector<AggregatorFunction *> &) {}
};

// FieldFunction (function_field.rs:13-73)
class FieldFunction : public Function {
   public:
    explicit FieldFunction(std::string name) : name_(std::move(name)) {}
    std::string display() const override { return name_; }
    DataType return_type(const DataSchema &s) const override;
    bool nullable(const DataSchema &s) const override;
    ColumnarValue eval(const DataBlock &b, ExecCtx &ctx) override;
    void set_depth(size_t d) override { depth_ = d; }
    void accumulate(const DataBlock &b, ExecCtx &ctx) override;
    std::vector<DataValue> accumulate_result() const override;
    void merge_state(const std::vector<DataValue> &) override;
    DataValue merge_result() const override;
    FunctionRef clone() const override { return std::make_shared<FieldFunction>(*this); }
    bool to_chain(const DataSchema &s, FusedChain &c) const override;
    const std::string *as_field() const override { return &name_; }

   private:
    size_t depth_ = 0;
    std::string name_;
};

// ConstantFunction (function_constant.rs:13-51)
class ConstantFunction : public Function {
   public:
    explicit ConstantFunction(DataValue v) : value_(std::move(v)) {}
    std::string display() const override { return value_.debug(); }
    DataType return_type(const DataSchema &) const override { return value_.data_type(); }
    bool nullable(const DataSchema &) const override { return value_.is_none(); }
    ColumnarValue eval(const DataBlock &b, ExecCtx &ctx) override;
    void set_depth(size_t) override {}
    void accumulate(const DataBlock &, ExecCtx &) override {}
    std::vector<DataValue> accumulate_result() const override { return {value_}; }
    void merge_state(const std::vector<DataValue> &) override {}
    DataValue merge_result() const override { return value_; }
    FunctionRef clone() const override { return std::make_shared<ConstantFunction>(*this); }
    const DataValue *as_constant() const override { return &value_; }

   private:
    DataValue value_;
};

// AliasFunction (function_alias.rs:13-59)
class AliasFunction : public Function {
   public:
    AliasFunction(std::string alias, FunctionRef f) : alias_(std::move(alias)), func_(std::move(f)) {}
    std::string display() const override { return alias_; }
    DataType return_type(const DataSchema &s) const override { return func_->return_type(s); }
    bool nullable(const DataSchema &s) const override { return func_->nullable(s); }
    ColumnarValue eval(const DataBlock &b, ExecCtx &ctx) override { return func_->eval(b, ctx); }
    void set_depth(size_t d) override { depth_ = d; }
    void accumulate(const DataBlock &b, ExecCtx &ctx) override { func_->accumulate(b, ctx); }
    std::vector<DataValue> accumulate_result() const override { return func_->accumulate_result(); }
    void merge_state(const std::vector<DataValue> &s) override { func_->merge_state(s); }
    DataValue merge_result() const override { return func_->merge_result(); }
    FunctionRef clone() const override { return std::make_shared<AliasFunction>(alias_, func_->clone()); }
    bool to_chain(const DataSchema &s, FusedChain &c) const override { return func_->to_chain(s, c); }
    bool to_pred(const DataSchema &s, FusedPred &p) const override { return func_->to_pred(s, p); }
    void collect_aggregators(std::vector<AggregatorFunction *> &v) override { func_->collect_aggregators(v); }

   private:
    size_t depth_ = 0;
    std::string alias_;
    FunctionRef func_;
};

// ArithmeticFunction (function_arithmetic.rs:16-89); op FQ_OP_MOD is the '%' extension
class ArithmeticFunction : public Function {
   public:
    ArithmeticFunction(int32_t op, FunctionRef l, FunctionRef r) : op_(op), left_(std::move(l)), right_(std::move(r)) {}
    std::string display() const override;
    DataType return_type(const DataSchema &s) const override;
    bool nullable(const DataSchema &) const override { return false; }
    ColumnarValue eval(const DataBlock &b, ExecCtx &ctx) override;
    void set_depth(size_t d) override {
        left_->set_depth(d);
        right_->set_depth(d + 1);
        depth_ = d;
    }
    void accumulate(const DataBlock &b, ExecCtx &ctx) override {
        left_->accumulate(b, ctx);
        right_->accumulate(b, ctx);
    }
    std::vector<DataValue> accumulate_result() const override;
    void merge_state(const std::vector<DataValue> &s) override {
        left_->merge_state(s);
        right_->merge_state(s);
    }
    DataValue merge_result() const override;
    FunctionRef clone() const override {
        auto f = std::make_shared<ArithmeticFunction>(op_, left_->clone(), right_->clone());
        f->depth_ = depth_;
        return f;
    }
    bool to_chain(const DataSchema &s, FusedChain &c) const override;
    void collect_aggregators(std::vector<AggregatorFunction *> &v) override {
        left_->collect_aggregators(v);
        right_->collect_aggregators(v);
    }

   private:
    size_t depth_ = 0;
    int32_t op_;
    FunctionRef left_, right_;
};

// ComparisonFunction (function_comparison.rs:17-86)
class ComparisonFunction : public Function {
   public:
    ComparisonFunction(int32_t cmp, FunctionRef l, FunctionRef r) : cmp_(cmp), left_(std::move(l)), right_(std::move(r)) {}
    std::string display() const override;
    DataType return_type(const DataSchema &) const override { return FQ_DT_BOOLEAN; }
    bool nullable(const DataSchema &) const override { return false; }
    ColumnarValue eval(const DataBlock &b, ExecCtx &ctx) override;
    void set_depth(size_t d) override { depth_ = d; }
    void accumulate(const DataBlock &b, ExecCtx &ctx) override {
        left_->accumulate(b, ctx);
        right_->accumulate(b, ctx);
    }
    std::vector<DataValue> accumulate_result() const override;
    void merge_state(const std::vector<DataValue> &) override;
    DataValue merge_result() const override;
    FunctionRef clone() const override {
        auto f = std::make_shared<ComparisonFunction>(cmp_, left_->clone(), right_->clone());
        f->depth_ = depth_;
        return f;
    }
    bool to_pred(const DataSchema &s, FusedPred &p) const override;
    void collect_aggregators(std::vector<AggregatorFunction *> &v) override {
        left_->collect_aggregators(v);
        right_->collect_aggregators(v);
    }

   private:
    size_t depth_ = 0;
    int32_t cmp_;
    FunctionRef left_, right_;
};

// LogicFunction (function_logic.rs:17-87): and/or of two Boolean arrays
class LogicFunction : public Function {
   public:
    LogicFunction(int32_t op, FunctionRef l, FunctionRef r) : op_(op), left_(std::move(l)), right_(std::move(r)) {}
    std::string display() const override;
    DataType return_type(const DataSchema &) const override { return FQ_DT_BOOLEAN; }
    bool nullable(const DataSchema &) const override { return false; }
    ColumnarValue eval(const DataBlock &b, ExecCtx &ctx) override;
    void set_depth(size_t d) override { depth_ = d; }
    void accumulate(const DataBlock &b, ExecCtx &ctx) override {
        left_->accumulate(b, ctx);
        right_->accumulate(b, ctx);
    }
    std::vector<DataValue> accumulate_result() const override;
    void merge_state(const std::vector<DataValue> &) override;
    DataValue merge_result() const override;
    FunctionRef clone() const override {
        auto f = std::make_shared<LogicFunction>(op_, left_->clone(), right_->clone());
        f->depth_ = depth_;
        return f;
    }
    void collect_aggregators(std::vector<AggregatorFunction *> &v) override {
        left_->collect_aggregators(v);
        right_->collect_aggregators(v);
    }
    bool to_pred(const DataSchema &s, FusedPred &p) const override;
    int32_t op() const { return op_; }
    const Function &left() const { return *left_; }
    const Function &right() const { return *right_; }

   private:
    size_t depth_ = 0;
    int32_t op_;  // FQ_LOGIC_AND / FQ_LOGIC_OR
    FunctionRef left_, right_;
};

// AggregatorFunction (function_aggregator.rs:17-144)
class AggregatorFunction : public Function {
   public:
    AggregatorFunction(uint32_t op, FunctionRef arg) : op_(op), arg_(std::move(arg)) {}
    std::string display() const override;
    DataType return_type(const DataSchema &s) const override;
    bool nullable(const DataSchema &) const override { return false; }
    ColumnarValue eval(const DataBlock &b, ExecCtx &ctx) override { return arg_->eval(b, ctx); }
    void set_depth(size_t d) override { depth_ = d; }
    void accumulate(const DataBlock &b, ExecCtx &ctx) override;
    std::vector<DataValue> accumulate_result() const override { return {state_}; }
    void merge_state(const std::vector<DataValue> &states) override;
    DataValue merge_result() const override { return state_; }
    FunctionRef clone() const override {
        auto f = std::make_shared<AggregatorFunction>(op_, arg_->clone());
        f->depth_ = depth_;
        f->state_ = state_;
        return f;
    }

    uint32_t op() const { return op_; }
    const Function &arg() const { return *arg_; }
    void collect_aggregators(std::vector<AggregatorFunction *> &v) override { v.push_back(this); }
    // GROUP BY: this group's state, as accumulate would have left it
    void set_state(const DataValue &v) { state_ = v; }
    // Replays the reference's per-block accumulate over a run of `st.blocks`
    // reference blocks summarised by one device scan (see fq_agg_state).
    void accumulate_summary(const fq_agg_state &st);
    // Non-deferred evaluation of this aggregator over one block.
    fq_agg_state summarize(const DataBlock &b, ExecCtx &ctx);

   private:
    size_t depth_ = 0;
    uint32_t op_;
    FunctionRef arg_;
    DataValue state_;  // DataValue::Null initially (function_aggregator.rs:29)
};

// ScalarFunctionFactory::get (function_factory.rs:14-40)
struct FactoryOptions {
    bool modulo = true;  // '%' extension
};
FunctionRef function_factory(const std::string &name, std::vector<FunctionRef> args, const FactoryOptions &o);

// The AggregatePartial pipes of ONE query (pipeline_builder.rs:50-66 builds one
// per source pipe) when they share one device queue.  Their scans run back to
// back there; a completion event behind each pipe's scans would sit between
// two scans (~9 us of idle queue each, profiles/r02_gap_probe_event_flags.txt).
// Instead every pipe arrives here once it has enqueued its scans (or failed);
// the pipe that arrives last records ONE event behind all of them, and every
// pipe that launched waits on it -- the partial states are needed together by
// AggregateFinal anyway (transform_aggregate_final.rs:50-66).
// FQ_OPT_PROFILE = 2 (span): one timing event before the query's first scan,
// so scan_ns gets (first scan start .. last scan end) once per query -- the
// scans and the launch gaps between them, nothing else on a resident column.
class ScanGroup {
   public:
    ScanGroup(Runtime *rt, int pipes) : rt_(rt), left_(pipes) {}
    ~ScanGroup();
    ScanGroup(const ScanGroup &) = delete;
    ScanGroup &operator=(const ScanGroup &) = delete;
    // a launch on ctx's queue follows (called under the queue's launch lock)
    void before_launch(ExecCtx &ctx);
    // a pipe has enqueued everything it will (or failed, or never started).
    // The last one to arrive records an end event on every queue the group
    // launched on; with `wait` the others block until it has (a failing pipe
    // leaves without waiting).  Never throws: a failure to record an end event
    // is kept and reported by wait_end, and the group closes either way, so no
    // pipe waits for a group that cannot close (it runs from destructors).
    void arrive(bool wait) noexcept;
    // every queue the group launched on, done (after arrive)
    void wait_end();
    // after wait_end: the spans' time into scan_ns (once per query)
    void account();

   private:
    struct QueueSpan {
        hipStream_t q = nullptr;
        std::mutex *launch_mu = nullptr;
        hipEvent_t start = nullptr, end = nullptr;
    };
    Runtime *rt_;
    std::mutex mu_;
    std::condition_variable cv_;
    int left_;
    bool closed_ = false, accounted_ = false;
    bool waiter_ = false, ended_ = false;  // wait_end: one pipe waits on the events
    hipError_t end_error_ = hipSuccess;
    std::string arrive_error_;       // the last arrival could not record an end event
    std::vector<QueueSpan> queues_;  // stable once every pipe has arrived
};
using ScanGroupRef = std::shared_ptr<ScanGroup>;

// The block-stream projections of ONE query (a row pipeline's
// ProjectionTransform pipes, fq_filter_project_blocks) timed as one span,
// like ScanGroup's scans: FQ_OPT_PROFILE 2 records a start event right before
// each queue's first launch of the query and, when the last pipe's stream has
// ended, an end event per queue -- project_ns gets the union of the queues'
// spans, earliest start to latest end (the launches, overlapped across the
// row queues, and every gap); no event sits between two launches.  (The end
// is recorded once that pipe has seen its last launch complete, so the span
// also holds that pipe's wake-up: it over-states, never under-states.)
class LaunchSpan {
   public:
    LaunchSpan(Runtime *rt, int pipes) : rt_(rt), left_(pipes) {}
    ~LaunchSpan();
    LaunchSpan(const LaunchSpan &) = delete;
    LaunchSpan &operator=(const LaunchSpan &) = delete;
    // a launch on ctx's queue follows (under the queue's launch lock)
    void before_launch(ExecCtx &ctx);
    // a pipe's stream has ended (or the pipe is gone); never throws
    void arrive() noexcept;

   private:
    struct QueueSpan {
        hipStream_t q = nullptr;
        std::mutex *launch_mu = nullptr;
        hipEvent_t start = nullptr;
    };
    Runtime *rt_;
    std::mutex mu_;
    int left_;
    std::vector<QueueSpan> queues_;
};
using LaunchSpanRef = std::shared_ptr<LaunchSpan>;

// One pipe's place in a ScanGroup: arrives exactly once -- from
// AggFusion::finish, or (a pipe that fails) when it goes out of scope, so the
// other pipes never wait for a pipe that is gone.  A pipe that fails before
// it makes its ticket (its ExecCtx could not be set up) arrives through
// AggregatePartialTransform::abandon instead.
class ScanTicket {
   public:
    explicit ScanTicket(ScanGroup *g) : g_(g) {}
    ~ScanTicket() {
        if (g_ && !done_) g_->arrive(false);
    }
    ScanTicket(const ScanTicket &) = delete;
    ScanTicket &operator=(const ScanTicket &) = delete;
    ScanGroup *group() const { return g_; }
    // this pipe has enqueued all its scans; launched: wait for the query's end
    void arrive(bool launched) {
        if (!g_ || done_) return;
        done_ = true;
        g_->arrive(launched);
        if (launched) {
            g_->wait_end();
            g_->account();
        }
    }
    // the same without waiting: the pipe's states are read later, by whoever
    // calls wait_end() (AggregatePartial's deferred block)
    void arrive_only() {
        if (!g_ || done_) return;
        done_ = true;
        g_->arrive(false);
    }

   private:
    ScanGroup *g_;
    bool done_ = false;
};

// Deferred, fused accumulate for AggregatePartialTransform: aggregators that
// share an argument expression (and the block's pending predicate) are served
// by ONE fq_aggregate scan per block; results are replayed into each
// aggregator in the reference's (block, function) order at finish().
class AggFusion {
   public:
    explicit AggFusion(ExecCtx &ctx, ScanTicket *ticket = nullptr);
    ~AggFusion();
    void add(AggregatorFunction *agg, const DataBlock &b);
    void add_error(const FQException &e);  // a non-aggregator failure at this point
    void end_block();                      // launch this block's scans
    void finish();                         // sync + replay; throws the first error
    // In a scan group: launch the last block's scans and arrive at the group
    // without waiting.  true: the caller keeps this object (and the context's
    // WorkerRes, ExecCtx::lease) and calls replay() after the group's
    // wait_end(), on any thread; false: nothing launched, call finish().
    bool finish_deferred();
    void replay();  // the scans have ended: states -> aggregators; throws the first error

   private:
    struct Group {
        std::string key;
        Column col;
        FusedChain value;
        bool has_pred = false;
        FusedPred pred;
        std::shared_ptr<Function> filter_keepalive;
        uint32_t mask = 0;
        int64_t block_rows = 0;
        uint64_t blocks = 0;
        size_t slot = 0;
    };
    struct Entry {
        AggregatorFunction *agg = nullptr;
        size_t slot = (size_t)-1;  // device result slot, or
        fq_agg_state st{};         // an immediate summary
        bool has_error = false;
        FQException err{0, ""};
    };
    ExecCtx &ctx_;  // the pipe's context: add() / end_block() only
    // what finish / replay / the destructor use, valid while the WorkerRes is
    // held (the context, or its lease)
    Runtime *rt_;
    WorkerRes *res_;
    hipStream_t stream_;
    std::mutex *launch_mu_;
    ScanTicket *ticket_ = nullptr;  // the query's pipes wait together (ScanGroup)
    std::vector<Group> cur_;
    std::vector<Entry> log_;
    std::vector<Column> keepalive_;
    size_t nslots_ = 0;
    bool launched_ = false, finished_ = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events_;
    size_t alloc_slot();
    fq_agg_state *slot_host(size_t k) const;
    void wait_launched();
};

// evaluate a predicate over a block into a Boolean column (one fused kernel
// when the predicate is a chain over one 64-bit column, else per node)
Column eval_predicate(Function &pred, const DataBlock &b, ExecCtx &ctx);

// ProjectionTransform's expressions (and the block's pending filter) through
// one fq_filter_project call; false when the shape is not fusable
bool project_fused(const DataBlock &b, const std::vector<FunctionRef> &funcs, const SchemaRef &schema, ExecCtx &ctx,
                   DataBlock &out,
                   bool block_stream = true,
                   LaunchSpan *span = nullptr);

}  // namespace fq
