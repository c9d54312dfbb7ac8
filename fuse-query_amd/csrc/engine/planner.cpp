// SQL subset -> PlanNode list -> Pipeline (see planner.h).
#include "planner.h"

#include <ctype.h>
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

namespace fq {

// ---------------------------------------------------------------------------
// ExpressionPlan
// ---------------------------------------------------------------------------
// plan_to_function (plan_expression.rs:40-75): the right child of a binary
// expression and every function argument are built one level deeper; that
// depth is the index AggregatorFunction::merge_state reads.
FunctionRef ExpressionPlan::plan_to_function(size_t depth, const FactoryOptions &o) const {
    switch (kind) {
        case kField: return std::make_shared<FieldFunction>(name);
        case kConstant: return std::make_shared<ConstantFunction>(value);
        case kBinary: {
            FunctionRef l = args[0].plan_to_function(depth, o);
            FunctionRef r = args[1].plan_to_function(depth + 1, o);
            FunctionRef f = function_factory(name, {l, r}, o);
            f->set_depth(depth);
            return f;
        }
        case kFunction: {
            std::vector<FunctionRef> fs;
            for (const auto &a : args) {
                FunctionRef f = a.plan_to_function(depth + 1, o);
                f->set_depth(depth);
                fs.push_back(f);
            }
            FunctionRef f = function_factory(name, fs, o);
            f->set_depth(depth);
            return f;
        }
        case kAlias: {
            FunctionRef f = args[0].plan_to_function(depth, o);
            f->set_depth(depth);
            return std::make_shared<AliasFunction>(name, f);
        }
        default: throw_internal("Cannot transform wildcard to function");
    }
}

bool ExpressionPlan::is_aggregate() const {
    switch (kind) {
        case kAlias: return args[0].is_aggregate();
        case kBinary: return args[0].is_aggregate() || args[1].is_aggregate();
        case kFunction: {
            std::string n = name;
            std::transform(n.begin(), n.end(), n.begin(), [](unsigned char c) { return (char)tolower(c); });
            return n == "max" || n == "min" || n == "avg" || n == "count" || n == "sum";
        }
        default: return false;
    }
}

std::string ExpressionPlan::debug() const {
    switch (kind) {
        case kAlias: return args[0].debug() + " as " + name;
        case kField: return name;
        case kConstant: return value.debug();
        case kBinary: return "(" + args[0].debug() + " " + name + " " + args[1].debug() + ")";
        case kFunction: {
            std::string s = name + "([";
            for (size_t i = 0; i < args.size(); ++i) {
                if (i) s += ", ";
                s += args[i].debug();
            }
            return s + "])";
        }
        default: return "*";
    }
}

DataField ExpressionPlan::to_field(const DataSchema &input, const FactoryOptions &o) const {
    FunctionRef f = to_function(o);
    return DataField{f->display(), f->return_type(input), f->nullable(input)};
}

// ---------------------------------------------------------------------------
// tokenizer
// ---------------------------------------------------------------------------
namespace {

struct Token {
    enum Kind { kEnd, kIdent, kNumber, kString, kSym } kind = kEnd;
    std::string text;
    bool quoted = false;
};

std::vector<Token> tokenize(const std::string &sql) {
    std::vector<Token> out;
    size_t i = 0;
    const size_t n = sql.size();
    while (i < n) {
        const char c = sql[i];
        if (isspace((unsigned char)c)) {
            ++i;
            continue;
        }
        Token t;
        if (isalpha((unsigned char)c) || c == '_') {
            size_t j = i;
            while (j < n && (isalnum((unsigned char)sql[j]) || sql[j] == '_')) ++j;
            t.kind = Token::kIdent;
            t.text = sql.substr(i, j - i);
            i = j;
        } else if (c == '"' || c == '`') {
            const size_t j = sql.find(c, i + 1);
            if (j == std::string::npos) throw FQException(FQ_E_PLAN, "SQLParser Error: unterminated quoted identifier");
            t.kind = Token::kIdent;
            t.quoted = true;
            t.text = sql.substr(i + 1, j - i - 1);
            i = j + 1;
        } else if (isdigit((unsigned char)c) || (c == '.' && i + 1 < n && isdigit((unsigned char)sql[i + 1]))) {
            size_t j = i;
            while (j < n && (isdigit((unsigned char)sql[j]) || sql[j] == '.')) ++j;
            if (j < n && (sql[j] == 'e' || sql[j] == 'E')) {
                size_t k = j + 1;
                if (k < n && (sql[k] == '+' || sql[k] == '-')) ++k;
                if (k < n && isdigit((unsigned char)sql[k])) {
                    j = k;
                    while (j < n && isdigit((unsigned char)sql[j])) ++j;
                }
            }
            t.kind = Token::kNumber;
            t.text = sql.substr(i, j - i);
            i = j;
        } else if (c == '\'') {
            std::string s;
            size_t j = i + 1;
            for (;;) {
                if (j >= n) throw FQException(FQ_E_PLAN, "SQLParser Error: Unterminated string literal");
                if (sql[j] == '\'') {
                    if (j + 1 < n && sql[j + 1] == '\'') {
                        s += '\'';
                        j += 2;
                        continue;
                    }
                    break;
                }
                s += sql[j++];
            }
            t.kind = Token::kString;
            t.text = s;
            i = j + 1;
        } else {
            static const char *two[] = {"<=", ">=", "<>", "!=", "=="};
            t.kind = Token::kSym;
            bool done = false;
            for (const char *s2 : two)
                if (i + 1 < n && sql[i] == s2[0] && sql[i + 1] == s2[1]) {
                    t.text = s2;
                    i += 2;
                    done = true;
                    break;
                }
            if (!done) {
                if (!strchr("(),.*+-/%=<>;", c))
                    throw FQException(FQ_E_PLAN, std::string("SQLParser Error: Unexpected character '") + c + "'");
                t.text = std::string(1, c);
                ++i;
            }
        }
        out.push_back(t);
    }
    out.push_back(Token{});
    return out;
}

bool kw(const Token &t, const char *w) {
    if (t.kind != Token::kIdent || t.quoted) return false;
    if (t.text.size() != strlen(w)) return false;
    for (size_t i = 0; i < t.text.size(); ++i)
        if (toupper((unsigned char)t.text[i]) != w[i]) return false;
    return true;
}

bool reserved(const Token &t) {
    static const char *words[] = {"SELECT", "FROM", "WHERE", "LIMIT", "GROUP", "BY", "HAVING", "AS",
                                  "AND", "OR", "NOT", "ORDER", "UNION", "JOIN", "EXPLAIN", "ON"};
    for (const char *w : words)
        if (kw(t, w)) return true;
    return false;
}

// ---------------------------------------------------------------------------
// parser: produces ExpressionPlans directly (sql_to_rex, plan_parser.rs:216-262)
// ---------------------------------------------------------------------------
struct SelectAst {
    bool explain = false;
    std::vector<ExpressionPlan> items;
    bool has_from = false;
    std::vector<std::string> table;  // [db,] table
    std::vector<ExpressionPlan> table_args;
    bool has_where = false;
    ExpressionPlan where;
    bool has_group = false, has_having = false;
    std::vector<ExpressionPlan> group;
    bool has_limit = false;
    ExpressionPlan limit;
};

class Parser {
   public:
    explicit Parser(const std::string &sql) : toks_(tokenize(sql)) {}

    SelectAst parse() {
        SelectAst a;
        if (kw(peek(), "EXPLAIN")) {
            ++p_;
            a.explain = true;
        }
        if (!kw(peek(), "SELECT")) err("Expected SELECT, found: " + peek().text);
        ++p_;
        for (;;) {
            a.items.push_back(select_item());
            if (!sym(",")) break;
        }
        if (kw(peek(), "FROM")) {
            ++p_;
            a.has_from = true;
            a.table.push_back(ident());
            if (sym(".")) a.table.push_back(ident());
            if (sym("(")) {
                if (!sym(")")) {
                    for (;;) {
                        a.table_args.push_back(expr(0));
                        if (sym(")")) break;
                        expect(",");
                    }
                }
            }
        }
        if (kw(peek(), "WHERE")) {
            ++p_;
            a.has_where = true;
            a.where = expr(0);
        }
        if (kw(peek(), "GROUP")) {
            ++p_;
            if (!kw(peek(), "BY")) err("Expected BY after GROUP");
            ++p_;
            a.has_group = true;
            for (;;) {
                a.group.push_back(expr(0));
                if (!sym(",")) break;
            }
        }
        if (kw(peek(), "HAVING")) {
            ++p_;
            a.has_having = true;
            (void)expr(0);
        }
        if (kw(peek(), "LIMIT")) {
            ++p_;
            a.has_limit = true;
            a.limit = expr(0);
        }
        sym(";");
        if (peek().kind != Token::kEnd) err("Expected end of statement, found: " + peek().text);
        return a;
    }

   private:
    std::vector<Token> toks_;
    size_t p_ = 0;

    const Token &peek(size_t k = 0) const { return toks_[std::min(p_ + k, toks_.size() - 1)]; }
    [[noreturn]] void err(const std::string &m) const { throw FQException(FQ_E_PLAN, "SQLParser Error: " + m); }
    bool sym(const char *s) {
        if (peek().kind == Token::kSym && peek().text == s) {
            ++p_;
            return true;
        }
        return false;
    }
    void expect(const char *s) {
        if (!sym(s)) err(std::string("Expected ") + s + ", found: " + peek().text);
    }
    std::string ident() {
        const Token &t = peek();
        if (t.kind != Token::kIdent) err("Expected identifier, found: " + t.text);
        ++p_;
        return t.text;
    }

    ExpressionPlan select_item() {
        if (sym("*")) {
            ExpressionPlan w;
            w.kind = ExpressionPlan::kWildcard;
            return w;
        }
        ExpressionPlan e = expr(0);
        std::string alias;
        if (kw(peek(), "AS")) {
            ++p_;
            alias = ident();
        } else if (peek().kind == Token::kIdent && !reserved(peek())) {
            alias = ident();
        }
        if (!alias.empty()) {
            ExpressionPlan a;
            a.kind = ExpressionPlan::kAlias;
            a.name = alias;
            a.args.push_back(e);
            return a;
        }
        return e;
    }

    // sqlparser 0.6 precedences: OR 5, AND 10, comparisons 20, + - 30, * / % 40
    int precedence(const Token &t, std::string &op) const {
        if (kw(t, "OR")) {
            op = "OR";
            return 5;
        }
        if (kw(t, "AND")) {
            op = "AND";
            return 10;
        }
        if (t.kind != Token::kSym) return 0;
        op = t.text;
        if (op == "=" || op == "<" || op == "<=" || op == ">" || op == ">=") return 20;
        if (op == "<>" || op == "!=") {
            op = "<>";
            return 20;
        }
        if (op == "+" || op == "-") return 30;
        if (op == "*" || op == "/" || op == "%") return 40;
        return 0;
    }

    ExpressionPlan expr(int min_prec) {
        ExpressionPlan lhs = prefix();
        for (;;) {
            std::string op;
            const int prec = precedence(peek(), op);
            if (prec == 0 || prec <= min_prec) break;
            ++p_;
            ExpressionPlan rhs = expr(prec);
            ExpressionPlan b;
            b.kind = ExpressionPlan::kBinary;
            b.name = op;
            b.args.push_back(lhs);
            b.args.push_back(rhs);
            lhs = b;
        }
        return lhs;
    }

    ExpressionPlan prefix() {
        const Token t = peek();
        if (t.kind == Token::kSym && t.text == "(") {
            ++p_;
            ExpressionPlan e = expr(0);
            expect(")");
            return e;  // Expr::Nested
        }
        if (t.kind == Token::kSym && (t.text == "-" || t.text == "+")) {
            ++p_;
            ExpressionPlan inner = expr(50);
            throw FQException(FQ_E_PLAN, "Error during plan: Unsupported ExpressionPlan: " + t.text + inner.debug());
        }
        if (t.kind == Token::kNumber) {
            ++p_;
            return number(t.text);
        }
        if (t.kind == Token::kString) {
            ++p_;
            ExpressionPlan c;
            c.kind = ExpressionPlan::kConstant;
            c.value = DataValue::string(t.text);
            return c;
        }
        if (t.kind == Token::kIdent) {
            if (kw(t, "NOT")) throw FQException(FQ_E_PLAN, "Error during plan: Unsupported ExpressionPlan: NOT");
            ++p_;
            if (sym("(")) {
                ExpressionPlan f;
                f.kind = ExpressionPlan::kFunction;
                f.name = t.text;
                if (!sym(")")) {
                    for (;;) {
                        if (peek().kind == Token::kSym && peek().text == "*")
                            throw FQException(FQ_E_PLAN, "Error during plan: Unsupported ExpressionPlan: *");
                        f.args.push_back(expr(0));
                        if (sym(")")) break;
                        expect(",");
                    }
                }
                return f;
            }
            if (peek().kind == Token::kSym && peek().text == ".")
                throw FQException(FQ_E_PLAN, "Error during plan: Unsupported ExpressionPlan: " + t.text + "." +
                                                 peek(1).text);
            ExpressionPlan f;
            f.kind = ExpressionPlan::kField;
            f.name = t.text;
            return f;
        }
        err("Expected an expression, found: " + (t.kind == Token::kEnd ? std::string("EOF") : t.text));
    }

    // Value::Number: i64 parse -> UInt64 (>= 0) / Int64, else f64 (plan_parser.rs:216-229)
    static ExpressionPlan number(const std::string &s) {
        ExpressionPlan c;
        c.kind = ExpressionPlan::kConstant;
        bool is_int = !s.empty() && std::all_of(s.begin(), s.end(), [](char ch) { return isdigit((unsigned char)ch); });
        if (is_int) {
            errno = 0;
            char *end = nullptr;
            const long long v = strtoll(s.c_str(), &end, 10);
            if (errno == 0 && end && *end == 0) {
                c.value = v >= 0 ? DataValue::u64((uint64_t)v) : DataValue::some(FQ_DT_INT64, (uint64_t)v);
                return c;
            }
        }
        char *end = nullptr;
        const double d = strtod(s.c_str(), &end);
        if (!end || *end) throw FQException(FQ_E_INTERNAL, "Internal Error: invalid float literal");
        uint64_t b;
        memcpy(&b, &d, 8);
        c.value = DataValue::some(FQ_DT_FLOAT64, b);
        return c;
    }
};

SchemaRef fields_schema(const std::vector<ExpressionPlan> &exprs, const DataSchema &input, const FactoryOptions &o) {
    auto s = std::make_shared<DataSchema>();
    for (const auto &e : exprs) s->fields.push_back(e.to_field(input, o));
    return s;
}

}  // namespace

// select_to_plan (plan_parser.rs:90-133)
QueryPlan build_from_sql(const std::string &sql, const QueryContext &ctx) {
    SelectAst a = Parser(sql).parse();
    QueryPlan qp;
    qp.explain = a.explain;
    if (a.has_having) throw_internal("HAVING is not implemented yet");
    if (!a.has_from)
        throw_status(FQ_E_UNSUPPORTED, "SELECT without FROM (an Empty plan) is outside the device hot path");
    // from: create_relation (plan_parser.rs:170-204)
    std::string db = ctx.default_db, table = a.table[0];
    if (a.table.size() == 2) {
        db = a.table[0];
        table = a.table[1];
    }
    TableRef t = ctx.get_table(db, table);
    SchemaRef input = t->schema();
    PlanNode rs;
    rs.kind = PlanNode::kReadSource;
    const DataValue *arg = nullptr;
    if (!a.table_args.empty() && a.table_args[0].kind == ExpressionPlan::kConstant) arg = &a.table_args[0].value;
    rs.read = t->read_plan(arg);
    rs.schema = rs.read.schema;
    qp.nodes.push_back(rs);
    // filter
    if (a.has_where) {
        PlanNode f;
        f.kind = PlanNode::kFilter;
        f.predicate = a.where;
        f.schema = input;
        qp.nodes.push_back(f);
    }
    // projection / aggregate
    std::vector<ExpressionPlan> items;
    for (const auto &e : a.items) {
        if (e.kind == ExpressionPlan::kWildcard)  // PlanBuilder::project expands `*`
            for (const auto &fl : input->fields) {
                ExpressionPlan fe;
                fe.kind = ExpressionPlan::kField;
                fe.name = fl.name;
                items.push_back(fe);
            }
        else items.push_back(e);
    }
    std::vector<ExpressionPlan> aggr;
    for (const auto &e : a.items)
        if (e.is_aggregate()) aggr.push_back(e);
    PlanNode pn;
    pn.exprs = aggr.empty() && !a.has_group ? items : aggr;
    if (!aggr.empty() || a.has_group) {
        // PlanParser::aggregate (plan_parser.rs:284-308): group + aggregate
        // expressions must account for the whole projection
        if (a.group.size() + aggr.size() != items.size()) throw_plan("Projection references non-aggregate values");
        pn.kind = PlanNode::kAggregate;
        pn.groups = a.group;
    } else {
        pn.kind = PlanNode::kProjection;
    }
    // PlanBuilder::aggregate (plan_builder.rs:63-83): schema = group ++ aggr
    std::vector<ExpressionPlan> out_exprs = pn.groups;
    out_exprs.insert(out_exprs.end(), pn.exprs.begin(), pn.exprs.end());
    pn.schema = fields_schema(out_exprs, *input, ctx.factory);
    qp.nodes.push_back(pn);
    // limit
    if (a.has_limit) {
        if (a.limit.kind != ExpressionPlan::kConstant || a.limit.value.kind != DataValue::kSome ||
            a.limit.value.dtype != FQ_DT_UINT64)
            throw_plan("Unexpected expression for LIMIT clause");
        PlanNode l;
        l.kind = PlanNode::kLimit;
        l.limit = (size_t)a.limit.value.bits;
        l.schema = pn.schema;
        qp.nodes.push_back(l);
    }
    return qp;
}

// ---------------------------------------------------------------------------
// Optimizer::create().optimize (optimizer.rs:20-32): the one optimizer the
// reference registers, FilterPushDownOptimizer
// (optimizer_filter_push_down.rs:18-81), run by the MySQL handler between
// planning and execution (mysql_handler.rs:58).
// ---------------------------------------------------------------------------
namespace {

// rewrite_alias_expr (optimizer_filter_push_down.rs:18-36): children first,
// then a Field naming a projection output becomes that output's expression
// (Alias stripped by projections_to_map, optimizer.rs:40-47).
ExpressionPlan rewrite_alias_expr(const ExpressionPlan &e, const std::vector<std::pair<std::string, ExpressionPlan>> &proj) {
    if (e.kind == ExpressionPlan::kField) {
        // HashMap::insert keeps the last field of a repeated name
        for (size_t i = proj.size(); i-- > 0;)
            if (proj[i].first == e.name) return proj[i].second;
        return e;
    }
    // expression_plan_children / rebuild_alias_from_exprs (optimizer.rs:59-70,
    // optimizer_filter_push_down.rs:38-60); constants and `*` have no children
    ExpressionPlan out = e;
    for (auto &a : out.args) a = rewrite_alias_expr(a, proj);
    return out;
}

}  // namespace

void optimize(QueryPlan &plan) {
    // projections_to_map (optimizer.rs:36-57): from the top of the plan down
    // through Limit / Filter / Aggregate to the first Projection
    std::vector<std::pair<std::string, ExpressionPlan>> proj;
    for (size_t k = plan.nodes.size(); k-- > 0;) {
        const PlanNode &n = plan.nodes[k];
        if (n.kind == PlanNode::kProjection) {
            for (size_t i = 0; i < n.schema->fields.size() && i < n.exprs.size(); ++i) {
                const ExpressionPlan &x = n.exprs[i];
                proj.emplace_back(n.schema->fields[i].name, x.kind == ExpressionPlan::kAlias ? x.args[0] : x);
            }
            break;
        }
        if (n.kind == PlanNode::kReadSource) break;
    }
    // every Filter's predicate is rewritten (node_to_plans / plans_to_node
    // rebuild the same chain; only the predicate changes)
    for (PlanNode &n : plan.nodes)
        if (n.kind == PlanNode::kFilter) n.predicate = rewrite_alias_expr(n.predicate, proj);
}

std::string QueryPlan::display() const {
    std::string out;
    size_t indent = 0;
    for (size_t k = nodes.size(); k-- > 0;) {
        const PlanNode &n = nodes[k];
        if (indent > 0) {
            out += "\n";
            for (size_t i = 0; i < indent; ++i) out += "  ";
        }
        out += "\xe2\x94\x94\xe2\x94\x80";
        switch (n.kind) {
            case PlanNode::kProjection:
            case PlanNode::kAggregate: {
                out += n.kind == PlanNode::kProjection ? " Projection: " : " Aggregate: ";
                for (size_t i = 0; i < n.exprs.size(); ++i) {
                    if (i) out += ", ";
                    out += n.exprs[i].debug();
                }
                // plan_display.rs:43-49 writes the group list straight after
                // the aggregate list (no separator between the two)
                for (size_t i = 0; i < n.groups.size(); ++i) {
                    if (i) out += ", ";
                    out += n.groups[i].debug();
                }
                break;
            }
            case PlanNode::kFilter: out += " Filter: " + n.predicate.debug(); break;
            case PlanNode::kLimit: out += " Limit: " + std::to_string(n.limit); break;
            case PlanNode::kReadSource:
                out += " ReadDataSource: scan parts [" + std::to_string(n.read.partitions.size()) + "]" +
                       n.read.description;
                break;
        }
        ++indent;
    }
    return out;
}

// PipelineBuilder::build (pipeline_builder.rs:26-106)
Pipeline build_pipeline(const QueryPlan &plan, const QueryContextRef &ctx, bool emit_states) {
    Pipeline p;
    // No aggregate above the source: a row pipeline.  With a LIMIT its pipes
    // read growing morsels on private queues (a satisfied LIMIT stops after
    // the first few); without one they read bounded pieces on the two row
    // queues (pipe p on queue p % 2: a projection launch's tail overlaps the
    // next one's start, Runtime::kRowQueues).  Aggregates share one queue.
    bool row_pipeline = true, has_limit = false;
    for (const PlanNode &n : plan.nodes) {
        if (n.kind == PlanNode::kAggregate) row_pipeline = false;
        if (n.kind == PlanNode::kLimit) has_limit = true;
    }
    const ReadMode mode = !row_pipeline ? ReadMode::kWhole : has_limit ? ReadMode::kMorsels : ReadMode::kChunks;
    p.set_queues(mode == ReadMode::kMorsels ? QueueKind::kOwn
                 : mode == ReadMode::kChunks ? QueueKind::kRow
                                             : QueueKind::kShared);
    for (const PlanNode &n : plan.nodes) {
        switch (n.kind) {
            case PlanNode::kLimit: {
                const size_t lim = n.limit;
                p.add_simple_transform([lim]() { return std::make_shared<LimitTransform>(lim); });
                if (p.pipe_num() > 1) {
                    p.merge_processor();
                    p.add_simple_transform([lim]() { return std::make_shared<LimitTransform>(lim); });
                }
                break;
            }
            case PlanNode::kProjection: {
                // the block-stream projections of the query's pipes are timed as one span (LaunchSpan)
                const bool blocks = mode != ReadMode::kMorsels;
                auto span = blocks ? std::make_shared<LaunchSpan>(ctx->rt, (int)std::max<size_t>(1, p.pipe_num()))
                                   : nullptr;
                p.add_simple_transform([&, span, blocks]() {
                    for (const auto &e : n.exprs)  // transform_projection.rs:24-31
                        if (e.is_aggregate()) throw_internal("Unsupported aggregator function: " + e.debug());
                    std::vector<FunctionRef> fs;
                    for (const auto &e : n.exprs) fs.push_back(e.to_function(ctx->factory));
                    return std::make_shared<ProjectionTransform>(n.schema, fs, blocks, span);
                });
                break;
            }
            case PlanNode::kAggregate: {
                if (!n.groups.empty()) {  // GROUP BY (no reference transform; fq_group_*)
                    if (n.groups.size() != 1)
                        throw_status(FQ_E_UNSUPPORTED, "GROUP BY supports one key expression on the device path");
                    auto shared = std::make_shared<GroupByShared>();
                    // partitions this rank reads (sizes the table when every
                    // block brings keys of its own)
                    for (const PlanNode &src : plan.nodes)
                        if (src.kind == PlanNode::kReadSource) {
                            const size_t np = src.read.partitions.size(), w = (size_t)std::max(1, ctx->world);
                            shared->blocks_hint = (int64_t)std::max<size_t>(1, (np + w - 1) / w);
                        }
                    auto funcs = [&]() {
                        std::vector<FunctionRef> fs;
                        for (const auto &e : n.exprs) fs.push_back(e.to_function(ctx->factory));
                        return fs;
                    };
                    const ExpressionPlan key = n.groups[0];
                    p.add_simple_transform([&, shared, key]() {
                        return std::make_shared<GroupByPartialTransform>(key.to_function(ctx->factory), funcs(), shared);
                    });
                    p.merge_processor();
                    p.add_simple_transform([&, shared]() {
                        return std::make_shared<GroupByFinalTransform>(n.schema, funcs(), shared, emit_states);
                    });
                    break;
                }
                auto funcs = [&]() {
                    std::vector<FunctionRef> fs;
                    for (const auto &e : n.exprs) fs.push_back(e.to_function(ctx->factory));
                    return fs;
                };
                // the query's partial pipes wait for their scans together (ScanGroup)
                auto group = std::make_shared<ScanGroup>(ctx->rt, (int)std::max<size_t>(1, p.pipe_num()));
                p.add_simple_transform(
                    [&, group]() { return std::make_shared<AggregatePartialTransform>(n.schema, funcs(), group); });
                p.merge_processor();
                p.add_simple_transform(
                    [&]() { return std::make_shared<AggregateFinalTransform>(n.schema, funcs(), emit_states); });
                break;
            }
            case PlanNode::kFilter: {
                p.add_simple_transform([&]() {
                    if (n.predicate.is_aggregate())  // transform_filter.rs:24-30
                        throw_internal("Aggregate function " + n.predicate.debug() + " is found in WHERE in query");
                    return std::make_shared<FilterTransform>(n.predicate.to_function(ctx->factory));
                });
                break;
            }
            case PlanNode::kReadSource: {
                std::vector<Partition> parts = n.read.partitions;
                if (ctx->world > 1 || ctx->rank > 0) {  // this rank's shard [8r/G, 8(r+1)/G)
                    const size_t np = parts.size();
                    const size_t lo = np * (size_t)ctx->rank / (size_t)ctx->world;
                    const size_t hi = np * (size_t)(ctx->rank + 1) / (size_t)ctx->world;
                    parts = std::vector<Partition>(parts.begin() + lo, parts.begin() + hi);
                }
                size_t workers = ctx->worker_threads;
                workers = (workers == 0 || workers >= parts.size()) ? 1 : parts.size() / workers;
                for (size_t i = 0; i < parts.size(); i += workers) {
                    std::vector<Partition> chunk(parts.begin() + i, parts.begin() + std::min(parts.size(), i + workers));
                    p.add_source(std::make_shared<SourceTransform>(ctx, n.read.db, n.read.table, chunk, mode));
                }
                if (parts.empty()) p.add_source(std::make_shared<BlocksProcessor>(std::vector<DataBlock>{}));
                break;
            }
        }
    }
    p.merge_processor();
    return p;
}

}  // namespace fq
