// SQL front-end restated for the supported subset:
//   Planner::build_from_sql / select_to_plan   src/planners/plan_parser.rs:16-329
//   ExpressionPlan (+ plan_to_function depths) src/planners/plan_expression.rs:14-105
//   PlanBuilder                                src/planners/plan_builder.rs
//   PipelineBuilder::build                     src/processors/pipeline_builder.rs:26-106
// Grammar: [EXPLAIN] SELECT item[, ...] FROM [db.]table[(args)] [WHERE expr]
//          [GROUP BY expr] [LIMIT n]; operators + - * / % = < <= > >= with sqlparser 0.6
//          precedence, function calls, parentheses, AS aliases.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "core.h"
#include "functions.h"
#include "pipeline.h"

namespace fq {

struct ExpressionPlan {
    enum Kind { kAlias, kField, kConstant, kBinary, kFunction, kWildcard } kind = kField;
    std::string name;  // alias / field / operator / function name
    DataValue value;   // kConstant
    std::vector<ExpressionPlan> args;  // kBinary: {left, right}; kFunction: args; kAlias: {expr}

    FunctionRef to_function(const FactoryOptions &o) const { return plan_to_function(0, o); }
    FunctionRef plan_to_function(size_t depth, const FactoryOptions &o) const;
    bool is_aggregate() const;
    std::string debug() const;  // fmt::Debug (plan_expression.rs:88-105)
    DataField to_field(const DataSchema &input, const FactoryOptions &o) const;
};

struct PlanNode {
    enum Kind { kReadSource, kFilter, kProjection, kAggregate, kLimit } kind = kReadSource;
    ReadDataSourcePlan read;
    ExpressionPlan predicate;
    std::vector<ExpressionPlan> exprs;  // projection / aggr exprs
    std::vector<ExpressionPlan> groups;  // GROUP BY exprs (kAggregate)
    SchemaRef schema;
    size_t limit = 0;
};

struct QueryPlan {
    bool explain = false;
    std::vector<PlanNode> nodes;  // leaf first (PlanNode::children_to_plans order)
    std::string display() const;  // plan_display.rs indent format
};

QueryPlan build_from_sql(const std::string &sql, const QueryContext &ctx);

// Optimizer::create().optimize: FilterPushDownOptimizer (aliases in WHERE
// replaced by the projected expressions), optimizer_filter_push_down.rs
void optimize(QueryPlan &plan);

// PipelineBuilder::build; emit_states = distributed partial (see fq_engine.h)
Pipeline build_pipeline(const QueryPlan &plan, const QueryContextRef &ctx, bool emit_states = false);

}  // namespace fq
