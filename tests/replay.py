"""Test helper: turn one device fq_agg_state (a run of `blocks` reference
blocks) into the partial DataValue state the reference's per-block loop
(AggregatorFunction::accumulate, function_aggregator.rs:57-100) would hold,
so kernel-level results compare 1:1 with the oracle's per-partition states.
(The product engine has its own C++ version of this replay.)"""
from fq_amd import abi
from oracle_c import FQO_NONE, FQO_NULL, FQO_SOME, OracleError


def replay(op, st, count_dtype=abi.DT_UINT64):
    if st.blocks == 0:
        return (FQO_NULL, abi.DT_NULL, 0)
    if st.flags & abi.STATE_DIV_ZERO:
        raise OracleError(abi.FQ_E_DIVIDE_BY_ZERO, "Internal Error: Divide by zero error")
    if st.flags & abi.STATE_CAST_NULL:
        raise OracleError(abi.FQ_E_UNSUPPORTED, "cast produced nulls")
    if op == abi.AGG_COUNT:
        return (FQO_SOME, count_dtype, st.count)
    if op == abi.AGG_SUM:
        if st.blocks == 1:
            return (FQO_SOME if st.count else FQO_NONE, st.dtype, st.sum if st.count else 0)
        if st.flags & abi.STATE_ANY_EMPTY:
            raise OracleError(abi.FQ_E_INTERNAL,
                              "Internal Error: DataValue to array cannot be NONE NULL")
        return (FQO_SOME, st.dtype, st.sum)
    v = st.max if op == abi.AGG_MAX else st.min
    return (FQO_SOME, st.dtype, v) if st.count else (FQO_NONE, st.dtype, 0)


def as_tuple(s):
    """fqo_state -> (kind, dtype, bits) with the bits zeroed for Null/None."""
    if s.kind != FQO_SOME:
        return (s.kind, s.dtype if s.kind == FQO_NONE else abi.DT_NULL, 0)
    return (s.kind, s.dtype, s.bits)
