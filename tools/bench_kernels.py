#!/usr/bin/env python3
"""Per-kernel HBM roofline of every C-ABI kernel on one MI355X, at the size of
one numbers_mt partition (1.25e9 u64 rows = 10 GB at N = 1e10).

Each entry point is called raw through include/fq_gpu.h (no flag buffer, so
no host sync), timed with HIP events on the stream it is launched on, median
of R repetitions; achieved GB/s = algorithmic bytes / time.  Results are
checked against numpy on a prefix.  Prints one JSON document.

usage: python tools/bench_kernels.py [--rows 1.25e9] [--reps 10] > gpurun_out/kernels.json
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fq_amd import abi, ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402
knobs.apply_env()
from fq_amd._lib import check, lib  # noqa: E402
from fq_amd.expr import chain, predicate  # noqa: E402

PEAK = 8000.0  # GB/s, MI355X HBM3E spec


def timed(fn, reps):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()  # warm (and JIT compile)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0.record(s)
        fn()
        e1.record(s)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1.25e9)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    n = int(args.rows)
    st = ops._stream()
    res = []

    def rec(name, ref, ms, nbytes, note=""):
        gbps = nbytes / (ms * 1e-3) / 1e9
        res.append({"kernel": name, "replaces": ref, "ms": ms, "algorithmic_bytes": nbytes,
                    "achieved_gbps": gbps, "frac_of_peak": gbps / PEAK, "note": note})
        print("%-34s %8.3f ms  %7.0f GB/s  %4.1f %%" % (name, ms, gbps, 100 * gbps / PEAK), file=sys.stderr)

    a = ops.empty_column(n, abi.DT_UINT64)
    b = ops.splitmix_column(7, 0, n)
    out = ops.empty_column(n, abi.DT_UINT64)
    bm = ops.empty_column(n, abi.DT_BOOLEAN)

    # source: NumbersStream::poll_next
    ms = timed(lambda: check(lib.fq_fill_numbers_u64(C.c_void_p(a.ptr), 0, n, st)), args.reps)
    rec("fill_numbers_u64", "numbers_stream.rs:65-83", ms, 8 * n)

    ac, bc, oc = a.col(), b.col(), out.col()
    one = abi.fq_value(abi.DT_UINT64, 1, 1)
    seven = abi.fq_value(abi.DT_UINT64, 1, 7)

    def arith(op, rhs_col=None, rhs_s=None):
        check(lib.fq_arith(op, C.byref(ac), None, C.byref(rhs_col) if rhs_col is not None else None,
                           C.byref(rhs_s) if rhs_s is not None else None, C.byref(oc), None, st))

    ms = timed(lambda: arith(abi.OP_BY_SYM["+"], rhs_s=one), args.reps)
    rec("arith u64 + const", "data_array_arithmetic.rs:14-55", ms, 16 * n)
    k = 1 << 20
    assert np.array_equal(out.to_numpy()[:k], np.arange(1, k + 1, dtype=np.uint64))
    ms = timed(lambda: arith(abi.OP_BY_SYM["*"], rhs_col=bc), args.reps)
    rec("arith u64 * col", "data_array_arithmetic.rs:14-55", ms, 24 * n)
    ms = timed(lambda: arith(abi.OP_BY_SYM["/"], rhs_s=seven), args.reps)
    rec("arith u64 / const 7", "data_array_arithmetic.rs:14-55", ms, 16 * n)
    assert np.array_equal(out.to_numpy()[:k], np.arange(0, k, dtype=np.uint64) // np.uint64(7))

    bound = abi.fq_value(abi.DT_UINT64, 1, (3 * 2**64) // 8)

    def compare():
        check(lib.fq_compare(abi.CMP_BY_SYM["<"], C.byref(bc), None, None, C.byref(bound),
                             C.c_void_p(bm.ptr), n, None, st))

    ms = timed(compare, args.reps)
    rec("compare u64 < const -> bitmap", "data_array_comparison.rs:14-94", ms, 8 * n + n // 8)
    hb = b.to_numpy()[:k]
    assert np.array_equal(bm.to_numpy()[:k], hb < np.uint64((3 * 2**64) // 8))

    ws = ops.Workspace(lib.fq_filter_workspace_bytes(n))
    kept = C.c_int64(0)

    def compact():
        check(lib.fq_filter_compact(C.byref(bc), C.c_void_p(bm.ptr), C.c_void_p(out.ptr), C.byref(kept),
                                    ws.ptr, ws.nbytes, st))

    ms = timed(compact, args.reps)
    rec("filter_compact (3/8 kept)", "transform_filter.rs:51 (arrow filter)", ms,
        8 * n + n // 8 + 8 * kept.value, "includes the host sync for out_len")

    aws = ops.Workspace(lib.fq_aggregate_workspace_bytes(n))
    dst = torch.empty(48, dtype=torch.uint8, device="cuda")
    ALL = abi.AGG_SUM | abi.AGG_MAX | abi.AGG_MIN | abi.AGG_COUNT

    def agg(col, pred=None, value=None, mask=ALL, br=10000):
        c = col.col()
        check(lib.fq_aggregate(C.byref(c), br, C.byref(pred) if pred is not None else None,
                               C.byref(value) if value is not None else None, mask,
                               C.c_void_p(dst.data_ptr()), aws.ptr, aws.nbytes, st))

    pb = abi.fq_pred()
    pb.kind = abi.PRED_BITMAP
    pb.bitmap = bm.ptr
    ms = timed(lambda: agg(b, pred=pb, mask=abi.AGG_MAX | abi.AGG_COUNT), args.reps)
    rec("aggregate, bitmap predicate", "function_aggregator.rs:57-100 + filter", ms, 8 * n + n // 8)
    ms = timed(lambda: agg(a), args.reps)
    rec("aggregate identity (C3 shape)", "function_aggregator.rs:57-100", ms, 8 * n)
    v, _ = chain(abi.DT_UINT64, [("+", 1)])
    p = predicate(abi.DT_UINT64, [("%", 8)], "<", 3)
    ms = timed(lambda: agg(a, pred=p, value=v, mask=abi.AGG_MAX | abi.AGG_COUNT), args.reps)
    rec("aggregate C4 shape (specialised)", "C4: max(number+1) WHERE (number%8)<3", ms, 8 * n)
    ms = timed(lambda: agg(a, pred=p, value=v, mask=abi.AGG_SUM), args.reps)
    rec("aggregate filtered sum (block mode)", "sum(number+1) WHERE (number%8)<3", ms, 8 * n)
    from fq_amd.expr import pred_tree
    tp = pred_tree(abi.DT_UINT64, [([("%", 8)], "<", 3), ([], ">", 1000)], [0, 1, "and"])
    ms = timed(lambda: agg(a, pred=tp, value=v, mask=abi.AGG_MAX | abi.AGG_COUNT), args.reps)
    rec("aggregate AND-tree predicate", "max(number+1) WHERE number%8<3 AND number>1000", ms, 8 * n)
    vf, _ = chain(abi.DT_UINT64, [("*", 1.5), ("+", 0.25)])
    ms = timed(lambda: agg(a, value=vf), args.reps)
    rec("aggregate f64 chain", "sum/max/min(number*1.5+0.25)", ms, 8 * n)
    vd, _ = chain(abi.DT_UINT64, [("%", 1000003)])
    ms = timed(lambda: agg(b, value=vd), args.reps)
    rec("aggregate u64 % 1000003 (magic)", "sum/max/min(x % 1000003)", ms, 8 * n)
    vm, _ = chain(abi.DT_UINT64, [("%", 1000)])
    ms = timed(lambda: agg(b, value=vm), args.reps)
    rec("aggregate u64 % 1000 (32-bit halves)", "sum/max/min(x % 1000)", ms, 8 * n)
    vq, _ = chain(abi.DT_UINT64, [("/", 1000)])
    ms = timed(lambda: agg(b, value=vq), args.reps)
    rec("aggregate u64 / 1000 (32-bit long division)", "sum/max/min(x / 1000)", ms, 8 * n)
    ops.jit_config(abi.JIT_OFF)
    ms = timed(lambda: agg(a, pred=p, value=v, mask=abi.AGG_MAX | abi.AGG_COUNT), args.reps)
    rec("aggregate C4 shape (interpreted)", "C4 with FQ_JIT_OFF", ms, 8 * n)
    ops.jit_config(abi.JIT_AUTO, 1 << 22)

    # expression trees (FQ_OP_PUSH / FQ_OPERAND_STACK) in the fused scan
    from fq_amd.expr import PUSH, STACK
    vt, _ = chain(abi.DT_UINT64, [("+", 1), PUSH, ("%", 1000), ("*", STACK, True)])
    ms = timed(lambda: agg(a, value=vt), args.reps)
    rec("aggregate tree (number+1)*(number%1000)", "sum/max/min of an ArithmeticFunction tree", ms, 8 * n)

    # FilterTransform -> ProjectionTransform fused (fq_filter_project)
    flag = ops.Workspace(8)
    readme_pred = predicate(abi.DT_UINT64, [("+", 1), PUSH, ("/", 2), ("+", STACK, True), ("+", 1)], "<", 100)
    ac2 = a.col()
    ms = timed(lambda: check(lib.fq_predicate_bitmap(C.byref(ac2), C.byref(readme_pred), C.c_void_p(bm.ptr),
                                                     flag.ptr, st)), args.reps)
    rec("predicate_bitmap (number+1)+(number/2)+1<100", "README WHERE, one kernel", ms, 8 * n + n // 8,
        "includes the host sync for the error flag")
    pws = ops.Workspace(lib.fq_filter_project_workspace_bytes(n))
    out2 = ops.empty_column(n, abi.DT_UINT64)
    p38 = predicate(abi.DT_UINT64, [], "<", (3 * 2**64) // 8)
    vals = (abi.fq_expr * 2)(chain(abi.DT_UINT64, [("+", 1)])[0], chain(abi.DT_UINT64, [("/", 2)])[0])
    outs = (C.c_void_p * 2)(out.ptr, out2.ptr)
    bc2 = b.col()

    def project():
        check(lib.fq_filter_project(C.byref(bc2), C.byref(p38), vals, 2, outs, C.byref(kept), pws.ptr, pws.nbytes, st))

    ms = timed(project, args.reps)
    rec("filter_project 3/8 kept -> x+1, x/2", "Filter + Projection fused", ms, 8 * n + 2 * 8 * kept.value,
        "two passes over the column (bits, scatter) + host sync for out_len")
    hb = b.to_numpy()[:k]
    kk = hb[hb < np.uint64((3 * 2**64) // 8)]
    assert np.array_equal(out.to_numpy()[:len(kk)], kk + np.uint64(1))
    vals1 = (abi.fq_expr * 1)(chain(abi.DT_UINT64, [("*", 3), ("+", 1)])[0])
    outs1 = (C.c_void_p * 1)(out.ptr)
    ms = timed(lambda: check(lib.fq_filter_project(C.byref(ac2), None, vals1, 1, outs1, C.byref(kept), pws.ptr,
                                                   pws.nbytes, st)), args.reps)
    rec("filter_project map x*3+1 (no predicate)", "Projection fused", ms, 16 * n, "host sync for out_len")

    # GROUP BY (fq_group_aggregate): LDS pre-aggregation, low and high cardinality
    key, _ = chain(abi.DT_UINT64, [("%", 1000)])
    aggs3 = [(abi.AGG_COUNT, abi.DT_UINT64), (abi.AGG_SUM, abi.DT_UINT64), (abi.AGG_MAX, abi.DT_UINT64)]
    gt = ops.GroupTable(1 << 12, aggs3)

    def group_low():
        check(lib.fq_group_table_init(C.byref(gt.desc), st))
        gt.aggregate(a, key=key)

    ms = timed(group_low, args.reps)
    rec("group by number%1000: count,sum,max", "no reference (plan_parser.rs:284-308)", ms, 8 * n,
        "includes the table init")
    assert gt.count() == 1000
    key8, _ = chain(abi.DT_UINT64, [("%", 8)])
    pred = predicate(abi.DT_UINT64, [("%", 8)], "<", 3)
    v1, _ = chain(abi.DT_UINT64, [("+", 1)])
    gt8 = ops.GroupTable(64, [(abi.AGG_MAX, abi.DT_UINT64), (abi.AGG_COUNT, abi.DT_UINT64)])

    def group_c4():
        check(lib.fq_group_table_init(C.byref(gt8.desc), st))
        gt8.aggregate(a, pred=pred, key=key8, values=[v1, None])

    ms = timed(group_c4, args.reps)
    rec("group by number%8 WHERE %8<3: max(+1),count", "C4 shape grouped", ms, 8 * n, "includes the table init")
    hn = min(n, 1 << 27)
    hc = ops.DeviceColumn(b.buf, hn, abi.DT_UINT64)
    gth = ops.GroupTable(1 << 28, [(abi.AGG_COUNT, abi.DT_UINT64)])

    def group_high():
        check(lib.fq_group_table_init(C.byref(gth.desc), st))
        gth.aggregate(hc)

    ms = timed(group_high, max(3, args.reps // 3))
    rec("group by x (distinct, %d rows): count" % hn, "high cardinality: HBM table, 2^28 slots", ms, 8 * hn,
        "includes the table init (4 GB)")

    print(json.dumps({"rows": n, "peak_gbps": PEAK, "device": torch.cuda.get_device_name(0),
                      "kernels": res}, indent=1))


if __name__ == "__main__":
    main()
