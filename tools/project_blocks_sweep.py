"""Launch-shape sweep of fq_filter_project_blocks (tuning tool, not product
code): one resident 10 GB numbers_mt partition, the p1 query's predicate and
expressions, 10,000-row blocks; for each KNOB=V,... setting the median of
several launches timed with HIP events, checked against the closed form.

  python tools/project_blocks_sweep.py SELECT_BLOCKS_RUN=0 SELECT_BLOCKS_RUN=8 ...
  (a setting may hold several knobs: SELECT_BLOCKS_RUN=8,SELECT_BLOCKS_WG_PER_CU=4)
"""
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from fq_amd import abi, ops  # noqa: E402
from fq_amd._lib import check, lib  # noqa: E402
from fq_amd.expr import chain, predicate  # noqa: E402

from bench import project_closed_form  # noqa: E402

U = abi.DT_UINT64
ROWS = int(float(os.environ.get("ROWS", "1.25e9")))
BR = int(os.environ.get("BLOCK_ROWS", "10000"))
REPS = int(os.environ.get("REPS", "7"))
PARTS = int(os.environ.get("PARTS", "1"))  # resident partitions cycled through (bench.py p1 holds 8)
FIRST = int(os.environ.get("FIRST", "0"))  # index of the first partition (rows from FIRST * ROWS)


def main():
    cols = [ops.numbers_column((FIRST + p) * ROWS, ROWS) for p in range(PARTS)]
    # OUT_SHIFT_KB: the outputs start this many KB into oversized buffers (placement A/B within one process)
    shifts = [int(x) for x in os.environ.get("OUT_SHIFT_KB", "0").split(",")]
    # OUT_SETS: separately allocated output pairs, each timed (placement A/B within one process)
    nsets = int(os.environ.get("OUT_SETS", "1"))
    # OUT_ALLOC=contig: output pairs from hipExtMallocWithFlags(hipDeviceMallocContiguous), raw pointers
    # (timed only: the parity check needs torch buffers)
    contig_out = os.environ.get("OUT_ALLOC", "") == "contig"
    # OUT_PAIR_SHIFT_KB: both outputs in ONE allocation, the second starting ROWS * 8 + shift KB after
    # the first (the two write streams' relative placement; each shift is one "output set")
    pair_shifts = [int(x) for x in os.environ.get("OUT_PAIR_SHIFT_KB", "").split(",") if x]
    if pair_shifts:
        one = torch.empty(2 * ROWS * 8 + max(pair_shifts) * 1024 + 4096, dtype=torch.uint8, device="cuda")
        nsets = len(pair_shifts)
    if contig_out:
        hip = C.CDLL("libamdhip64.so.7")  # torch's runtime, already loaded
        hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]

        def raw(nbytes):
            pp = C.c_void_p()
            rc = hip.hipExtMallocWithFlags(C.byref(pp), nbytes, 0x4)
            if rc != 0:
                raise SystemExit("hipExtMallocWithFlags(contiguous) failed: %d" % rc)
            return pp.value
        bigs = [[raw(ROWS * 8 + max(shifts) * 1024 + 4096) for _ in range(2)] for _ in range(nsets)]
    elif not pair_shifts:
        bigs = [[torch.empty(ROWS * 8 + max(shifts) * 1024 + 4096, dtype=torch.uint8, device="cuda")
                 for _ in range(2)] for _ in range(nsets)]
    nb = -(-ROWS // BR)
    counts = ops.Workspace(8 * nb)
    ws = ops.Workspace(max(lib.fq_filter_project_blocks_workspace_bytes(), lib.fq_filter_project_workspace_bytes(ROWS)))
    pred = predicate(U, [("%", 8)], "<", 3)
    exprs = (abi.fq_expr * 2)(chain(U, [("+", 1)])[0], chain(U, [("/", 2)])[0])
    settings = [(si, sh, st) for si in range(nsets) for sh in shifts for st in (sys.argv[1:] or ["SELECT_BLOCKS_RUN=1"])]
    kept = C.c_int64(0)
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream)
    cs = [col.col() for col in cols]
    exps = [project_closed_form((FIRST + p) * ROWS, (FIRST + p) * ROWS + ROWS - 1) for p in range(PARTS)]
    alg = 8 * ROWS + 16 * exps[0][0]
    for si, shift, setting in settings:
        if pair_shifts:
            outs = [ops.DeviceColumn(one, ROWS, U, offset=0),
                    ops.DeviceColumn(one, ROWS, U, offset=ROWS * 8 + pair_shifts[si] * 1024)]
            ptrs = (C.c_void_p * 2)(outs[0].ptr, outs[1].ptr)
        elif contig_out:
            outs = []
            ptrs = (C.c_void_p * 2)(bigs[si][0] + shift * 1024, bigs[si][1] + shift * 1024)
        else:
            outs = [ops.DeviceColumn(b, ROWS, U, offset=shift * 1024) for b in bigs[si]]
            ptrs = (C.c_void_p * 2)(outs[0].ptr, outs[1].ptr)
        ops.tune_reset()
        contig = False
        for kv in setting.split(","):
            if kv == "CONTIG":  # fq_filter_project (contiguous output, look-back) instead
                contig = True
                continue
            k, v = kv.split("=")
            ops.tune_set(k, int(v))

        def launch(p):
            if contig:
                check(lib.fq_filter_project(C.byref(cs[p]), C.byref(pred), exprs, 2, ptrs, C.byref(kept), ws.ptr,
                                            ws.nbytes, sp))
                return
            check(lib.fq_filter_project_blocks(C.byref(cs[p]), BR, C.byref(pred), exprs, 2, ptrs, counts.ptr,
                                               C.byref(kept), ws.ptr, ws.nbytes, sp))
        for o in outs[:1]:
            o.buf.zero_()
        launch(PARTS - 1)
        sums = tuple(int(o.buf[o.offset:o.offset + ROWS * 8].view(torch.int64).sum().item()) % (1 << 64) for o in outs)
        if contig_out:
            sums = exps[-1][1:]
        if (kept.value,) + sums != exps[-1]:
            print("%s: PARITY FAILURE %r != %r" % (setting, (kept.value,) + sums, exps[-1]), flush=True)
            continue
        ms = []
        for r in range(REPS * PARTS):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            launch(r % PARTS)
            e1.record(stream)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        med = statistics.median(ms)
        print("%s (%d partitions from %d, output set %d +%d KB, second output +%s KB): %.3f ms (min %.3f) = %.0f GB/s algorithmic, frac %.3f" % (
            setting, PARTS, FIRST, si, shift, pair_shifts[si] if pair_shifts else "-", med, min(ms), alg / med / 1e6, alg / med / 1e6 / 8000), flush=True)


if __name__ == "__main__":
    main()
