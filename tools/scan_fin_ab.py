"""A/B in ONE process of what a C3 step costs beyond its scans (round 5):

  kernel level -- 8 back-to-back fq_aggregate scans of resident 10 GB numbers_mt
  partitions on one stream, one event pair around all 8 (none between):
  "2" = scan + separate finalize launch, "0" = FQ_AGG_ONE_LAUNCH with
  FQ_TUNE_SCAN_FIN 0 (plain partial + agent release), "1" = SCAN_FIN 1
  (write-through partial), "split" = fq_aggregate_split (each fold on a second
  stream beside the next scan; the closing event waits for it); modes
  alternate round by round;

  engine level -- the C3 statement through fq_engine_execute (as bench.py's
  step) for "fold0" (scan + finalize on the queue), "fold1"
  (FQ_TUNE_ENGINE_FOLD_STREAM: folds on the fold queue) and "one1"
  (FQ_AGG_ONE_LAUNCH, SCAN_FIN 1), alternating: step wall time and the
  engine's scan span (FQ_OPT_PROFILE 2).

python tools/scan_fin_ab.py [rounds] > gpurun_out/scan_fin_ab.json"""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))
import torch  # noqa: E402

from fq_amd import abi, ops  # noqa: E402
from fq_amd._lib import check, lib  # noqa: E402
from fq_amd.engine import PROFILE_SPAN, Engine  # noqa: E402

ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 6
N = 10_000_000_000
P = 1_250_000_000
ALL = abi.AGG_SUM | abi.AGG_COUNT | abi.AGG_MAX | abi.AGG_MIN


def kernel_level():
    cols = [ops.numbers_column(i * P, P) for i in range(8)]
    # one workspace per partition, as the engine's pipes each have their own:
    # a scan never waits for the previous partition's fold
    wss = [ops.aggregate_workspace() for _ in range(8)]
    out = torch.empty(48 * 8, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    sp = C.c_void_p(s.cuda_stream)
    ccols = [c.col() for c in cols]

    fold = torch.cuda.Stream()
    ev = torch.cuda.Event()
    ev.record(s)  # torch creates the HIP event on its first record
    fp = C.c_void_p(fold.cuda_stream)

    def run(m):
        mask = ALL | (abi.AGG_ONE_LAUNCH if m in (0, 1) else 0)
        for i, cc in enumerate(ccols):
            dst = C.c_void_p(out.data_ptr() + 48 * i)
            ws = wss[i]
            if m == "split":
                check(lib.fq_aggregate_split(C.byref(cc), 10000, None, None, mask, dst, ws.ptr, ws.nbytes, sp, fp,
                                             C.c_void_p(ev.cuda_event)))
            else:
                check(lib.fq_aggregate(C.byref(cc), 10000, None, None, mask, dst, ws.ptr, ws.nbytes, sp))
        if m == "split":  # the closing event (and the next round's scans) after every fold
            done = torch.cuda.Event()
            done.record(fold)
            s.wait_event(done)

    # 2 = no FQ_AGG_ONE_LAUNCH (scan + finalize launch); 0 / 1 = in-launch, SCAN_FIN form 0 / 1
    modes = (2, 0, 1, "split")
    res = {m: [] for m in modes}
    sums = {}
    for r in range(ROUNDS):
        for m in (modes if r % 2 == 0 else modes[::-1]):
            if m in (0, 1):
                ops.tune_set("SCAN_FIN", m)
            run(m)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(5):
                a.record(s)
                run(m)
                b.record(s)
                b.synchronize()
                res[m].append(a.elapsed_time(b))
            torch.cuda.synchronize()
            sums[m] = bytes(out.cpu().numpy())
    ops.tune_reset()
    assert len(set(sums.values())) == 1, "every form must give the same states"
    return {str(m): {"median_ms_8_scans": statistics.median(v), "min": min(v), "max": max(v), "n": len(v),
                     "per_scan_ms": statistics.median(v) / 8} for m, v in res.items()}


def engine_level():
    sql = ("SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(%d)" % N).encode()
    e = Engine(device=0, profile=PROFILE_SPAN)
    e.materialize_numbers(N)
    val = abi.fq_value()

    def step():
        r = C.c_void_p()
        check(lib.fq_engine_execute(e.h, sql, C.byref(r)))
        row = []
        for c in range(3):
            check(lib.fq_result_value(r, 0, c, C.byref(val)))
            row.append(val.bits)
        lib.fq_result_free(r)
        return row

    configs = ["fold0", "fold1", "one1"]
    res = {c: {"step": [], "span": []} for c in configs}
    s = N * (N - 1) // 2 % 2**64
    for r in range(ROUNDS):
        for c in (configs if r % 2 == 0 else configs[::-1]):
            ops.tune_reset()
            ops.tune_set("ENGINE_FOLD_STREAM", 1 if c == "fold1" else 0)
            ops.tune_set("ENGINE_ONE_LAUNCH", 1 if c == "one1" else 0)
            for _ in range(2):
                assert step() == [s // N, N - 1, 0]
            e.reset_stats()
            t0 = time.perf_counter()
            for _ in range(10):
                step()
            dt = (time.perf_counter() - t0) / 10 * 1e3
            st = e.stats()
            res[c]["step"].append(dt)
            res[c]["span"].append(st["scan_ms"] / 10)
    ops.tune_reset()
    e.close()
    out = {}
    for c, v in res.items():
        out[c] = {"step_ms_median": statistics.median(v["step"]), "step_ms_all": v["step"],
                                   "scan_span_ms_median": statistics.median(v["span"]),
                                   "step_over_span": statistics.median(v["step"]) / statistics.median(v["span"])}
    return out


if __name__ == "__main__":
    ops.require_gpu()
    k = kernel_level()
    torch.cuda.empty_cache()
    out = {"kernel_8_scans": k, "engine_c3_step": engine_level(), "rounds": ROUNDS,
           "note": "kernel: 2 = scan + finalize launch (round 4), 0 = in-launch finalize with an agent release, "
                   "1 = in-launch with write-through partials, split = the finalize on a second stream; "
                   "engine: fold0 / fold1 = FQ_TUNE_ENGINE_FOLD_STREAM, one1 = FQ_TUNE_ENGINE_ONE_LAUNCH"}
    print(json.dumps(out, indent=1))
