"""How long does a process's scan stay slow after ANOTHER process freed a lot
of HBM?  (profiles/r05_b_host_spread/: a run right after a free scans 3-4 %
slower.)  Mode "free": a child process allocates and touches GB of HBM, frees
it and exits; then this process runs the C3 statement back to back for
SECONDS and prints each step's wall time and scan span with its time since the
child exited.  Mode "none": the same without the child.

python tools/reclaim_probe.py free|none [GB] [SECONDS] > gpurun_out/reclaim_probe_<mode>.json"""
import ctypes as C
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODE = sys.argv[1] if len(sys.argv) > 1 else "free"
GB = int(sys.argv[2]) if len(sys.argv) > 2 else 80
SECONDS = float(sys.argv[3]) if len(sys.argv) > 3 else 12.0
N = 10_000_000_000

CHILD = """
import torch
x = torch.empty(%d * (1 << 30), dtype=torch.uint8, device="cuda")
x.fill_(1)
torch.cuda.synchronize()
del x
torch.cuda.empty_cache()
""" % GB


def main():
    sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))
    t_child = None
    if MODE == "free":
        # the child runs and exits BEFORE this process touches the GPU
        subprocess.run([sys.executable, "-c", CHILD], check=True, timeout=300)
        t_child = time.time()
    import torch  # noqa: F401

    from fq_amd import abi
    from fq_amd._lib import check, lib
    from fq_amd.engine import PROFILE_SPAN, Engine
    e = Engine(device=0, profile=PROFILE_SPAN)
    e.materialize_numbers(N)
    t_ready = time.time()
    sql = ("SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(%d)" % N).encode()
    val = abi.fq_value()
    steps = []
    t0 = time.time()
    while time.time() - t0 < SECONDS:
        e.reset_stats()
        a = time.perf_counter()
        r = C.c_void_p()
        check(lib.fq_engine_execute(e.h, sql, C.byref(r)))
        check(lib.fq_result_value(r, 0, 1, C.byref(val)))
        lib.fq_result_free(r)
        b = time.perf_counter()
        st = e.stats()
        now = time.time()
        steps.append({"t_since_child_s": (now - t_child) if t_child else None, "t_since_ready_s": now - t_ready,
                      "step_ms": (b - a) * 1e3, "span_ms": st["scan_ms"],
                      "frac": 8e10 / (st["scan_ms"] * 1e-3) / 8e12})
        assert val.bits == N - 1
    e.close()
    # per-second medians
    buckets = {}
    for s in steps:
        buckets.setdefault(int(s["t_since_ready_s"]), []).append(s["frac"])
    summary = {k: sorted(v)[len(v) // 2] for k, v in sorted(buckets.items())}
    print(json.dumps({"mode": MODE, "gb_freed_by_child": GB if MODE == "free" else 0,
                      "ready_after_child_s": (t_ready - t_child) if t_child else None,
                      "frac_median_per_second_since_ready": summary, "steps": len(steps),
                      "first_10": steps[:10]}, indent=1))


if __name__ == "__main__":
    main()
