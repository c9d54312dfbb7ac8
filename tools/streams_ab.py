"""In-ONE-process A/B of an aggregate query over engine / kernel configs:
the engine's shared device queues (STREAMS=n, FQ_OPT_STREAMS: the pipes'
launches on 1 queue back to back, or spread over n) and launch-shape knobs
(KNOB=V[,KNOB=V...], abi.TUNE names; a bare integer n means STREAMS=n).
Configs alternate round by round; every step's row is checked against the
first one's.

python tools/streams_ab.py [rounds] [steps] [query] [config ...] > gpurun_out/streams_ab.json"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

bench._load_runtime()
torch, ops = bench.torch, bench.ops
from fq_amd.engine import OPT_STREAMS, PROFILE_SPAN, Engine  # noqa: E402

ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 4
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 20
QUERY = sys.argv[3] if len(sys.argv) > 3 else "c3"


def parse_config(a):
    if "=" not in a:
        return (("STREAMS", int(a)),)
    return tuple((k.upper(), int(v)) for k, v in (kv.split("=") for kv in a.split(",")))


CONFIGS = [parse_config(a) for a in (sys.argv[4:] or ["1", "2"])]
N = 10_000_000_000


def main():
    ops.require_gpu()
    sql = bench.QUERIES[QUERY].format(N=N)
    eng = Engine(device=0, profile=PROFILE_SPAN)
    eng.materialize_numbers(N, 0, 1)
    torch.cuda.synchronize()
    def row():
        return [v.bits for v in eng.execute_row(sql)]

    want = row()
    res = {c: [] for c in CONFIGS}
    span = {c: [] for c in CONFIGS}  # scan span per launch (FQ_OPT_PROFILE 2)
    for r in range(ROUNDS):
        for c in (CONFIGS if r % 2 == 0 else CONFIGS[::-1]):
            ops.tune_reset()
            eng.set_option(OPT_STREAMS, dict(c).get("STREAMS", 1))
            for k, v in c:
                if k != "STREAMS":
                    ops.tune_set(k, v)
            for _ in range(3):
                if row() != want:
                    raise SystemExit("PARITY FAILURE at %r" % (c,))
            torch.cuda.synchronize()
            eng.reset_stats()
            t0 = time.perf_counter()
            for _ in range(STEPS):
                got = row()
            dt = (time.perf_counter() - t0) / STEPS * 1e3
            st = eng.stats()
            span[c].append(st["scan_ms"] / max(st["scan_launches"], 1))
            if got != want:
                raise SystemExit("PARITY FAILURE at %r" % (c,))
            res[c].append(dt)
    ops.tune_reset()
    eng.set_option(OPT_STREAMS, 1)
    eng.close()
    print(json.dumps({"rounds": ROUNDS, "steps": STEPS, "workload": sql, "result": list(want),
                      "configs": {",".join("%s=%d" % kv for kv in c): {"step_ms_median": statistics.median(v),
                                                                          "step_ms_all": v,
                                                                          "scan_ms_per_launch": span[c]}
                                  for c, v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
