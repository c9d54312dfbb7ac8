"""In-ONE-process A/B of the engine's shared device queues (FQ_OPT_STREAMS)
on the aggregate queries: the pipes' launches on 1 queue (back to back) or
spread over n (a launch's tail and the next one's ramp overlap).  Configs
alternate round by round; every step's row is checked against the closed form.

python tools/streams_ab.py [rounds] [steps] [query] [n ...] > gpurun_out/streams_ab.json"""
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
CONFIGS = [int(x) for x in sys.argv[4:]] or [1, 2]
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
    for r in range(ROUNDS):
        for c in (CONFIGS if r % 2 == 0 else CONFIGS[::-1]):
            eng.set_option(OPT_STREAMS, c)
            for _ in range(3):
                if row() != want:
                    raise SystemExit("PARITY FAILURE at %d queues" % c)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(STEPS):
                got = row()
            dt = (time.perf_counter() - t0) / STEPS * 1e3
            if got != want:
                raise SystemExit("PARITY FAILURE at %d queues" % c)
            res[c].append(dt)
    eng.set_option(OPT_STREAMS, 1)
    eng.close()
    print(json.dumps({"rounds": ROUNDS, "steps": STEPS, "workload": sql, "result": list(want),
                      "configs": {"STREAMS=%d" % c: {"step_ms_median": statistics.median(v), "step_ms_all": v}
                                  for c, v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
