"""In-ONE-process A/B of the p1 engine step (bench.py --query p1) over
fq_jit_pblocks store variants (round 5): kept rows stored straight from the
lanes' registers (FQ_TUNE_SELECT_BLOCKS_STAGE 0, the round-4 kernel) against
staged in LDS by in-tile rank and written by consecutive threads as 16-byte row
pairs (STAGE S: a stage of 1/S of the tile, 256 x rows x 8 / S bytes of LDS,
which caps the workgroups per CU; a tile keeping more rows than the stage
holds takes several passes), at 8 / 16 / 32 rows per thread.  Configs alternate
round by round in one process (a fresh process after another freed its HBM runs
slower, profiles/r05_b_host_spread/).  Every config's first query is checked
against the closed forms (kept rows + both columns' wrapping sums), every timed
one by its kept count.

python tools/p1_stage_ab.py [rounds] [steps] [S:R ...] > gpurun_out/p1_stage_ab.json"""
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
from fq_amd.engine import OPT_STREAMS, Engine  # noqa: E402

ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 4
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 8
N = 10_000_000_000
# configs: S:R = (FQ_TUNE_SELECT_BLOCKS_STAGE, FQ_TUNE_SELECT_BLOCKS_ROWS), or any
# knobs as KNOB=V[,KNOB=V...] (abi.TUNE names; STREAMS=n is the engine's
# FQ_OPT_STREAMS, 1 when a config does not name it); argv[3:] overrides the default set


def parse_config(a):
    if "=" in a:
        return tuple((k.upper(), int(v)) for k, v in (kv.split("=") for kv in a.split(",")))
    st, rows = (int(x) for x in a.split(":"))
    return (("SELECT_BLOCKS_STAGE", st), ("SELECT_BLOCKS_ROWS", rows))


CONFIGS = [parse_config(a) for a in (sys.argv[3:] or ["0:32", "1:16", "2:16", "2:32", "4:32"])]


def main():
    ops.require_gpu()
    sql = bench.PROJECT_SQL.format(N=N)
    mine = bench.shard(bench.generate_parts(N), 0, 1)
    expect = bench._p1_expect(mine)
    # P1_PROFILE: 2 (default) one span per query, 1 an event pair per launch, 0 none (kernel_ms then from rocprof)
    eng = Engine(device=0, profile=int(os.environ.get("P1_PROFILE", "2")))
    eng.materialize_numbers(N, 0, 1)
    torch.cuda.synchronize()

    def step(check=False):
        kept = s1 = s2 = 0
        with eng.execute_blocks(sql, 0, 1) as st:
            for b in st:
                if check:
                    k, x, y = bench._device_block_sums(b)
                    kept, s1, s2 = kept + k, (s1 + x) % bench.U64, (s2 + y) % bench.U64
                else:
                    kept += b.rows
        return (kept, s1, s2) if check else kept

    res = {c: {"step_ms": [], "kernel_ms": [], "frac": []} for c in CONFIGS}
    for r in range(ROUNDS):
        for c in (CONFIGS if r % 2 == 0 else CONFIGS[::-1]):
            ops.tune_reset()
            eng.set_option(OPT_STREAMS, dict(c).get("STREAMS", 1))
            for k, v in c:
                if k != "STREAMS":
                    ops.tune_set(k, v)
            got = step(check=(r == 0))
            if r == 0 and got != expect:
                raise SystemExit("PARITY FAILURE %r: got %r expected %r" % (c, got, expect))
            step()
            eng.reset_stats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(STEPS):
                if step() != expect[0]:
                    raise SystemExit("PARITY FAILURE %r: kept count" % (c,))
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / STEPS * 1e3
            st = eng.stats()
            launches = max(st["project_launches"], 1)
            kms = st["project_ms"] / launches
            res[c]["step_ms"].append(dt)
            res[c]["kernel_ms"].append(kms)
            res[c]["frac"].append(st["project_bytes"] / launches / (kms * 1e-3) / 1e9 / bench.HBM_PEAK_GBPS
                                  if kms > 0 else None)
    ops.tune_reset()
    eng.close()
    out = {"rounds": ROUNDS, "steps": STEPS, "workload": sql, "configs": {}}
    for c, v in res.items():
        out["configs"][",".join("%s=%d" % kv for kv in c)] = {
            "step_ms_median": statistics.median(v["step_ms"]), "kernel_ms_median": statistics.median(v["kernel_ms"]),
            "frac_median": statistics.median(v["frac"]) if None not in v["frac"] else None, "kernel_ms_all": v["kernel_ms"], "step_ms_all": v["step_ms"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
