#!/usr/bin/env python3
"""bench.py -- rows/s + achieved HBM GB/s on the numbers_mt aggregation hot path
(BASELINE.json metric), 1..8 GPUs of one node.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--query c3]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Workload (BASELINE.json configs[2], the north_star query):
  SELECT sum(number)/count(number), max(number), min(number)
  FROM system.numbers_mt(1e10 x N_gpus)
Weak scaling: every GPU owns 1e10 rows = its share [8r/G, 8(r+1)/G) of the
8 numbers_mt partitions, materialised in HBM before timing (the 8-GPU run is
configs[4], numbers_mt(8e10)).  --rows-total 1e10 instead fixes N (strong
scaling: the 10B-row query split over 1/2/4/8 GPUs).  One step = the hot path over the resident
column: per partition one fused scan kernel (sum/count/max/min in one read)
-> partial states -> AggregateFinal merge, across GPUs one RCCL all-reduce of
the 48-byte states over xGMI.  Rank 0 prints ONE JSON line.
"""
import argparse
import glob
import json
import os
import platform
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "fuse-query_amd"), os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def _numbers_module():
    """fq_amd/numbers.py on its own: importing it through the package would run
    fq_amd/__init__.py, which loads the HIP library."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("fq_numbers", os.path.join(ROOT, "fuse-query_amd", "fq_amd",
                                                                             "numbers.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


_numbers = _numbers_module()
BLOCK_SIZE, generate_parts, shard, stream_rows = (_numbers.BLOCK_SIZE, _numbers.generate_parts, _numbers.shard,
                                                  _numbers.stream_rows)

sys.path.insert(0, os.path.join(ROOT, "tools"))
from srchash import kernel_sources_sha256  # noqa: E402

# torch and the HIP library are imported by _load_runtime(), after the
# launcher decision: a `--gpus N` parent that starts the ranks never loads the
# HIP runtime (it only spawns processes), and the C-host leg runs as a child
# before this process touches the GPU.
torch = dist = abi = ops = fqd = Engine = None
OPT_GROUP_CHUNK_ROWS = PROFILE_SPAN = None
HIP_MODULES = ("torch", "fq_amd._lib", "fq_amd.ops", "fq_amd.engine")


def _load_runtime():
    global torch, dist, abi, ops, fqd, Engine, OPT_GROUP_CHUNK_ROWS, PROFILE_SPAN
    import torch as _torch
    import torch.distributed as _dist

    from fq_amd import abi as _abi
    from fq_amd import dist as _fqd
    from fq_amd import ops as _ops
    from fq_amd.engine import OPT_GROUP_CHUNK_ROWS as _ogc
    from fq_amd.engine import PROFILE_SPAN as _ps
    from fq_amd.engine import Engine as _Engine
    torch, dist, abi, ops, fqd, Engine, OPT_GROUP_CHUNK_ROWS, PROFILE_SPAN = (
        _torch, _dist, _abi, _ops, _fqd, _Engine, _ogc, _ps)

METRIC = "rows/s + achieved HBM GB/s on 10B-row numbers_mt agg, 1/2/4/8 GPUs"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# reference README.md:57 / :62 (8 vCPU KVM), BASELINE.md section 1: the only
# published numbers for these exact queries (sum; sum/count, max, min)
README_SECONDS = {"c2": (1.77, 57), "max": (2.83, 58), "max1": (6.13, 59), "avg": (2.04, 61), "c3": (6.40, 62)}
README_ROWS_PER_S = {q: 1e10 / t for q, (t, _) in README_SECONDS.items()}
README_REF = {q: "reference README.md:%d (%.2f s for 1e10 rows, 8 vCPU KVM)" % (line, t)
              for q, (t, line) in README_SECONDS.items()}
U64 = 2**64

QUERIES = {
    "c2": "SELECT sum(number) FROM system.numbers_mt({N})",
    "c3": "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt({N})",
    "c4": "SELECT max(number+1) FROM system.numbers_mt({N}) WHERE (number%8)<3",
    # the README's other timed queries (README.md:58-61; count(number) aside:
    # it needs no column read)
    "max": "SELECT max(number) FROM system.numbers_mt({N})",
    "max1": "SELECT max(number+1) FROM system.numbers_mt({N})",
    "avg": "SELECT sum(number) / count(number) FROM system.numbers_mt({N})",
    # not a BASELINE config: filtered SUM, which needs the per-block emptiness
    # of the reference's state machine (block-mode scan)
    "c4s": "SELECT sum(number+1) FROM system.numbers_mt({N}) WHERE (number%8)<3",
    # not a BASELINE config: GROUP BY (no reference transform)
    "g1": "SELECT number%1000, count(number), sum(number), max(number) FROM system.numbers_mt({N}) "
          "GROUP BY number%1000",
    # high cardinality: more groups than an LDS table holds (radix-partitioned launches)
    "g2": "SELECT number%100000, count(number), sum(number), max(number) FROM system.numbers_mt({N}) "
          "GROUP BY number%100000",
}
GROUP_MOD = {"g1": 1000, "g2": 100000}
# not a BASELINE config: FilterTransform -> ProjectionTransform (SURVEY 8f rank
# 1), the README's expressions without its LIMIT.  Its result is 3.75e9 rows x 2
# columns (60 GB), left in HBM: measured through the engine's block stream
# (fq_engine_execute_blocks), checked by kept count and per-column wrapping
# sums (closed forms).
PROJECT_SQL = "SELECT number+1, number/2 FROM system.numbers_mt({N}) WHERE (number%8)<3"


def closed_form(query, n):
    """Expected results for numbers 0..n-1 (n a multiple of 80,000: no dropped rows)."""
    s = (n * (n - 1) // 2) % U64
    if query == "c2":
        return [s]
    if query == "c3":
        return [s // n, n - 1, 0]
    if query == "max":
        return [n - 1]
    if query == "max1":
        return [n]
    if query == "avg":
        return [s // n]
    if query in GROUP_MOD:
        m = GROUP_MOD[query]
        per = n // m  # n is a multiple of 800,000
        return [(k, per, (k * per + m * per * (per - 1) // 2) % U64, k + m * (per - 1)) for k in range(m)]
    if query == "c4s":
        tot = 0
        for r in range(3):
            k = (n - r + 7) // 8 if n > r else 0
            tot += 8 * k * (k - 1) // 2 + (r + 1) * k
        return [tot % U64]
    top = n - 1
    while top % 8 >= 3:
        top -= 1
    return [top + 1]


def project_closed_form(b, e):
    """(kept rows, sum(number+1), sum(number/2)) over rows b..e with number%8 < 3."""
    kept = s1 = s2 = 0
    for c in range(3):
        j0 = max(0, -(-(b - c) // 8))
        j1 = (e - c) // 8 if e >= c else -1
        cnt = max(0, j1 - j0 + 1)
        sj = (j0 + j1) * cnt // 2
        kept += cnt
        s1 += 8 * sj + cnt * (c + 1)
        s2 += 4 * sj + cnt * (c // 2)
    return kept, s1 % U64, s2 % U64


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def settle(step, seconds, world, backend):
    """Untimed steps for about `seconds` before the warmup.  For a few seconds
    after a process frees HBM the driver clears it in the background, and a
    scan that overlaps the clearing runs 3-4 % slower: in a fresh process, the
    first second after another process freed 80 GB, the first three after 160 GB
    (profiles/r05_j_reclaim_probe/; the GPU test suite before a bench frees more).
    At world > 1 every step is a collective, so every rank runs the same count:
    the most any rank needs for the rest of `seconds` at its SECOND step's pace
    (the first compiles hipRTC kernels and maps buffers: at its pace a c4
    settle ran ~0.1 s instead of 3).  -> steps run."""
    if seconds <= 0:
        return 0
    t0 = time.perf_counter()
    step()
    t1 = time.perf_counter()
    step()
    t2 = time.perf_counter()
    one = max(t2 - t1, 1e-4)
    n = max(int((seconds - (t2 - t0)) / one), 0)
    if world > 1:
        t = torch.tensor([n], dtype=torch.int64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n = int(t.item())
    for _ in range(n):
        step()
    return n + 2


def latest_pmc_traffic(kernel_substr, query, rows_per_launch):
    """(HBM bytes per launch scaled to rows_per_launch, provenance) from the
    most recently MEASURED committed rocprofv3 --pmc summary of this query
    (profiles/*pmc_<query>[_.]*.json, tools/pmc_summary.py, gfx950 FETCH_SIZE
    x2 correction applied).  Measurement order is the summary's
    `measured_at_unix` stamp (tools/pmc_import.py: the import time, which
    follows the gpurun call that measured it; summaries from before the stamp
    carry their commit's time), not its file name; files without a stamp count
    as oldest.  The summary must have been measured on the current kernel
    sources (its query_sources_sha256): otherwise traffic is None and the
    provenance says the file is stale.  The fingerprint covers the query's own
    kernel sources (tools/srchash.py QUERY_SOURCES)."""
    files = set(glob.glob(os.path.join(ROOT, "profiles", "*pmc_%s.json" % query)) +
                glob.glob(os.path.join(ROOT, "profiles", "*pmc_%s_*.json" % query)))
    summaries = []
    for f in files:
        try:
            d = json.load(open(f))
        except Exception:
            continue
        summaries.append((float(d.get("measured_at_unix") or 0.0), os.path.basename(f), d))
    summaries.sort(key=lambda x: (x[0], x[1]))
    subs = [kernel_substr] if isinstance(kernel_substr, str) else list(kernel_substr)
    cur = kernel_sources_sha256(query)
    stale = None
    for when, name, d in reversed(summaries):  # the newest measured on the current sources; else report the newest
        ks = [k for k in d.get("kernels", []) if k.get("hbm_bytes_per_launch") and
              any(x in k.get("name", "") for x in subs)]
        if not ks:
            continue
        src = {"file": "profiles/" + name, "measured_at_commit": d.get("measured_at_commit"),
               "measured_at_unix": d.get("measured_at_unix"), "query_sources_sha256": d.get("query_sources_sha256")}
        if d.get("query_sources_sha256") != cur:
            if stale is None:
                src["status"] = "stale: kernel sources changed since this PMC pass (current %s)" % cur[:12]
                stale = src
            continue
        src["status"] = "current kernel sources"
        # several names: one launch of each per unit (the partitioned GROUP BY's kernel set)
        per = sum(k["hbm_bytes_per_launch"] for k in ks)
        rows = ks[0].get("rows_per_launch")
        return (per * rows_per_launch / rows if rows else None), src
    if stale is not None:
        return None, stale
    return None, {"status": "no PMC summary for this query in profiles/"}


def host_split(st, steps, ms_per_step, world):
    """Rank 0's step, split by the engine's own host timers (fq_engine_stats),
    per step.  One GPU: plan (SQL -> pipeline), exec (pipeline until the result
    block), first_launch (query start -> first scan enqueued), tail (the scans'
    end event seen -> the result block: merge + AggregateFinal), outside_exec
    (the step minus plan and exec: result rows, frees, the binding's calls).  World > 1: the
    distributed split -- partial (fq_engine_execute_partial: plan + this rank's
    scans + local merge), exchange (the all-reduce rounds, including the wait for
    the slowest rank), final (AggregateFinal over every rank's states) -- and
    what those three account for of the step (the rest is the binding's
    Python)."""
    out = {"plan": st["plan_ms"] / steps, "first_launch": st["first_launch_ms"] / steps, "exec": st["exec_ms"] / steps}
    if world == 1:
        out.update({"tail": st["tail_ms"] / steps, "tail_states": st["complete_ms"] / steps,
                    "outside_exec": ms_per_step - (st["plan_ms"] + st["exec_ms"]) / steps})
    if world > 1:
        part, xch, fin = (st[k] / steps for k in ("partial_ms", "exchange_ms", "final_ms"))
        out.update({"partial": part, "exchange": xch, "final": fin,
                    "scans_event_ms": st["scan_ms"] / steps,
                    "exchange_rounds": st["exchange_rounds"] / steps,
                    "exchange_bytes": st["exchange_bytes"] / steps,
                    "accounted_frac": (part + xch + fin) / ms_per_step if ms_per_step else None})
    return out


CPU_RUNS = 3  # the median of 3 timed runs after one warmup


def cpu_baseline(sample_rows, threads, query="c3"):
    """Restated reference CPU path (oracle/fq_oracle.c) on the host cores,
    over the same query as the GPU line."""
    import oracle_c
    if query in GROUP_MOD:
        return cpu_baseline_group(sample_rows, threads, query)
    from fq_amd.expr import chain, predicate
    native = True
    try:
        oracle_c.build(native=True)
    except Exception:
        native = False
    pred = None
    if query == "c2":
        aggs = [(abi.AGG_SUM, None)]
    elif query == "c3":
        aggs = [(abi.AGG_SUM, None), (abi.AGG_COUNT, None), (abi.AGG_MAX, None), (abi.AGG_MIN, None)]
    elif query == "max":
        aggs = [(abi.AGG_MAX, None)]
    elif query == "max1":
        aggs = [(abi.AGG_MAX, chain(abi.DT_UINT64, [("+", 1)])[0])]
    elif query == "avg":
        aggs = [(abi.AGG_SUM, None), (abi.AGG_COUNT, None)]
    else:
        aggs = [(abi.AGG_MAX if query == "c4" else abi.AGG_SUM, chain(abi.DT_UINT64, [("+", 1)])[0])]
        pred = predicate(abi.DT_UINT64, [("%", 8)], "<", 3)
    L = oracle_c.lib(native)
    n = sample_rows

    def check(rows):
        res = [oracle_c.merge_states(op, [r[a] for r in rows])[2] for a, (op, _) in enumerate(aggs)]
        if query == "c3":
            s, c, mx, mn = res
            res = [s // c, mx, mn]
        elif query == "avg":
            res = [res[0] // res[1]]
        assert res == closed_form(query, n), "cpu baseline parity"

    def timed(run):
        t0 = time.perf_counter()
        rows = run()
        dt = time.perf_counter() - t0
        check(rows)
        return dt

    def reference_shape():  # 8 partitions, one thread each (the reference's 8-way parallelism)
        rows, st, err = oracle_c.numbers_partial(n, aggs, pred=pred, threads=threads, native=native)
        assert not any(st), err
        return rows

    # one warmup, then the median of 3 timed runs
    oracle_c.numbers_partial(min(n, 80_000_000), aggs, pred=pred, threads=threads, native=native)
    runs = [timed(reference_shape) for _ in range(CPU_RUNS)]
    dt = statistics.median(runs)
    # the all-cores leg: the box's CPU share, each partition's blocks cut into
    # slices so more than 8 threads have work (the reference cannot: 8 fixed
    # partitions, numbers_table.rs:29-55)
    cores = host_threads()
    slices = max(1, -(-cores // 8))

    def all_cores():
        rows, rc, err = oracle_c.numbers_partial_split(n, aggs, pred=pred, threads=cores, slices=slices,
                                                       native=native)
        assert not rc, err
        return rows

    all_runs = [timed(all_cores) for _ in range(CPU_RUNS)]
    del L
    return {
        "value": n / dt, "unit": "rows/s", "cores": threads, "kind": "port",
        "median_of": CPU_RUNS, "runs_s": runs, "warmup": "one run over numbers_mt(%d)" % min(n, 80_000_000),
        "all_cores": {"value": n / statistics.median(all_runs), "cores": cores, "runs_s": all_runs,
                      "median_of": CPU_RUNS, "tasks": 8 * slices,
                      "note": "each of the 8 partitions' 10,000-row blocks cut into %d runs, %d tasks on %d threads "
                              "(the box's CPU share: sched affinity capped by OMP_NUM_THREADS); more parallelism "
                              "than the reference's fixed 8 partitions allow" % (slices, 8 * slices, cores)},
        "sample": "%s query over numbers_mt(%d): 8 partitions, one thread per partition, "
                  "10,000-row blocks regenerated per block, one pass per aggregator%s "
                  "(oracle/fq_oracle.c, %s); median %.2f s wall of %d runs on %s (nproc=%d).  A lower bound on the "
                  "reference's own CPU cost: the port keeps its per-block state machine but not its per-block 1-row "
                  "arrays, serde_json partial states or tokio channel hand-offs (%s)"
                  % (query.upper(), n, ", constant broadcast + filter compaction per block" if pred else "",
                     "-O3 -march=native" if native else "-O3 -march=x86-64-v2", dt, CPU_RUNS, _cpu_model(),
                     os.cpu_count() or 0, README_REF.get(query, "no published reference time for this query")),
    }


def host_threads():
    """The CPU share this process may use: its affinity set, capped by
    OMP_NUM_THREADS when set (16 on the GPU box, whose nproc is the whole host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_baseline_project(sample_rows, threads):
    """Filter -> Projection on the host cores: oracle/fq_oracle.c
    fqo_numbers_project (per 10,000-row block: compaction, then each
    expression into its own array), over numbers_mt(sample_rows)."""
    import oracle_c
    from fq_amd.expr import chain, predicate
    native = True
    try:
        oracle_c.build(native=True)
    except Exception:
        native = False
    U = abi.DT_UINT64
    pred = predicate(U, [("%", 8)], "<", 3)
    outs = [chain(U, [("+", 1)])[0], chain(U, [("/", 2)])[0]]
    n = sample_rows - sample_rows % 80_000
    oracle_c.numbers_project(8_000_000, outs, pred=pred, threads=threads, native=native)  # warm
    t0 = time.perf_counter()
    kept, sums = oracle_c.numbers_project(n, outs, pred=pred, threads=threads, native=native)
    dt = time.perf_counter() - t0
    assert (kept, sums[0], sums[1]) == project_closed_form(0, n - 1), "cpu baseline parity"
    return {
        "value": n / dt, "unit": "rows/s", "cores": threads, "kind": "port",
        "sample": "P1 over numbers_mt(%d): 8 partitions, one thread per partition, 10,000-row blocks regenerated "
                  "per block, FilterTransform compaction then each projected expression into its own array "
                  "(transform_filter.rs:38-55, transform_projection.rs:45-56; oracle/fq_oracle.c "
                  "fqo_numbers_project, %s); %.2f s wall on %s (nproc=%d).  A lower bound on the reference's own "
                  "CPU cost (no arrow RecordBatch per block, no tokio hand-offs)"
                  % (n, "-O3 -march=native" if native else "-O3 -march=x86-64-v2", dt, _cpu_model(),
                     os.cpu_count() or 0),
    }


def _p1_expect(parts):
    """(kept, sum(number+1), sum(number/2)) over numbers_mt partitions (closed forms)."""
    kept = s1 = s2 = 0
    for _, b, e in parts:
        rows = stream_rows(b, e)
        k, x, y = project_closed_form(b, b + rows - 1)
        kept, s1, s2 = kept + k, (s1 + x) % U64, (s2 + y) % U64
    return kept, s1, s2


def _device_block_sums(b):
    """(valid rows, wrapping sum of each column over its valid rows) of one
    fq_device_block (block-stream layout or plain columns), on the GPU."""
    out = [int(b.rows)]
    n = b.columns[0].len if b.n_columns else 0
    valid = None
    if b.block_rows > 0 and n:
        counts = ops.device_view(b.d_counts, 8 * b.n_blocks).view(torch.int64)
        valid = (torch.arange(n, device="cuda") % b.block_rows) < \
            counts.repeat_interleave(b.block_rows)[:n]
    for j in range(b.n_columns):
        c = b.columns[j]
        if not c.len:
            out.append(0)
            continue
        col = ops.device_view(c.data, 8 * c.len).view(torch.int64)
        if valid is None:
            col = col[:b.rows]
        else:
            col = torch.where(valid, col, torch.zeros_like(col))
        out.append(int(col.sum().item()) % U64)
    return out


def run_project_engine(args, rank, world, local):
    """--query p1, default path: FilterTransform -> ProjectionTransform through
    the ENGINE (fq_engine_execute_blocks): SQL -> PipelineBuilder -> Source x P
    -> Filter -> Projection -> Merge, the projection of each device block one
    fq_filter_project_blocks launch (fq_jit_pblocks), pipe p on row queue p % 2, the
    filtered and projected DataBlocks handed to the host in HBM in the
    reference's per-10,000-row-block geometry (stream_expression.rs:38-50,
    transform_projection.rs:45-56).  One step = the whole query, every block
    pulled by the host; checked against the closed forms (every block's valid
    rows summed on the GPU) before and after the timed steps."""
    from fq_amd.engine import OPT_CHUNK_ROWS, Engine
    if args.rows_total:
        n_total = int(args.rows_total)
    else:
        n_total = int(args.rows_per_gpu) * world
    sql = PROJECT_SQL.format(N=n_total)
    mine = shard(generate_parts(n_total), rank, world)
    total_rows = sum(stream_rows(b, e) for _, b, e in mine)
    # FQ_OPT_PROFILE 2: the query's projection launches timed as one span over
    # the row queues (no event between two launches, engine/functions.h LaunchSpan)
    eng = Engine(device=local, profile=PROFILE_SPAN, streams=args.streams)
    if args.p1_chunk_rows:
        eng.set_option(OPT_CHUNK_ROWS, int(args.p1_chunk_rows))
    eng.materialize_numbers(n_total, rank, world)
    torch.cuda.synchronize()
    log(rank, "p1 (engine): %d partitions, %d rows (%.1f GB) resident on rank %d" % (
        len(mine), total_rows, total_rows * 8 / 1e9, rank))
    expect = _p1_expect(mine)

    def step(check=False):
        kept = s1 = s2 = 0
        blocks = 0
        with eng.execute_blocks(sql, rank, world) as st:
            for b in st:
                blocks += 1
                if check:
                    k, x, y = _device_block_sums(b)
                    kept, s1, s2 = kept + k, (s1 + x) % U64, (s2 + y) % U64
                else:
                    kept += b.rows
        return (kept, s1, s2) if check else kept, blocks

    settled = settle(step, args.settle_s, world, args.dist_backend)
    for _ in range(max(args.warmup, 1)):
        got, blocks = step(check=True)
        if got != expect:
            raise SystemExit("PARITY FAILURE: got %r expected %r" % (got, expect))
    log(rank, "result: kept rows and per-column wrapping sums == closed form (%d device blocks per query)" % blocks)
    eng.reset_stats()
    per_step = []
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    bad = 0
    for _ in range(args.steps):
        a = eng.stats()
        k, _ = step()
        b = eng.stats()
        bad |= k != expect[0]
        per_step.append(((b["project_ms"] - a["project_ms"]), (b["project_launches"] - a["project_launches"]),
                         (b["project_bytes"] - a["project_bytes"])))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if bad:
        raise SystemExit("PARITY FAILURE: a timed step kept another row count")
    st = eng.stats()
    got, _ = step(check=True)
    if got != expect:
        raise SystemExit("PARITY FAILURE after the timed steps: got %r expected %r" % (got, expect))
    launches = max(st["project_launches"], 1)
    avg_ms = st["project_ms"] / launches
    bytes_per_launch = st["project_bytes"] / launches
    rows_per_launch = st["project_rows"] / launches
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    steps_frac = sorted((by / max(l, 1)) / ((ms / max(l, 1)) * 1e-3) / 1e9 / HBM_PEAK_GBPS for ms, l, by in per_step)
    value = n_total * args.steps / dt
    if rank == 0:
        traffic, traffic_src = latest_pmc_traffic("fq_jit_pblocks", "p1", rows_per_launch)
        out = {
            "metric": METRIC, "value": value, "unit": "rows/s", "n_gpus": world, "ranks_seen": world,
            "steps": args.steps, "warmup": args.warmup, "settle": {"s": args.settle_s, "steps": settled},
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong" if args.rows_total else "weak", "vs_baseline": None,
            "vs_baseline_ref": "no published reference number for this query",
            "dtype": "u64", "data": "synthetic: system.numbers_mt iota column (u64), resident in HBM before timing",
            "config": {"workload": sql, "query": "p1", "rows_per_gpu": total_rows, "rows_total": n_total,
                       "partitions_per_gpu": len(mine), "block_rows": BLOCK_SIZE,
                       "device_blocks_per_step": blocks,
                       "path": "fq_engine_execute_blocks: SQL -> PipelineBuilder -> Source x P -> FilterTransform -> "
                               "ProjectionTransform (fq_filter_project_blocks per device block, fq_jit_pblocks) -> "
                               "Merge; the host pulls every filtered + projected DataBlock, left in HBM in the "
                               "reference's per-10,000-row-block geometry",
                       "parallelism": "dp%d (numbers_mt partitions sharded, no exchange)" % world},
            "achieved_hbm_gbps": achieved, "kernel_ms_per_launch": avg_ms,
            "scan_launches_per_step": st["project_launches"] / args.steps,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "fq_jit_pblocks (hipRTC-specialised) launched by the engine's ProjectionTransform, "
                                   "one launch per device block; algorithmic bytes = 8 B per row read + 8 B per kept "
                                   "row per projected column; timed by one HIP-event span per query over the engine's "
                                   "two row queues (the earliest first-launch start to the latest end event the last "
                                   "pipe records: launches overlapped across the queues, gaps included) / launches",
                         "bytes_per_launch": bytes_per_launch,
                         "frac_per_step": {"median": steps_frac[len(steps_frac) // 2], "min": steps_frac[0],
                                           "max": steps_frac[-1], "steps": len(steps_frac)}},
            "result": {"kept_rows_per_step": expect[0], "sum_number_plus_1": expect[1], "sum_number_div_2": expect[2]},
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline_project(int(args.cpu_sample_rows or 1e10), args.cpu_threads)
            except Exception as e:  # report, never hide
                out["cpu_baseline"] = {"error": repr(e)}
        if args.tuned:
            out["tune"] = args.tuned
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_project(args, rank, world):
    """--query p1 --project-path blocks|contiguous: the kernel alone at the C
    ABI over this rank's resident numbers_mt partitions, outputs in HBM; one
    step = every partition once.  blocks: fq_filter_project_blocks over the
    partition's 10,000-row blocks (block b's kept rows at output rows
    [b * 10,000, + count[b])); contiguous: fq_filter_project (one contiguous
    output per partition, decoupled look-back).  The launches cycle over
    --p1-output-sets freshly allocated output pairs, and the line reports the
    per-launch distribution (median / min / max) and each set's mean: which
    pages an output pair lands on moves the kernel's time."""
    import ctypes as C

    from fq_amd._lib import check, lib
    from fq_amd.expr import chain, predicate
    if args.rows_total:
        n_total = int(args.rows_total)
    else:
        n_total = int(args.rows_per_gpu) * world
    sql = PROJECT_SQL.format(N=n_total)
    mine = shard(generate_parts(n_total), rank, world)
    U = abi.DT_UINT64
    cols, expect = [], []
    for _, b, e in mine:
        rows = stream_rows(b, e)
        if rows != e - b + 1:
            raise SystemExit("p1 needs numbers_mt(N) with whole 10,000-row blocks per partition")
        cols.append(ops.numbers_column(b, rows))
        expect.append(project_closed_form(b, e))
    blocks = args.project_path == "blocks"
    maxr = max(c.len for c in cols)
    alloc = ops.contiguous_column if args.p1_outputs == "contiguous" else ops.empty_column
    nsets = max(1, args.p1_output_sets)
    sets = [[alloc(maxr, U), alloc(maxr, U)] for _ in range(nsets)]
    nb_max = -(-maxr // BLOCK_SIZE)
    counts = ops.Workspace(8 * nb_max)
    ws = ops.Workspace(max(lib.fq_filter_project_workspace_bytes(maxr), lib.fq_filter_project_blocks_workspace_bytes()))
    pred = predicate(U, [("%", 8)], "<", 3)
    exprs = (abi.fq_expr * 2)(chain(U, [("+", 1)])[0], chain(U, [("/", 2)])[0])
    ptr_sets = [(C.c_void_p * 2)(o[0].ptr, o[1].ptr) for o in sets]
    kept = C.c_int64(0)
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream)
    torch.cuda.synchronize()
    total_rows = sum(c.len for c in cols)
    log(rank, "p1 (%s kernel): %d partitions, %d rows (%.1f GB) resident on rank %d, %d output sets" % (
        args.project_path, len(cols), total_rows, total_rows * 8 / 1e9, rank, nsets))

    def launch(col, k, use_blocks=blocks):
        c = col.col()
        if use_blocks:
            check(lib.fq_filter_project_blocks(C.byref(c), BLOCK_SIZE, C.byref(pred), exprs, 2, ptr_sets[k], counts.ptr,
                                               C.byref(kept), ws.ptr, ws.nbytes, sp))
        else:
            check(lib.fq_filter_project(C.byref(c), C.byref(pred), exprs, 2, ptr_sets[k], C.byref(kept), ws.ptr,
                                        ws.nbytes, sp))
        return kept.value

    def checked(col, k, use_blocks=blocks):
        """(kept, wrapping sum of each output over its valid rows) of one
        launch: outputs zeroed first, so rows past a block's count add nothing."""
        for o in sets[k]:
            o.buf.zero_()
        n_kept = launch(col, k, use_blocks)
        n = col.len if use_blocks else n_kept
        sums = tuple(int(o.buf[:n * 8].view(torch.int64).sum().item()) % U64 for o in sets[k])
        if use_blocks:
            nb = -(-col.len // BLOCK_SIZE)
            if int(counts.buf[:8 * nb].view(torch.int64).sum().item()) != n_kept:
                raise SystemExit("PARITY FAILURE: block counts do not add up to the kept rows")
        return (n_kept,) + sums

    for _ in range(max(args.warmup, 1)):
        for i, (col, exp) in enumerate(zip(cols, expect)):
            got = checked(col, i % nsets)
            if got != exp:
                raise SystemExit("PARITY FAILURE: got %r expected %r" % (got, exp))
    log(rank, "result: kept rows and per-column wrapping sums == closed form on every partition")
    evs = []
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    kept_total = 0
    i = 0
    for _ in range(args.steps):
        for col in cols:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            kept_total += launch(col, i % nsets)
            e1.record(stream)
            evs.append((e0, e1, col.len, i % nsets))
            i += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if checked(cols[-1], 0) != expect[-1]:
        raise SystemExit("PARITY FAILURE after the timed steps")
    ms = [e0.elapsed_time(e1) for e0, e1, _, _ in evs]
    avg_ms = sum(ms) / len(ms)
    kept_per_launch = kept_total / len(evs)
    rows_per_launch = sum(r for _, _, r, _ in evs) / len(evs)
    bytes_per_launch = 8 * rows_per_launch + 16 * kept_per_launch
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    fr = sorted(bytes_per_launch / (m * 1e-3) / 1e9 / HBM_PEAK_GBPS for m in ms)
    set_ms = [sum(m for m, (_, _, _, k) in zip(ms, evs) if k == s) / max(1, sum(1 for e in evs if e[3] == s))
              for s in range(nsets)]
    value = n_total * args.steps / dt
    if rank == 0:
        kname = "fq_jit_pblocks" if blocks else "fq_jit_pselect"
        traffic, traffic_src = latest_pmc_traffic(kname, "p1", rows_per_launch)
        path = ("fq_filter_project_blocks at the C ABI per resident partition (the kernel alone, not the engine): "
                "the partition's 10,000-row blocks filtered and projected block by block, block b's kept rows at "
                "output rows [b * 10,000, + count[b]), per-block counts in HBM"
                if blocks else
                "fq_filter_project at the C ABI per resident partition: predicate, decoupled look-back, both "
                "expressions, one contiguous output per partition")
        out = {
            "metric": METRIC, "value": value, "unit": "rows/s", "n_gpus": world, "ranks_seen": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong" if args.rows_total else "weak", "vs_baseline": None,
            "vs_baseline_ref": "no published reference number for this query",
            "dtype": "u64", "data": "synthetic: system.numbers_mt iota column (u64), resident in HBM before timing",
            "config": {"workload": sql, "query": "p1", "rows_per_gpu": total_rows, "rows_total": n_total,
                       "partitions_per_gpu": len(cols), "block_rows": BLOCK_SIZE, "path": path,
                       "outputs": ("%d pairs in physically contiguous HBM (hipDeviceMallocContiguous), cycled per "
                                   "launch" if args.p1_outputs == "contiguous" else
                                   "%d pairs of torch caching-allocator buffers, cycled per launch") % nsets,
                       "parallelism": "dp%d (numbers_mt partitions sharded)" % world},
            "achieved_hbm_gbps": achieved, "kernel_ms_per_launch": avg_ms, "scan_launches_per_step": len(cols),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": fr[len(fr) // 2], "frac_of_mean_ms": achieved / HBM_PEAK_GBPS,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "%s (hipRTC-specialised), one launch per partition; algorithmic bytes = 8 B per "
                                   "row read + 16 B per kept row written; frac = the median launch" % kname,
                         "bytes_per_launch": bytes_per_launch,
                         "frac_per_launch": {"median": fr[len(fr) // 2], "min": fr[0], "max": fr[-1],
                                             "launches": len(fr)},
                         "ms_per_output_set": set_ms},
            "result": {"kept_rows_per_step": kept_total // args.steps},
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline_project(int(args.cpu_sample_rows or 1e10), args.cpu_threads)
            except Exception as e:  # report, never hide
                out["cpu_baseline"] = {"error": repr(e)}
        if args.tuned:
            out["tune"] = args.tuned
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _cpu_model():
    cpu = platform.processor() or platform.machine()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu


def cpu_baseline_group(sample_rows, threads, query):
    """GROUP BY on the host cores: oracle/fq_oracle.c fqo_numbers_group (the
    reference has no GROUP BY transform, so this is a plain CPU hash
    aggregation over the same 10,000-row blocks, one table per partition
    thread, merged), over numbers_mt(sample_rows)."""
    import numpy as np
    import oracle_c
    from fq_amd.expr import chain
    native = True
    try:
        oracle_c.build(native=True)
    except Exception:
        native = False
    m = GROUP_MOD[query]
    key = chain(abi.DT_UINT64, [("%", m)])[0]
    U = abi.DT_UINT64
    aggs = [(abi.AGG_COUNT, U, None), (abi.AGG_SUM, U, None), (abi.AGG_MAX, U, None)]
    n = sample_rows - sample_rows % 800_000  # closed form: whole cycles of every key per partition
    oracle_c.numbers_group(8_000_000, key, aggs, threads=threads, cap_groups=2 * m, native=native)  # warm
    t0 = time.perf_counter()
    keys, st = oracle_c.numbers_group(n, key, aggs, threads=threads, cap_groups=2 * m, native=native)
    dt = time.perf_counter() - t0
    o = np.argsort(keys)
    got = [(int(k), int(c), int(s), int(x)) for k, (c, s, x) in zip(keys[o], st[o])]
    assert got == closed_form(query, n), "cpu baseline parity"
    return {
        "value": n / dt, "unit": "rows/s", "cores": threads, "kind": "port",
        "sample": "%s query over numbers_mt(%d): 8 partitions, one thread per partition, 10,000-row blocks "
                  "regenerated per block, key and arguments evaluated per block, one hash-table insert per row, "
                  "partition tables merged (oracle/fq_oracle.c fqo_numbers_group, %s; no reference GROUP BY "
                  "transform exists to time); %.2f s wall on %s (nproc=%d)"
                  % (query.upper(), n, "-O3 -march=native" if native else "-O3 -march=x86-64-v2", dt, _cpu_model(),
                     os.cpu_count() or 0),
    }


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`--gpus N` (N > 1) started without a launcher: run N fresh rank
    processes through torch.distributed.run (127.0.0.1 rendezvous) and exit
    with their status.  This process never touches the GPU (it has made no HIP
    call when it gets here), and every rank is a new process, so no GPU state
    crosses a fork or an exec.  Rank 0's JSON line reaches stdout directly."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    print("[bench] launching %d ranks: %s" % (n, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def stdout_to_stderr(fn, *a):
    """Run fn with file descriptor 1 pointed at stderr: RCCL prints its version
    banner on stdout at communicator init, and stdout carries ONE JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        return fn(*a)
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def rccl_world1(eng, sql, expect, device, args):
    return stdout_to_stderr(_rccl_world1, eng, sql, expect, device, args)


def _rccl_world1(eng, sql, expect, device, args):
    """The multi-GPU step's transport at world 1: fq_engine_execute_rccl (partial
    -> the state exchange through the library's own RCCL communicator, host
    staged: memcpy -> H2D -> ncclAllReduce -> D2H -> sync -> final), steps x
    the same statement, every result checked.  The 8-GPU run uses the same
    calls; one box has one GPU and RCCL takes one rank per device, so this is
    the exchange's fixed cost, not its xGMI time."""
    try:
        comm = fqd.RcclComm.single(device)
    except Exception as e:  # report, never hide
        return {"error": repr(e)}
    try:
        for _ in range(max(args.warmup, 1)):
            r = list(fqd.execute(eng, sql, comm).rows[0])
        if r != expect:
            return {"error": "result %r != closed form %r" % (r, expect)}
        eng.reset_stats()
        t0 = time.perf_counter()
        bad = 0
        for _ in range(args.steps):
            bad |= list(fqd.execute(eng, sql, comm).rows[0]) != expect
        dt = time.perf_counter() - t0
        st = eng.stats()
        k = args.steps
        ms = dt / k * 1e3
        out = {"transport": "fq_engine_execute_rccl over fq_comm_init(world 1): ncclAllReduce of the [length, "
                            "states] row, staged through pinned host memory",
               "ms_per_step": ms, "result_ok": not bad,
               "partial_ms": st["partial_ms"] / k, "exchange_ms": st["exchange_ms"] / k,
               "final_ms": st["final_ms"] / k, "exchange_rounds": st["exchange_rounds"] / k,
               "exchange_bytes": st["exchange_bytes"] / k}
        log(0, "rccl world 1: %.3f ms/step, exchange %.1f us, %d B in %d round(s)"
            % (ms, out["exchange_ms"] * 1e3, out["exchange_bytes"], out["exchange_rounds"]))
        return out
    except Exception as e:
        return {"error": repr(e)}
    finally:
        comm.close()


def check_rank_device(args, rank, world, local):
    """This rank's GPU, checked by the rank itself (the launcher parent never
    touches HIP): RCCL needs one visible GPU per local rank; the gloo rehearsal
    lets ranks share the visible GPUs.  Exits non-zero when the GPU is missing."""
    ops.require_gpu()
    visible = torch.cuda.device_count()
    if args.dist_backend == "nccl" and world > 1 and local >= visible:
        raise SystemExit("bench.py rank %d: --gpus %d with RCCL needs a GPU per rank (LOCAL_RANK %d, %d visible; "
                         "--dist-backend gloo rehearses N ranks on fewer)" % (rank, args.gpus, local, visible))
    return local % visible if args.dist_backend == "gloo" else local


def run_c_host(args):
    """fq_c_client --bench STEPS N WARMUP as a child process (the C host of the
    C ABI: libfq_amd.so on /opt/rocm's HIP runtime, no Python or torch), over the
    same C3 workload; its JSON line, or an error record.  It materialises its
    own numbers_mt(N) (80 GB at 1e10 beside this process's 80 GB: 288 GB of
    HBM hold both)."""
    exe = os.path.join(ROOT, "fuse-query_amd", "lib", "fq_c_client")
    n_total = int(args.rows_total or args.rows_per_gpu)
    cmd = [exe, "--bench", str(args.steps), str(n_total), str(max(args.warmup, 1))]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    except Exception as e:  # report, never hide
        return {"error": repr(e), "cmd": " ".join(cmd[1:])}
    if p.returncode != 0:
        return {"error": "exit %d: %s" % (p.returncode, p.stderr.strip()[-500:]), "cmd": " ".join(cmd[1:])}
    try:
        out = json.loads(p.stdout.strip().splitlines()[-1])
    except Exception as e:
        return {"error": "unparsable output %r: %r" % (p.stdout[-300:], e)}
    out["cmd"] = "fuse-query_amd/lib/fq_c_client " + " ".join(cmd[1:])
    log(0, "c_host: %.1f G rows/s, %.3f ms/step, scan frac %.3f (C host, no torch)"
        % (out.get("value", 0) / 1e9, out.get("ms_per_step", 0), out.get("frac", 0)))
    return out


def cpu_only_line(args):
    """The restated reference CPU path alone (no GPU): BASELINE.md 2's C1 line
    (`--query c2 --rows-per-gpu 1e8`: SELECT sum(number) over numbers_mt(1e8)
    at 8 threads, BASELINE.json configs[0]) or any other query's, beside the
    README's published time for that query (taken at 1e10 rows, so scaled to
    the sample at the README's own rate, and said so)."""
    _load_runtime()
    n = int(args.rows_per_gpu)
    sql = QUERIES[args.query].format(N=n)
    cb = cpu_baseline(n, args.cpu_threads, args.query)
    out = {"metric": METRIC, "value": cb["value"], "unit": "rows/s", "n_gpus": 0, "higher_is_better": True,
           "kind": "cpu_baseline_only", "dtype": "u64", "data": "synthetic: numbers_mt regenerated per block",
           "config": {"workload": sql, "query": args.query, "rows": n,
                      "baseline_config": "BASELINE.json configs[0]" if (args.query, n) == ("c2", 100_000_000)
                      else None},
           "cpu_baseline": cb}
    if args.query in README_SECONDS:
        t, line = README_SECONDS[args.query]
        rate = 1e10 / t
        out["reference_published"] = {
            "source": "reference README.md:%d" % line, "seconds_at_1e10_rows": t, "rows_per_s": rate,
            "hardware": "8 vCPU KVM cloud instance, rustc 1.50.0-nightly (README.md:49-53)",
            "scaled_to_sample": {"rows": n, "seconds": n / rate,
                                 "note": "the README times 1e10 rows; its rate applied to this sample"},
            "port_over_reference": cb["value"] / rate}
    print(json.dumps(out), flush=True)


def dry_run(rank, world):
    """--dry-run: the launch and the rendezvous without the GPU -- every rank
    joins a gloo group and rank 0 prints which ranks arrived (the CPU test of
    the launcher)."""
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if world > 1:
        dist.init_process_group("gloo")
    mine = [rank, int(os.environ.get("LOCAL_RANK", "0")), os.getpid()]
    seen = [None] * world
    if world > 1:
        dist.all_gather_object(seen, mine)
    else:
        seen = [mine]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": seen}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle-s", type=float, default=3.0,
                    help="untimed steps for about this long before the warmup: HBM that earlier processes freed is "
                         "cleared by the driver in the background for a few seconds, and scans that overlap it run "
                         "3-4 %% slower (0 = none)")
    ap.add_argument("--query", default="c3", choices=sorted(list(QUERIES) + ["p1"]))
    ap.add_argument("--rows-per-gpu", type=float, default=1e10)
    ap.add_argument("--rows-total", type=float, default=None,
                    help="strong scaling: fix numbers_mt(N) at this N for every GPU count "
                         "(e.g. 1e10 = the 10B-row metric split over 1/2/4/8 GPUs)")
    ap.add_argument("--cpu-sample-rows", type=float, default=None,
                    help="rows of the CPU-baseline sample (default: the whole 1e10-row workload, ~1.5 s on the "
                         "box's 8 threads for c3, ~5 s for p1; 4e9 rows for GROUP BY, a hash insert per row, ~3-10 s)")
    ap.add_argument("--cpu-threads", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c-host", action="store_true",
                    help="skip the C-host leg (fq_c_client --bench in a child process, c3 at N=1)")
    ap.add_argument("--no-rccl-world1", action="store_true",
                    help="skip the world-1 RCCL exchange leg (fq_engine_execute_rccl, aggregates at N=1)")
    ap.add_argument("--project-path", default="engine", choices=("engine", "blocks", "contiguous"),
                    help="p1: through the engine (fq_engine_execute_blocks, default), or the kernel alone at the "
                         "C ABI: block-stream output (fq_filter_project_blocks) or one contiguous output per "
                         "partition (fq_filter_project)")
    ap.add_argument("--p1-outputs", default="contiguous", choices=("contiguous", "torch"),
                    help="p1 kernel paths: output columns in physically contiguous HBM (default) or torch buffers")
    ap.add_argument("--p1-output-sets", type=int, default=4,
                    help="p1 kernel paths: freshly allocated output pairs the launches cycle over")
    ap.add_argument("--p1-chunk-rows", type=float, default=None,
                    help="p1 engine path: rows per device block (FQ_OPT_CHUNK_ROWS; default 4e8)")
    ap.add_argument("--streams", type=int, default=1,
                    help="device queues the pipes share (FQ_OPT_STREAMS); 1 = the scans run back to back")
    ap.add_argument("--group-chunk-rows", type=int, default=None,
                    help="rows per radix-partitioned GROUP BY launch (FQ_OPT_GROUP_CHUNK_ROWS; tuning)")
    ap.add_argument("--comm-timeout-ms", type=int, default=60000,
                    help="deadline of every cross-GPU exchange step (FQ_COMM_TIMEOUT_MS): a rank that dies or never "
                         "arrives fails the others with FQ_E_RCCL instead of a wait without end")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl = RCCL over xGMI (default); gloo rehearses N ranks on fewer GPUs")
    ap.add_argument("--tune", action="append", default=[], metavar="KNOB=VALUE",
                    help="launch-shape knob through fq_tune_set (abi.TUNE names; sweeps only, the defaults "
                         "are the measured best)")
    ap.add_argument("--cpu-only", action="store_true",
                    help="no GPU: only the CPU baseline of --query at --rows-per-gpu rows, one JSON line "
                         "(C1 = --query c2 --rows-per-gpu 1e8, BASELINE.json configs[0])")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch and rendezvous only (gloo, no GPU): rank 0 prints the ranks that arrived")
    args = ap.parse_args()

    if args.cpu_only:
        return cpu_only_line(args)

    # --gpus N is the world size.  Without a launcher (no WORLD_SIZE) and N > 1,
    # start N ranks and relay their status; under a launcher the two must agree.
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            # The parent only spawns the ranks: it has loaded neither torch nor
            # the HIP library (HIP_MODULES), so no HIP state exists to cross a
            # fork; every rank checks its own device (check_rank_device).
            loaded = [m for m in HIP_MODULES if m in sys.modules]
            print("[bench] launcher parent: HIP-touching modules loaded before spawning: %s" % (loaded or "none"),
                  file=sys.stderr, flush=True)
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%s ranks"
                         % (args.gpus, os.environ["WORLD_SIZE"]))
    if args.dry_run:
        return dry_run(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    _load_runtime()
    args.tuned = {}
    for kv in args.tune:
        k, v = kv.split("=", 1)
        ops.tune_set(k.upper(), int(v))
        args.tuned[k.upper()] = int(v)
    local = check_rank_device(args, rank, world, local)
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    if args.query == "p1":
        if args.project_path == "engine":
            return run_project_engine(args, rank, world, local)
        return run_project(args, rank, world)
    if args.rows_total:
        n_total = int(args.rows_total)
        rows_per_gpu = n_total // world
    else:
        rows_per_gpu = int(args.rows_per_gpu)
        n_total = rows_per_gpu * world
    sql = QUERIES[args.query].format(N=n_total)

    # The engine: SQL -> Source x P -> [Filter] -> AggregatePartial x P -> Merge
    # -> AggregateFinal on this GPU (one host thread per pipe, fused scans).
    # FQ_OPT_PROFILE 2: one event span per query around its back-to-back scans
    # (no event between two scans); with several queues an event pair per scan
    eng = Engine(device=local, profile=PROFILE_SPAN if args.streams == 1 else True, streams=args.streams)
    if args.group_chunk_rows:
        eng.set_option(OPT_GROUP_CHUNK_ROWS, args.group_chunk_rows)
    mine = shard(generate_parts(n_total), rank, world)
    total_rows = sum(stream_rows(b, e) for _, b, e in mine)
    eng.materialize_numbers(n_total, rank, world)  # SourceTransform's column, resident in HBM
    torch.cuda.synchronize()
    log(rank, "materialised %d partitions, %d rows (%.1f GB) on rank %d"
        % (len(mine), total_rows, total_rows * 8 / 1e9, rank))

    # cross-GPU exchange: the library's own RCCL communicator (torch.distributed
    # only ships its unique id); the gloo rehearsal drives the same native
    # protocol through a torch callback
    comm = None
    if world > 1 and args.dist_backend == "nccl":
        ok = 1
        try:
            comm = stdout_to_stderr(fqd.RcclComm, local, None, args.comm_timeout_ms)
        except Exception as e:  # reported; the same protocol then runs over torch's RCCL group
            log(rank, "native RCCL communicator unavailable on rank %d: %r" % (rank, e))
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device="cuda")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if not int(flag.item()) and comm is not None:  # every rank takes the same transport
            comm.close()
            comm = None
    # the world the exchange really spans: the RCCL communicator's own count
    # (fq_comm_info), else the torch.distributed group's
    ranks_seen = comm.info()[1] if comm is not None else (dist.get_world_size() if world > 1 else 1)
    if ranks_seen != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the exchange spans %d ranks" % (args.gpus, ranks_seen))

    # One step on one GPU is what a host binding the C ABI does
    # (INTEGRATION.md): fq_engine_execute_row -- execute, the one result row's
    # values, the result freed, in one call; no Python Result object (its ~50 us
    # of interpreter work per step is harness, not query).
    import ctypes as C

    from fq_amd._lib import check as _check
    from fq_amd._lib import lib as _lib
    sql_b = sql.encode()
    row_buf = (abi.fq_value * 8)()
    ncols = C.c_int32(0)
    ncols_ref = C.byref(ncols)
    execute_row = _lib.fq_engine_execute_row
    eng_h = eng.h

    if world == 1:
        def c_row_call():
            # one call: execute, the row's values into row_buf, the result freed (fq_engine_execute_row)
            st = execute_row(eng_h, sql_b, row_buf, 8, ncols_ref)
            if st:
                _check(st)
    elif comm is not None:
        # one call at world > 1 too: partial -> RCCL exchange -> final -> the row
        # (fq_engine_execute_rccl_row), the exchange bounded by the communicator's deadline
        rccl_row, comm_h = _lib.fq_engine_execute_rccl_row, comm.h

        def c_row_call():
            st = rccl_row(eng_h, sql_b, comm_h, row_buf, 8, ncols_ref)
            if st:
                _check(st)
    else:
        # the gloo rehearsal: the same protocol through the torch callback
        ex_row, fn = _lib.fq_engine_execute_exchange_row, fqd.torch_allreduce_fn(None, args.comm_timeout_ms / 1e3)

        def c_row_call():
            st = ex_row(eng_h, sql_b, rank, world, fn, None, row_buf, 8, ncols_ref)
            if st:
                _check(st)

    def row_values():
        return [v.bits if v.is_some else None for v in row_buf[:ncols.value]]

    def c_row():
        c_row_call()
        return row_values()

    def c_groups():
        # GROUP BY result columns as numpy arrays (fq_result_values), rows in key order
        import numpy as np
        out = C.c_void_p()
        _check(_lib.fq_engine_execute(eng.h, sql_b, C.byref(out)))
        try:
            n = _lib.fq_result_num_rows(out)
            cols = []
            for c in range(_lib.fq_result_num_columns(out)):
                arr = (abi.fq_value * max(n, 1))()
                _check(_lib.fq_result_values(out, c, arr, n))
                cols.append(np.frombuffer(arr, dtype=[("dtype", "<i4"), ("is_some", "<i4"), ("bits", "<u8")])["bits"][:n])
            return cols
        finally:
            _lib.fq_result_free(out)

    def step():
        if args.query not in GROUP_MOD:
            return c_row()
        if world == 1:
            return c_groups()
        return fqd.execute(eng, sql, comm).rows

    def same_result(got, expect):
        if args.query in GROUP_MOD and world == 1:
            import numpy as np
            exp = np.array(expect, dtype=np.uint64).reshape(-1, len(got)) if expect else np.zeros((0, len(got)), np.uint64)
            return all(np.array_equal(g, exp[:, c]) for c, g in enumerate(got))
        return got == expect

    settled = settle(step, args.settle_s, world, args.dist_backend)
    for _ in range(max(args.warmup, 1)):
        res = step()
    expect = closed_form(args.query, n_total)
    if not same_result(res, expect):
        raise SystemExit("PARITY FAILURE: got %r expected %r" % (res, expect))
    ngroups = (len(res[0]) if world == 1 else len(res)) if args.query in GROUP_MOD else 0
    log(rank, "result", res if args.query not in GROUP_MOD else "%d groups" % ngroups, "== closed form")

    jit0 = ops.jit_stats()
    eng.reset_stats()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    # an ungrouped query: each timed step is ONE library call (world 1:
    # fq_engine_execute_row; world > 1: fq_engine_execute_rccl_row) that leaves
    # its row in row_buf; the Python list is built once, from the last step's row
    one_row = args.query not in GROUP_MOD
    timed = c_row_call if one_row else step
    for _ in range(args.steps):
        res = timed()
    if one_row:
        res = row_values()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    assert same_result(res, expect)

    st = eng.stats()
    jit1 = ops.jit_stats()
    jitted = jit1["jit_launches"] - jit0["jit_launches"]
    kernel = "fq_jit_groupby" if args.query in GROUP_MOD else ("fq_jit_scan" if jitted else "agg_flat_kernel")
    launches = max(st["scan_launches"], 1)
    avg_launch_ms = st["scan_ms"] / launches
    bytes_per_launch = st["scan_bytes"] / launches
    rows_per_launch = st["scan_rows"] / launches
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9  # algorithmic GB/s of the fused scan
    value = n_total * args.steps / dt
    # every rank's own scan fraction and exchange time: the line reports the
    # spread (the slowest rank sets the step)
    per_rank = None
    if world > 1:
        mine_stats = torch.tensor([achieved / HBM_PEAK_GBPS, st.get("exchange_ms", 0.0) / args.steps,
                                   st.get("partial_ms", 0.0) / args.steps],
                                  dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        gathered = [torch.zeros_like(mine_stats) for _ in range(world)]
        dist.all_gather(gathered, mine_stats)
        g = [t.cpu().tolist() for t in gathered]
        per_rank = {"scan_frac": {"min": min(x[0] for x in g), "max": max(x[0] for x in g)},
                    "exchange_ms_per_step": {"min": min(x[1] for x in g), "max": max(x[1] for x in g)},
                    "partial_ms_per_step": {"min": min(x[2] for x in g), "max": max(x[2] for x in g)},
                    "ranks": world}
    rccl_w1 = None
    if world == 1 and args.dist_backend == "nccl" and args.query not in GROUP_MOD and not args.no_rccl_world1:
        rccl_w1 = rccl_world1(eng, sql, expect, local, args)
    # The drop-in stack a C/Rust host binds (tests/native/fq_c_client.c: no
    # torch, /opt/rocm's HIP runtime) on the same workload, in a child process
    # AFTER this one's timed steps, while this one holds its memory and idles:
    # a process that starts right after another freed ~80 GB of HBM runs its
    # scans ~3-4 % slower while the driver reclaims that memory -- whichever
    # host it is (profiles/r05_b_host_spread/), so neither leg may follow a free.
    c_host = None
    if world == 1 and args.query == "c3" and not args.no_c_host:
        torch.cuda.synchronize()
        c_host = run_c_host(args)
    out = None
    if rank == 0:
        # the partitioned GROUP BY (g2): gpart + block scatter + bins per chunk
        traffic, traffic_src = latest_pmc_traffic(("fq_jit_gpart", "group_blk_", "fq_jit_groupby_bins")
                                                  if args.query == "g2" else kernel, args.query, rows_per_launch)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"s": args.settle_s, "steps": settled},
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.rows_total else "weak",
            "vs_baseline": value / README_ROWS_PER_S[args.query] if args.query in README_ROWS_PER_S else None,
            "vs_baseline_ref": README_REF.get(args.query, "no published reference number for this query"),
            "dtype": "u64",
            "data": "synthetic: system.numbers_mt iota column (u64), resident in HBM before timing",
            "config": {
                "workload": sql,
                "query": args.query,
                "rows_per_gpu": rows_per_gpu,
                "rows_total": n_total,
                "partitions_per_gpu": len(mine),
                "block_rows": BLOCK_SIZE,
                "path": "fq_engine_execute: SQL -> PipelineBuilder -> Source x P -> AggregatePartial x P "
                        "(fused gfx950 scan) -> Merge -> AggregateFinal"
                        + ("" if world == 1 else " ; cross-GPU: fq_engine_execute_rccl_row (one call per step), one "
                            "ncclAllReduce of partial states" if comm is not None else
                            " ; cross-GPU: fq_engine_execute_exchange_row over torch.distributed (%s)"
                            % args.dist_backend),
                "parallelism": "dp%d (numbers_mt partitions sharded, %s all-reduce of states)"
                               % (world, "RCCL" if args.dist_backend == "nccl" else "gloo rehearsal"),
            },
            "achieved_hbm_gbps": achieved,
            "kernel_ms_per_launch": avg_launch_ms,
            "scan_launches_per_step": st["scan_launches"] / args.steps,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": ("fq_group_aggregate (fq_jit_groupby, hipRTC-specialised), one launch per partition"
                           if args.query == "g1" else
                           "fq_group_aggregate_partitioned (fq_jit_gpart + block grouping + fq_jit_groupby_bins), "
                           "one set per partition; achieved = the column's 8 B/row over the set"
                           if args.query == "g2" else
                           "fq_aggregate fused scan (%s, then agg_finalize_kernel folds its workgroup partials), "
                           "one launch per partition%s; %s"
                           % (kernel, " (hipRTC-specialised for this expression shape)" if jitted else "",
                              "timed by one HIP-event span per query on the engine's queue (first scan start to "
                              "last scan end, launch gaps included) / launches" if args.streams == 1 else
                              "timed by an event pair per launch")),
                "bytes_per_launch": bytes_per_launch,
            },
            "result": res if args.query not in GROUP_MOD else (
                {"groups": ngroups, "first": [int(c[0]) for c in res], "last": [int(c[-1]) for c in res]}
                if world == 1 else {"groups": ngroups, "first": list(res[0]), "last": list(res[-1])}),
            "host_ms_per_step": host_split(st, args.steps, dt / args.steps * 1e3, world),
            # the whole step against its scans: what the step spends beyond them
            "step_over_scans": (dt / args.steps * 1e3) / (avg_launch_ms * st["scan_launches"] / args.steps)
            if st["scan_launches"] else None,
            "jit": {"specialised_launches": jitted, "kernels_compiled": jit1["kernels_compiled"],
                    "compile_ms": jit1["compile_ms"], "mode": jit1["mode"]},
        }
        if per_rank is not None:
            out["per_rank"] = per_rank
            out["roofline"]["frac_min_over_ranks"] = per_rank["scan_frac"]["min"]
    if world > 1:
        dist.barrier()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            sample = args.cpu_sample_rows or (4e9 if args.query in GROUP_MOD else 1e10)
            out["cpu_baseline"] = cpu_baseline(int(sample), args.cpu_threads, args.query)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        if c_host is not None:
            out["c_host"] = c_host
        if rccl_w1 is not None:
            out["rccl_world1"] = rccl_w1
        if args.tuned:
            out["tune"] = args.tuned
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
