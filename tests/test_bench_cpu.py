"""CPU checks of bench.py's bookkeeping (no kernel runs): roofline.traffic
comes from the most recently measured committed PMC summary of the current
kernel sources, never from a stale one or an older one that merely sorts later
by name, and a stale one is reported as such with its file and commit; and
`--gpus N` is the world size -- without a launcher bench.py starts N ranks
itself, under one it refuses a different WORLD_SIZE."""
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _summary(path, sha, per_launch, rows=1000, commit="abc", when=None):
    json.dump({"measured_at_commit": commit, "query_sources_sha256": sha, "measured_at_unix": when,
               "kernels": [{"name": "agg_flat_kernel<...>", "hbm_bytes_per_launch": per_launch,
                            "rows_per_launch": rows}]}, open(path, "w"))


def test_traffic_prefers_current_sources_over_a_later_stale_file(tmp_path, monkeypatch):
    b = _bench()
    prof = tmp_path / "profiles"
    prof.mkdir()
    cur = b.kernel_sources_sha256("c3")
    _summary(prof / "r09_final_pmc_c3.json", cur, 8000.0, commit="good")
    _summary(prof / "r09_pmc_c3.json", "0" * 64, 9999.0, commit="old")  # sorts after the current one
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    t, src = b.latest_pmc_traffic("agg_flat", "c3", 2000)
    assert t == 16000.0  # 8000 B per 1000 rows, scaled to 2000 rows
    assert src["file"] == "profiles/r09_final_pmc_c3.json" and src["status"] == "current kernel sources"
    assert src["measured_at_commit"] == "good"


def test_traffic_reports_a_stale_file_when_none_is_current(tmp_path, monkeypatch):
    b = _bench()
    prof = tmp_path / "profiles"
    prof.mkdir()
    _summary(prof / "r09_pmc_c3.json", "0" * 64, 9999.0, commit="old")
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    t, src = b.latest_pmc_traffic("agg_flat", "c3", 2000)
    assert t is None
    assert src["file"] == "profiles/r09_pmc_c3.json" and src["status"].startswith("stale")
    monkeypatch.setattr(b, "ROOT", str(tmp_path / "nowhere"))
    t, src = b.latest_pmc_traffic("agg_flat", "c3", 2000)
    assert t is None and src["status"].startswith("no PMC summary")



def test_traffic_takes_the_newest_measurement_not_the_last_name(tmp_path, monkeypatch):
    # r03_s4_head_* sorts after r03_s4_final_* by name but was measured first
    b = _bench()
    prof = tmp_path / "profiles"
    prof.mkdir()
    cur = b.kernel_sources_sha256("c3")
    _summary(prof / "r03_s4_final_pmc_c3.json", cur, 8000.0, commit="later", when=2000.0)
    _summary(prof / "r03_s4_head_pmc_c3.json", cur, 8100.0, commit="earlier", when=1000.0)
    _summary(prof / "r03_s4_zzz_pmc_c3.json", cur, 9000.0, commit="unstamped")  # no stamp: oldest
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    t, src = b.latest_pmc_traffic("agg_flat", "c3", 1000)
    assert t == 8000.0 and src["file"] == "profiles/r03_s4_final_pmc_c3.json"
    assert src["measured_at_commit"] == "later" and src["measured_at_unix"] == 2000.0


def test_committed_summaries_carry_a_measurement_time():
    # every committed summary bench.py may pick from has its measurement order
    import glob
    for f in glob.glob(os.path.join(ROOT, "profiles", "r0[3-9]*pmc_*.json")):
        d = json.load(open(f))
        if d.get("measured_at_commit"):
            assert d.get("measured_at_unix"), f


def _run_bench(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_gpus_n_without_a_launcher_starts_n_ranks():
    # no WORLD_SIZE: bench.py runs torch.distributed.run itself; every rank
    # joins the (gloo) rendezvous and rank 0 reports who arrived
    p = _run_bench(["--gpus", "3", "--dry-run"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["dry_run"] and out["n_gpus"] == 3
    assert sorted(r[0] for r in out["ranks"]) == [0, 1, 2]
    assert len({r[2] for r in out["ranks"]}) == 3  # three processes
    assert "launching 3 ranks" in p.stderr


def test_gpus_and_launcher_world_mismatch_exits_nonzero():
    p = _run_bench(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert p.returncode != 0
    assert "--gpus 2 but the launcher started WORLD_SIZE=3" in p.stderr
    p = _run_bench(["--gpus", "1", "--dry-run"], {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=8" in p.stderr


def test_gpus_n_with_rccl_needs_n_visible_gpus():
    # no GPU here: the parent starts the ranks without touching HIP, and every
    # rank checks its own device and exits non-zero
    p = _run_bench(["--gpus", "2", "--no-cpu-baseline"], timeout=240)
    assert p.returncode != 0
    assert "launching 2 ranks" in p.stderr
    assert "no GPU" in p.stderr or "needs a GPU per rank" in p.stderr, p.stderr[-3000:]


def test_launcher_parent_loads_no_hip_module():
    # `bench.py --gpus N` without a launcher only spawns processes: neither
    # torch nor the HIP library is imported in the parent before it does
    p = _run_bench(["--gpus", "2", "--dry-run"], timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "launcher parent: HIP-touching modules loaded before spawning: none" in p.stderr


def test_bench_module_imports_without_the_hip_runtime():
    # importing bench.py (what the tests above do) loads no HIP-touching module
    code = ("import importlib.util, sys; spec = importlib.util.spec_from_file_location('b', %r); "
            "m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m); "
            "print(sorted(x for x in m.HIP_MODULES if x in sys.modules))" % os.path.join(ROOT, "bench.py"))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 0, p.stderr
    assert p.stdout.strip() == "[]"


def test_settle_runs_untimed_steps_for_about_the_requested_time():
    # bench.settle: steps for ~`seconds` at the SECOND step's pace (world 1: no
    # collective); 0 s runs none, a step slower than the budget runs twice, and
    # a slow first step (hipRTC compile, first mapping) does not cut the settle
    import time
    b = _bench()
    calls = []

    def step():
        calls.append(time.perf_counter())
        time.sleep(0.002)

    assert b.settle(step, 0, 1, "gloo") == 0 and not calls
    n = b.settle(step, 0.05, 1, "gloo")
    assert n == len(calls) and 10 <= n <= 30, n
    calls.clear()
    assert b.settle(lambda: (calls.append(1), time.sleep(0.03)), 0.01, 1, "gloo") == 2 and len(calls) == 2
    calls.clear()

    def slow_first():
        time.sleep(0.05 if not calls else 0.002)
        calls.append(time.perf_counter())

    t0 = time.perf_counter()
    n = b.settle(slow_first, 0.2, 1, "gloo")
    assert n == len(calls) and time.perf_counter() - t0 >= 0.15, (n, time.perf_counter() - t0)


def test_kernel_gaps_busy_time_is_the_union_of_launch_intervals(tmp_path):
    # tools/kernel_gaps.py --window: the rocprof figure held beside bench.py's
    # span when launches on the two row queues overlap -- the time at least one
    # launch ran (never their sum), over the COUNT launches ending SKIP_LAST
    # before the last
    import csv
    import json
    import subprocess
    import sys
    path = tmp_path / "trace.csv"
    rows = [(0, 100, "fq_jit_pblocks"), (50, 150, "fq_jit_pblocks"),  # overlap: busy 150
            (150, 160, "other"), (200, 300, "fq_jit_pblocks"),          # gap 50, busy +100
            (1000, 1100, "fq_jit_pblocks")]                            # the checked step, skipped
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for s, e, n in rows:
            w.writerow([n, s, e])
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "kernel_gaps.py"), str(path), "pblocks",
                          "--window", "3", "1"], capture_output=True, text=True, check=True).stdout
    d = json.loads(out)
    assert d["launches"] == 3
    assert abs(d["busy_union_ms"] - 250e-6) < 1e-12, d   # ns -> ms: 250 ns
    assert abs(d["span_ms"] - 300e-6) < 1e-12, d
    assert abs(d["kernel_ms_mean"] - 100e-6) < 1e-12, d
