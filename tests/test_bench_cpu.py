"""CPU checks of bench.py's bookkeeping (no kernel runs): roofline.traffic
comes from the last committed PMC summary measured on the current kernel
sources, never from a stale one that merely sorts later by name, and a stale
one is reported as such with its file and commit."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _summary(path, sha, per_launch, rows=1000, commit="abc"):
    json.dump({"measured_at_commit": commit, "query_sources_sha256": sha,
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

