"""pytest setup: import paths for the product package (fuse-query_amd/fq_amd)
and the test-only oracle (oracle/), plus the `gpu` marker."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "fuse-query_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


def pytest_sessionstart(session):
    # sweeps re-run the GPU suites under a launch-shape knob (FQ_TUNE_<KNOB>=v,
    # tools/knobs.py); the library itself reads no environment for them
    if any(k.startswith("FQ_TUNE_") for k in os.environ):
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import knobs
        knobs.apply_env()
