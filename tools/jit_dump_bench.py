"""Run bench.py with the hipRTC sources and code objects dumped to a
directory (fq_tune_jit_dump_dir), for disassembly.
usage: jit_dump_bench.py DIR [bench args]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))
from fq_amd._lib import check, lib  # noqa: E402

d = os.path.abspath(sys.argv[1])
os.makedirs(d, exist_ok=True)
check(lib.fq_tune_jit_dump_dir(d.encode()))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
