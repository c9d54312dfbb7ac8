#!/bin/bash
# p1 through the engine: the memset-free launch vs the async path, in one process; parity first
out=gpurun_out/r05x; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests/test_project_blocks_gpu.py tests/test_engine_blocks_gpu.py tests/test_engine_gpu.py \
  tests/test_reference_suite_gpu.py -x -q --timeout 300 --timeout-method thread > $out/pytest.txt 2>&1 || exit 1
timeout -k 10 500 python3 tools/p1_stage_ab.py 4 8 ENGINE_PROJECT_LAUNCH=1 ENGINE_PROJECT_LAUNCH=0 > $out/p1_launch_ab.json 2> $out/p1_launch_ab.err || exit 1
timeout -k 10 300 python3 bench.py --query p1 > $out/bench_p1.json 2> $out/bench_p1.err || exit 1
echo done
