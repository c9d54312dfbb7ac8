#!/bin/bash
# the select kernel on one ticket counter: its tests both ways, the memory / LIMIT engine tests, LIMIT latency, the contiguous p1 path
out=gpurun_out/r05r; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_project_gpu.py tests/test_memory_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 240 --timeout-method thread > $out/pytest.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/limit_probe.py > $out/limit_probe.json 2> $out/limit_probe.err || exit 1
timeout -k 10 300 python3 bench.py --query p1 --project-path contiguous --no-cpu-baseline > $out/bench_p1_contiguous_v0.json 2> $out/p1c0.err || exit 1
timeout -k 10 300 python3 bench.py --query p1 --project-path contiguous --no-cpu-baseline --tune SELECT_VARIANT=1 > $out/bench_p1_contiguous_v1.json 2> $out/p1c1.err || exit 1
echo done
