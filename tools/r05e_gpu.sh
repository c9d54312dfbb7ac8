#!/bin/bash
# p1 store variants (tests both ways, then the in-process A/B) and the C3 step's host tail split
out=gpurun_out/r05e; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_project_blocks_gpu.py tests/test_engine_blocks_gpu.py -x -q \
  --timeout 240 --timeout-method thread > $out/pytest_blocks.txt 2>&1 || exit 1
timeout -k 10 400 python3 tools/p1_stage_ab.py 4 8 > $out/p1_stage_ab.json 2> $out/p1_stage_ab.err || exit 1
timeout -k 10 200 fuse-query_amd/lib/fq_c_client --bench 20 10000000000 3 > $out/c_client_bench.json 2> $out/c_client.err || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-c-host --no-rccl-world1 > $out/bench_c3.json 2> $out/bench_c3.err || exit 1
echo done
