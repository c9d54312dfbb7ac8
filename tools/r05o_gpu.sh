#!/bin/bash
# pipe 0 inline + slots read once: the engine / merge / distributed tests, then both hosts' C3 lines
out=gpurun_out/r05o; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests/test_engine_gpu.py tests/test_reference_suite_gpu.py tests/test_dist_gpu.py \
  tests/test_functions_gpu.py tests/test_c5_gpu.py tests/test_fuzz_gpu.py tests/test_engine_blocks_gpu.py -x -q \
  --timeout 240 --timeout-method thread > $out/pytest.txt 2>&1 || exit 1
sleep 5
timeout -k 10 200 fuse-query_amd/lib/fq_c_client --bench 20 10000000000 3 > $out/c_client_bench.json 2> $out/c_client.err || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-c-host --no-rccl-world1 > $out/bench_c3.json 2> $out/bench_c3.err || exit 1
timeout -k 10 200 fuse-query_amd/lib/fq_c_client --bench 20 10000000000 3 > $out/c_client_bench2.json 2> $out/c_client2.err || exit 1
echo done
