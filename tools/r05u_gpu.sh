#!/bin/bash
# execute_row + lazy fold queues: engine / C-host tests, the c3 and p1 lines, LIMIT latency
out=gpurun_out/r05u; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests/test_engine_gpu.py tests/test_c_client_gpu.py tests/test_engine_blocks_gpu.py -x -q \
  --timeout 300 --timeout-method thread > $out/pytest.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $out/bench_c3.json 2> $out/bench_c3.err || exit 1
timeout -k 10 300 python3 bench.py --query p1 > $out/bench_p1.json 2> $out/bench_p1.err || exit 1
timeout -k 10 200 python3 tools/limit_probe.py > $out/limit_probe.txt 2> $out/limit_probe.err || exit 1
echo done
