#!/bin/bash
# deferred AggregatePartial states + staged p1 kernel: the whole GPU suite, then the c3 and p1 lines
out=gpurun_out/r05f; mkdir -p $out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $out/bench_c3.json 2> $out/bench_c3.err || exit 1
timeout -k 10 300 python3 bench.py --query p1 > $out/bench_p1.json 2> $out/bench_p1.err || exit 1
echo done
