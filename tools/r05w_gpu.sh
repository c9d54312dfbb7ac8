#!/bin/bash
# p1 launches without memset / copy: parity, the p1 line, the kernel trace's gaps
R=$(pwd); out=gpurun_out/r05w; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_project_blocks_gpu.py tests/test_engine_blocks_gpu.py -x -q \
  --timeout 300 --timeout-method thread > $out/pytest.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --query p1 > $out/bench_p1.json 2> $out/bench_p1.err || exit 1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof_p1" -o run -- python3 "$R/bench.py" --query p1 --steps 10 --no-cpu-baseline > "$R/$out/p1_under_rocprof.json" 2> "$R/$out/prof_p1.err") || exit 1
echo done
