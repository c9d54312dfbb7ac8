#!/bin/bash
# the C3 query traced again after the single-waiter end (tools/window_timeline.py), then the bench line
R=$(pwd); out=gpurun_out/r05d; mkdir -p $out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$R/$out/trace" -o run -- \
  python3 "$R/tools/readme_window.py" c3 2 > "$R/$out/window.txt" 2> "$R/$out/trace.err") || exit 1
K=$(find $out/trace -name "*kernel_trace.csv" | head -1); A=$(find $out/trace -name "*hip_api_trace.csv" | head -1)
python3 tools/window_timeline.py $out/window.txt "$K" "$A" > $out/c3_query_timeline.txt || exit 1
rm -rf $out/trace
sleep 15
timeout -k 10 300 python3 bench.py > $out/bench_c3.json 2> $out/bench_c3.err || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_engine_gpu.py tests/test_reference_suite_gpu.py tests/test_dist_gpu.py -x -q \
  --timeout 240 --timeout-method thread > $out/pytest_engine.txt 2>&1 || exit 1
echo done
