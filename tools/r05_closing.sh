#!/bin/bash
# closing evidence on the final sources: bench lines + rocprof stats (r05_fin_benches.sh), then the driver's
# order -- the GPU suite, smoke, and the default bench line right after them
out=${1:-gpurun_out/fin2}; mkdir -p "$out"
bash tools/r05_fin_benches.sh "$out" || exit 1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest_gpu.txt" 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > "$out/bench_c3_after_suite.json" 2> "$out/bench_c3_after_suite.err" || exit 1
echo done
