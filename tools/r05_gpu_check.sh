#!/bin/bash
# Round-5 GPU pass: the in-launch finalize + grouped scan waits first (their
# kernel and engine tests), then the C3 bench line (C-host and world-1 RCCL
# legs included), its rocprofv3 kernel stats, and the whole GPU suite.
# usage: tools/r05_gpu_check.sh OUTDIR [full]
R=$(pwd)
out=${1:-gpurun_out/r05}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py -x -q -k "one_launch or identity or specialised or block_mode" \
  --timeout 120 --timeout-method thread > "$out/pytest_kernels.txt" 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests/test_engine_gpu.py tests/test_c_client_gpu.py tests/test_functions_gpu.py \
  tests/test_engine_blocks_gpu.py tests/test_memory_gpu.py -x -q --timeout 240 --timeout-method thread \
  > "$out/pytest_engine.txt" 2>&1 || exit 1
cp -f gpurun_out/c_client_handles_c3.json gpurun_out/c_client_bench_c3.json "$out/" 2>/dev/null
timeout -k 10 300 python3 bench.py > "$out/bench_c3.json" 2> "$out/bench_c3.err" || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof_c3" -o run -- \
  python3 "$R/bench.py" --steps 10 --no-cpu-baseline --no-c-host --no-rccl-world1 > "$R/$out/c3_under_rocprof.json" \
  2> "$R/$out/prof_c3.err") || exit 1
if [ "$2" = "full" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$out/pytest_gpu.txt" 2>&1 || exit 1
fi
echo done
