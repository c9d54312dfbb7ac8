#!/bin/bash
# fold queue (fq_aggregate_split) + the half-tile p1 stage: parity subset, the finalize A/B, bench lines, rocprof
R=$(pwd); out=gpurun_out/r05h; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_reference_suite_gpu.py \
  tests/test_dist_gpu.py tests/test_functions_gpu.py tests/test_project_blocks_gpu.py tests/test_engine_blocks_gpu.py \
  tests/test_c5_gpu.py -x -q --timeout 240 --timeout-method thread > $out/pytest.txt 2>&1 || exit 1
timeout -k 10 400 python3 tools/scan_fin_ab.py 6 > $out/scan_fin_ab.json 2> $out/scan_fin_ab.err || exit 1
sleep 10
timeout -k 10 300 python3 bench.py > $out/bench_c3.json 2> $out/bench_c3.err || exit 1
timeout -k 10 300 python3 bench.py --query p1 > $out/bench_p1.json 2> $out/bench_p1.err || exit 1
export TMPDIR=/tmp
for Q in c3 p1; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof_$Q" -o $Q -- python3 "$R/bench.py" --query $Q --steps 5 --warmup 1 --no-cpu-baseline --no-c-host --no-rccl-world1 > "$R/$out/prof_bench_$Q.json" 2> "$R/$out/prof_bench_$Q.err") || exit 1
done
echo done
