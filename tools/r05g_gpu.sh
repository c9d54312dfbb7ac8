#!/bin/bash
# stage-capacity variants of fq_jit_pblocks: parity three ways, the in-process A/B, rocprof of the default p1 line
R=$(pwd); out=gpurun_out/r05g; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_project_blocks_gpu.py -x -q --timeout 240 --timeout-method thread > $out/pytest_blocks.txt 2>&1 || exit 1
timeout -k 10 400 python3 tools/p1_stage_ab.py 4 8 > $out/p1_stage_ab.json 2> $out/p1_stage_ab.err || exit 1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$out/prof_p1" -o p1 -- python3 "$R/bench.py" --query p1 --steps 5 --warmup 1 --no-cpu-baseline > "$R/$out/prof_bench_p1.json" 2> "$R/$out/prof_bench_p1.err") || exit 1
echo done
