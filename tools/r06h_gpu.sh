#!/bin/bash
# round 6: row pipelines on two row queues -- engine/projection GPU tests, the p1 line, its kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_engine_blocks_gpu.py tests/test_engine_gpu.py tests/test_memory_gpu.py tests/test_project_gpu.py tests/test_project_blocks_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06h_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06h_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --query p1 > gpurun_out/r06h_bench_p1.json 2> gpurun_out/r06h_bench_p1.err || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06h_p1prof -o p1 -- python3 $R/bench.py --query p1 --steps 10 --no-cpu-baseline > $R/gpurun_out/r06h_p1prof.json 2> $R/gpurun_out/r06h_p1prof.err) || exit $?
echo done
