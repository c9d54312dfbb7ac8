#!/bin/bash
# round 6: the GPU suite on the current tree (+ RCCL deadline at world 2 with an absent rank), p1 + C3 lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "never_arrives" > gpurun_out/r06e_pytest_rccl_deadline.txt 2>&1
rc=$?; tail -3 gpurun_out/r06e_pytest_rccl_deadline.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06e_pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/r06e_pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
sleep 20
timeout -k 10 200 python -u bench.py --query p1 > gpurun_out/r06e_bench_p1.json 2> gpurun_out/r06e_bench_p1.err || exit $?
echo done
