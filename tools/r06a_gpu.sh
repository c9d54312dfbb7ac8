#!/bin/bash
# round 6, first GPU call: the GPU suite on the pruned ABI, then the p1 queue-form A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06a_pytest_gpu.txt 2>&1
rc=$?
tail -5 gpurun_out/r06a_pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u tools/p1_stage_ab.py 4 8 ENGINE_PROJECT_LAUNCH=0 ENGINE_PROJECT_LAUNCH=1 ENGINE_PROJECT_LAUNCH=2 \
    > gpurun_out/r06a_p1_queue_ab.json 2> gpurun_out/r06a_p1_queue_ab.err || exit $?
P1_PROFILE=0 timeout -k 10 150 python -u tools/p1_stage_ab.py 4 8 ENGINE_PROJECT_LAUNCH=0 ENGINE_PROJECT_LAUNCH=1 ENGINE_PROJECT_LAUNCH=2 \
    > gpurun_out/r06a_p1_queue_ab_noprof.json 2> gpurun_out/r06a_p1_queue_ab_noprof.err || exit $?
timeout -k 10 150 python -u bench.py > gpurun_out/r06a_bench_c3.json 2> gpurun_out/r06a_bench_c3.err || exit $?
echo done
