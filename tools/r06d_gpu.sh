#!/bin/bash
# round 6: span-timed block projections + light polling -- parity subset, A/B, kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_blocks_gpu.py tests/test_engine_gpu.py tests/test_memory_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06d_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06d_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/p1_stage_ab.py 4 8 ENGINE_PROJECT_LAUNCH=0 ENGINE_PROJECT_LAUNCH=1 ENGINE_PROJECT_LAUNCH=2 > gpurun_out/r06d_p1_queue_ab.json 2> gpurun_out/r06d_p1_queue_ab.err || exit $?
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06d_p1trace -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/p1_stage_ab.py 1 4 ENGINE_PROJECT_LAUNCH=1 ENGINE_PROJECT_LAUNCH=2 > $GRAFT_REPO_ROOT/gpurun_out/r06d_p1trace.json 2> $GRAFT_REPO_ROOT/gpurun_out/r06d_p1trace.err || exit $?
echo done
