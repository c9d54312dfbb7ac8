#!/bin/bash
# round 3: GROUP BY suites after the merge home-slot / kept-workspace / gpart fixes, then a g2 bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_groupby_gpu.py tests/test_memory_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --durations=15 > gpurun_out/r03b_pytest.log 2>&1
rc=$?; tail -25 gpurun_out/r03b_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --query g2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03b_g2.json 2> gpurun_out/r03b_g2.err
rc=$?; tail -3 gpurun_out/r03b_g2.err; cat gpurun_out/r03b_g2.json; exit $rc
