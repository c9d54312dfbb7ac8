#!/bin/bash
# group-by suites, then g2 kernel stats with narrow partition rows on and off
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_groupby_gpu.py tests/test_fuzz_groupby_gpu.py > gpurun_out/g2rot_pytest.txt 2>&1 || { tail -30 gpurun_out/g2rot_pytest.txt; exit 1; }
tail -2 gpurun_out/g2rot_pytest.txt
bash tools/r03_g2_quick.sh
