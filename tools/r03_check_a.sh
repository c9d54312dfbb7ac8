#!/bin/bash
# round 3: Function-ABI GPU tests + select/golden suites after the knob move, then c3 PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_functions_gpu.py tests/test_golden_gpu.py tests/test_project_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03a_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r03a_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_pass.sh --query c3 && python3 tools/pmc_summary.py gpurun_out/pmc_c3.json 1250000000 $(find gpurun_out/pmc -name "*counter_collection*.csv")
