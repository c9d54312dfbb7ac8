cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tree_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tree.log 2>&1; rc=$?; tail -30 gpurun_out/tree.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/limit_probe.py > gpurun_out/limit.log 2>&1; rc=$?; cat gpurun_out/limit.log; exit $rc
