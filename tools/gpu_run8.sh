cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_kernels.py > gpurun_out/kernels.json 2> gpurun_out/kernels.err; rc=$?; tail -24 gpurun_out/kernels.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/limit_probe.py > gpurun_out/limit.log 2>&1; rc=$?; tail -7 gpurun_out/limit.log; exit $rc
