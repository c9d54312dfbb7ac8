cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_project_gpu.py tests/test_tree_gpu.py -x -q --timeout 60 --timeout-method thread > gpurun_out/proj.log 2>&1; rc=$?; tail -30 gpurun_out/proj.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_kernels.py > gpurun_out/kernels.json 2> gpurun_out/kernels.err; rc=$?; grep -i "filter_project\|predicate_bitmap" gpurun_out/kernels.err; exit $rc
