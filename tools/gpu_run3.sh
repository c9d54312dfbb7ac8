cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u tools/limit_probe.py > gpurun_out/limit.log 2>&1; rc=$?; cat gpurun_out/limit.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_limit" -o run -- python3 "$R/tools/limit_probe.py" > "$R/gpurun_out/prof_limit.log" 2>&1; rc=$?; echo prof rc=$rc; exit $rc
