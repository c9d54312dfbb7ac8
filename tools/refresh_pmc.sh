#!/bin/bash
# Parity tests of the select kernels, then PMC + rocprof stats + bench line for
# the given queries (default p1 g2).  Outputs under gpurun_out/refresh/.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); O="$R/gpurun_out/refresh"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_project_blocks_gpu.py tests/test_project_gpu.py > "$O/pytest_select.txt" 2>&1 || exit 1
export TMPDIR=/tmp
for Q in ${@:-p1 g2}; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$Q" -o $Q -- python3 "$R/bench.py" --query $Q --steps 5 --warmup 1 --no-cpu-baseline --no-c-host --no-rccl-world1 > "$O/prof_bench_$Q.json" 2> "$O/prof_bench_$Q.err") || exit 1
  bash tools/pmc_pass.sh --query $Q > "$O/pmc_$Q.txt" 2>&1 || exit 1
  mkdir -p "$O/pmc_$Q" && cp -r gpurun_out/pmc/* "$O/pmc_$Q/" && rm -rf gpurun_out/pmc
  timeout -k 10 300 python bench.py --query $Q > "$O/bench_$Q.json" 2> "$O/bench_$Q.err" || exit 1
done
echo done > "$O/done"
