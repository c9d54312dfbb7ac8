#!/bin/bash
# HEAD check on one GPU box (gpurun): GPU suite, smoke, then per query (default
# c3 p1 g2) a bench line under rocprofv3 --kernel-trace --stats, the PMC
# traffic passes and the bench line with its CPU baseline.  Stops at the first
# failing step.  Outputs under gpurun_out/head/.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); O="$R/gpurun_out/head"; mkdir -p "$O"
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=15 > "$O/pytest_gpu.txt" 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 || exit 1
export TMPDIR=/tmp
for Q in ${@:-c3 p1 g2}; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$Q" -o $Q -- python3 "$R/bench.py" --query $Q --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof_bench_$Q.json" 2> "$O/prof_bench_$Q.err") || exit 1
  bash tools/pmc_pass.sh --query $Q > "$O/pmc_$Q.txt" 2>&1 || exit 1
  mkdir -p "$O/pmc_$Q" && cp -r gpurun_out/pmc/* "$O/pmc_$Q/" && rm -rf gpurun_out/pmc
  timeout -k 10 300 python bench.py --query $Q > "$O/bench_$Q.json" 2> "$O/bench_$Q.err" || exit 1
done
echo done > "$O/done"
