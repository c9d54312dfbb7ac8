#!/bin/bash
# Closing run, part 1 (one per round, on the final kernel sources): rocprofv3
# kernel stats of the headline bench commands, then the FETCH_SIZE / WRITE_SIZE
# passes (tools/pmc_pass.sh) of every bench query.  Summarise + import here
# with tools/pmc_summary.py / tools/pmc_import.py before part 2
# (tools/closing_bench.sh), whose bench lines then carry current traffic.
# usage: tools/closing_pmc.sh OUTDIR [QUERIES...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); O="$R/${1:-gpurun_out/close}"; shift
QS="$*"; [ -n "$QS" ] || QS="c3 p1 c4 g1 g2"
mkdir -p "$O"
export TMPDIR=/tmp
for Q in c3 p1; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$Q" -o $Q -- python3 "$R/bench.py" --query $Q --steps 10 --no-cpu-baseline --no-c-host --no-rccl-world1 > "$O/prof_bench_$Q.json" 2> "$O/prof_bench_$Q.err") || exit 1
  echo "prof $Q ok"
done
for Q in $QS; do
  bash tools/pmc_pass.sh --query $Q > "$O/pmc_$Q.txt" 2>&1 || exit 1
  rm -rf "$O/pmc_$Q" && mkdir -p "$O/pmc_$Q" && cp -r gpurun_out/pmc/* "$O/pmc_$Q/" && rm -rf gpurun_out/pmc || exit 1
  echo "pmc $Q ok"
done
echo done
