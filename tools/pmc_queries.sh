#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (tools/pmc_pass.sh) for each bench query named
# on the command line (default: c2 c4s max max1 avg), each kept under
# gpurun_out/pmcq/<query>/ for tools/pmc_summary.py + tools/pmc_import.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
QS="$*"; [ -n "$QS" ] || QS="c2 c4s max max1 avg"
for Q in $QS; do
  bash tools/pmc_pass.sh --query $Q > gpurun_out/pmc_$Q.txt 2>&1 || exit 1
  rm -rf gpurun_out/pmcq/$Q && mkdir -p gpurun_out/pmcq/$Q && cp -r gpurun_out/pmc/* gpurun_out/pmcq/$Q/ && rm -rf gpurun_out/pmc
done
echo done
