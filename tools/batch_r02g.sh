#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE separately) for the c3 and g1 bench kernels
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd)
for q in c3 g1; do
  bash tools/pmc_pass.sh --query $q || exit $?
  python3 tools/pmc_summary.py gpurun_out/pmc_$q.json 1250000000 $(find gpurun_out/pmc -name "*counter_collection*.csv") || exit $?
  rm -rf gpurun_out/pmc
done
