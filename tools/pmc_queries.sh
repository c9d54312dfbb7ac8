#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
for Q in c2 c4s max max1 avg; do
  bash tools/pmc_pass.sh --query $Q > gpurun_out/pmc_$Q.txt 2>&1 || exit 1
  mkdir -p gpurun_out/pmcq/$Q && cp -r gpurun_out/pmc/* gpurun_out/pmcq/$Q/ && rm -rf gpurun_out/pmc
done
echo done
