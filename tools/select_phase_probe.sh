#!/bin/bash
# fq_jit_pselect per-phase cycles (FQ_TUNE_SELECT_DEBUG=1, tuning only) for a few
# selectivities / output counts: does the store phase scale with the stores?
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/select_phase_probe.txt
: > $OUT
for cfg in "0.375 1" "0.375 2" "0 2" "1.0 1" "0.1 2"; do
  set -- $cfg
  echo "== keep=$1 nout=$2" >> $OUT
  FQ_TUNE_SELECT_DEBUG=1 KEEP=$1 NOUT=$2 timeout -k 10 120 python tools/select_probe.py 2>&1 | grep -v amdgpu.ids | sed -n '1,4p;$p' >> $OUT || exit $?
done
