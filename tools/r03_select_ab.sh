#!/bin/bash
# select kernel: parity under the ring variant, then the 10 GB probe over variants / tile shapes
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
FQ_TUNE_SELECT_VARIANT=3 FQ_TUNE_SELECT_ROWS=32 timeout -k 10 300 python -u -m pytest tests/test_project_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sel_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/sel_pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/sel_probe.txt
for cfg in ${CFGS:-1:256:32 3:256:32 3:256:16 2:256:16}; do
IFS=: read v th rows <<< "$cfg"
  echo -n "variant=$v threads=$th rows=$rows " >> gpurun_out/sel_probe.txt
  FQ_TUNE_SELECT_VARIANT=$v FQ_TUNE_SELECT_THREADS=$th FQ_TUNE_SELECT_ROWS=$rows KEEP=0.375 NOUT=2 timeout -k 10 120 python tools/select_probe.py >> gpurun_out/sel_probe.txt 2>>gpurun_out/sel_probe.err || exit $?
done
cat gpurun_out/sel_probe.txt
