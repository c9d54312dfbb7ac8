#!/bin/bash
# GROUP BY launch shape sweep (threads, LDS budget, workgroups per CU, row map)
# over one 10 GB numbers_mt partition; tools/groupby_sweep.py per variant
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/gsweep; mkdir -p $OUT
for v in "1024 128 1 1" "1024 128 1 0" "1024 64 2 1" "512 64 2 1" "512 32 4 1" "256 32 4 1" "256 16 8 1" "1024 32 2 1"; do
  set -- $v
  echo "== threads=$1 lds_kb=$2 wg_per_cu=$3 rowmap=$4"
  FQ_TUNE_GROUP_THREADS=$1 FQ_TUNE_GROUP_LDS_KB=$2 FQ_TUNE_GROUP_WG_PER_CU=$3 FQ_TUNE_GROUP_ROWMAP=$4 timeout -k 10 200 python tools/groupby_sweep.py 1.25e9 8,64,1000 1,3 || exit $?
done 2>&1 | grep -v amdgpu.ids | tee $OUT/sweep.txt
