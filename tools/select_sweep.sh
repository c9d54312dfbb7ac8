#!/bin/bash
# fq_filter_project tile-shape / variant sweep on a 10 GB column
# (tools/select_probe.py; FQ_SELECT_VARIANT bit 0 per-XCD tickets, bit 1
# two tiles per workgroup; FQ_SELECT_LBW look-back words per lane).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/select_sweep.txt
: > $OUT
for sl in ${SLEEPS:-2}; do
for lbw in ${LBWS:-4}; do
for v in ${VARIANTS:-0 1 2 3}; do
 for th in ${THREADS:-256}; do
 for rows in ${ROWS:-16 32}; do
  for wg in ${WGS:-8}; do
    for keep in ${KEEPS:-0.375 0}; do
      echo -n "sleep=$sl variant=$v lbw=$lbw threads=$th rows=$rows " >> $OUT
      FQ_TUNE_SELECT_SLEEP=$sl FQ_TUNE_SELECT_LBW=$lbw FQ_TUNE_SELECT_VARIANT=$v FQ_TUNE_SELECT_THREADS=$th FQ_TUNE_SELECT_ROWS=$rows FQ_TUNE_SELECT_WG_PER_CU=$wg KEEP=$keep timeout -k 10 120 python tools/select_probe.py >> $OUT 2>>gpurun_out/select_sweep.err || exit $?
    done
  done
 done
 done
done
done
done
cat $OUT
