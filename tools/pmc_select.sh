#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; one counter set per run) over
# tools/select_probe.py.  KEEP / FQ_SELECT_* pass through.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); OUT="$R/gpurun_out/pmc_select${TAG}"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/$C" -o pmc -- python3 "$R/tools/select_probe.py" > "$OUT/$C.txt" 2> "$OUT/$C.err"
  rc=$?; echo "$C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 "$R/tools/pmc_summary.py" "$OUT/summary.json" 1250000000 $(find "$OUT" -name "*counter_collection*.csv")
