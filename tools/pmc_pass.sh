#!/bin/bash
# PMC passes for the bench kernel (separate passes, kernel-trace free; see
# MI355X_MICROARCH.md rocprofv3 PMC slots).  Usage: tools/pmc_pass.sh [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); OUT="$R/gpurun_out/pmc"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/$C" -o pmc -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-c-host --no-rccl-world1 --settle-s 0 "$@" > "$OUT/$C.json" 2> "$OUT/$C.err"
  rc=$?; echo "$C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
find "$OUT" -name "*counter_collection*.csv"
