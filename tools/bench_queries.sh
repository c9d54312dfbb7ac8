#!/bin/bash
# Bench every query on one GPU and a kernel-trace profile of each.
# Usage: [CPU=1] tools/bench_queries.sh [queries...]  (CPU=1 keeps the cpu_baseline leg)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); OUT="$R/gpurun_out/q"; mkdir -p "$OUT"
export TMPDIR=/tmp
QS=${*:-c2 c3 c4}
for q in $QS; do
  CPUARG=--no-cpu-baseline; [ -n "$CPU" ] && CPUARG=
  timeout -k 10 300 python bench.py --query $q --steps 10 --warmup 2 $CPUARG > "$OUT/$q.json" 2> "$OUT/$q.err"
  rc=$?; echo "$q bench rc=$rc"; cat "$OUT/$q.json"; [ $rc -eq 0 ] || exit $rc
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$q" -o run -- python3 "$R/bench.py" --query $q --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof_$q.json" 2> "$OUT/prof_$q.err")
  rc=$?; echo "$q prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
