#!/bin/bash
# Closing run, part 2: smoke(), the bench lines (each a fresh process, the
# default line first), the C1 CPU line and the strong-scaling rank rehearsal.
# usage: tools/closing_bench.sh OUTDIR [QUERIES...]   (default p1 c4 g1 g2 after the default C3 line)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O="${1:-gpurun_out/close}"; mkdir -p "$O"; shift
QS="$*"; [ -n "$QS" ] || QS="p1 c4 g1 g2"
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.txt" 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || exit 1
for Q in $QS; do
  timeout -k 10 300 python3 -u bench.py --query $Q > "$O/bench_$Q.json" 2> "$O/bench_$Q.err" || exit 1
  echo "bench $Q ok"
done
timeout -k 10 120 python3 -u bench.py --cpu-only --query c2 --rows-per-gpu 1e8 > "$O/c1_cpu.json" 2> "$O/c1_cpu.err" || exit 1
timeout -k 10 180 python3 -u tools/rank_rehearsal.py --rank 7 --world 8 --rows 1e10 --steps 40 > "$O/rank7of8.json" 2> "$O/rank7of8.err" || exit 1
echo done
