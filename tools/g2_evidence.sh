#!/bin/bash
# g2 (GROUP BY number%100000) evidence on one GPU: bench line with the CPU
# baseline, kernel-trace stats, FETCH_SIZE / WRITE_SIZE PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); OUT="$R/gpurun_out/g2e"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --query g2 --steps 10 --warmup 3 > "$OUT/bench_g2.json" 2> "$OUT/bench_g2.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_g2.json"; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --query g2 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof.json" 2> "$OUT/prof.err"
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/$C" -o pmc -- python3 "$R/bench.py" --query g2 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_$C.json" 2> "$OUT/pmc_$C.err"
  rc=$?; echo "$C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
