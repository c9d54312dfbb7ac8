#!/bin/bash
# GROUP BY narrow partition rows: suites, g2 bench, kernel stats, PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); OUT="$R/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_groupby_gpu.py tests/test_fuzz_groupby_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/g2_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/g2_pytest.log"; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --query g2 --steps 5 --warmup 2 > "$OUT/g2_bench.json" 2> "$OUT/g2_bench.err" || exit $?
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_g2n" -o run -- python3 "$R/bench.py" --query g2 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof_g2n.json" 2> "$OUT/prof_g2n.err") || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_g2/$C" -o pmc -- python3 "$R/bench.py" --query g2 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_g2_$C.json" 2> "$OUT/pmc_g2_$C.err") || exit $?
done
python3 tools/pmc_summary.py "$OUT/pmc_g2.json" 416666688 $(find "$OUT/pmc_g2" -name "*counter_collection*.csv") | cut -c1-200
head -5 "$OUT/prof_g2n/run_kernel_stats.csv" | cut -c1-120
python3 -c "import json;d=json.load(open('$OUT/g2_bench.json'));print('g2', d['ms_per_step'], d['kernel_ms_per_launch'], d['value']/1e9)"
