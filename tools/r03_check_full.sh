#!/bin/bash
# round 3 HEAD check: full GPU suite with per-test durations, smoke, C3 and p1 bench lines, p1 PMC + kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); OUT="$R/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider --durations=0 > "$OUT/full_pytest.log" 2>&1
rc=$?; grep -E "passed|failed" "$OUT/full_pytest.log" | tail -3; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/full_smoke.log" 2>&1 || exit $?
tail -2 "$OUT/full_smoke.log"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > "$OUT/full_bench_c3.json" 2> "$OUT/full_bench_c3.err" || exit $?
timeout -k 10 300 python bench.py --query p1 --steps 5 --warmup 2 > "$OUT/full_bench_p1.json" 2> "$OUT/full_bench_p1.err" || exit $?
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_p1/$C" -o pmc -- python3 "$R/bench.py" --query p1 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_p1_$C.json" 2> "$OUT/pmc_p1_$C.err") || exit $?
done
python3 tools/pmc_summary.py "$OUT/pmc_p1.json" 1250000000 $(find "$OUT/pmc_p1" -name "*counter_collection*.csv") > /dev/null || exit $?
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_p1" -o run -- python3 "$R/bench.py" --query p1 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof_p1.json" 2> "$OUT/prof_p1.err") || exit $?
python3 -c "
import json
for q in ('c3','p1'):
    d=json.load(open('$OUT/full_bench_%s.json' % q)); r=d['roofline']
    print(q, round(d['value']/1e9,1), 'G rows/s', round(d['ms_per_step'],3), 'ms/step frac', round(r['frac'],3), 'traffic', r.get('traffic_source',{}).get('status'))
"
