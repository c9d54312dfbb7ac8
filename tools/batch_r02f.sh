#!/bin/bash
# dense-key GROUP BY: GPU tests (groupby + fuzz), g1 bench, kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); OUT=$R/gpurun_out/r02f; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_groupby_gpu.py tests/test_fuzz_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --query g1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_g1.json 2> $OUT/bench_g1.err; rc=$?; cut -c1-300 $OUT/bench_g1.json; grep -o '"kernel_ms_per_launch": [0-9.]*' $OUT/bench_g1.json; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --query g1 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof.json 2> $OUT/prof.err; rc=$?
cut -c1-160 $(find $OUT/prof -name "*kernel_stats.csv") | head -6; exit $rc
