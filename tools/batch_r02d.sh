#!/bin/bash
# GROUP BY: GPU tests, then the g2 / g1 benches
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/r02d; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_groupby_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for q in g2 g1; do
timeout -k 10 300 python bench.py --query $q --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_$q.json 2> $OUT/bench_$q.err; rc=$?; cat $OUT/bench_$q.json; [ $rc -eq 0 ] || exit $rc
done
