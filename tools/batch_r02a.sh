#!/bin/bash
# round-2 probes: timing-event flags between scans, step overhead, g2 host path
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/r02a; mkdir -p $OUT
timeout -k 10 150 python tools/gap_probe.py > $OUT/gap_probe.txt 2>&1; rc=$?; cat $OUT/gap_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/step_overhead.py > $OUT/step_overhead.txt 2>&1; rc=$?; cat $OUT/step_overhead.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --query g2 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_g2.json 2> $OUT/bench_g2.err; rc=$?; cat $OUT/bench_g2.json; tail -3 $OUT/bench_g2.err; exit $rc
