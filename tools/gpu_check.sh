#!/bin/bash
# One GPU session: gpu tests -> smoke -> bench -> rocprofv3 stats.
# Stops at the first crash/timeout (exit >= 2 from pytest, or any signal).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd)
OUT="$R/gpurun_out"
mkdir -p "$OUT"
STEPS=${STEPS:-10}
rc_ok() { # $1 = exit code; test failures (1) are reported, crashes stop the script
  [ "$1" -eq 0 ] || [ "$1" -eq 1 ]
}
echo "== pytest -m gpu"
timeout -k 10 ${PYTEST_T:-420} python -m pytest tests -m gpu -q ${PYTEST_ARGS} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -25 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"
rc_ok $rc || exit $rc
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -5 "$OUT/smoke.log"; echo "smoke rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
echo "== bench"
timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -5 "$OUT/bench.err"; cat "$OUT/bench.json"; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_PROF" ] && exit 0
echo "== rocprofv3 kernel trace"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --steps $STEPS --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"
rc=$?; echo "rocprof rc=$rc"; find "$OUT/prof" -name "*stats*" | head
exit $rc
