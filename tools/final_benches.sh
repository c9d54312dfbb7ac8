#!/bin/bash
# Round-end bench lines (with CPU baselines), rocprof kernel stats of the
# headline queries, the GPU test suite and smoke(), into OUTDIR.
# usage: final_benches.sh OUTDIR
out=${1:-gpurun_out/fin}
mkdir -p "$out"
for q in c3 p1 g2 g1 c4; do
  timeout -k 10 300 python3 bench.py --query $q > "$out/bench_$q.json" 2> "$out/bench_$q.err" || exit 1
done
for q in c3 p1 g2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$q" -o run -- python3 bench.py --query $q --steps 10 --no-cpu-baseline --no-c-host --no-rccl-world1 > "$out/${q}_under_rocprof.json" 2> "$out/prof_$q.err" || exit 1
done
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$out/pytest_gpu.txt" 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 || exit 1
echo done
