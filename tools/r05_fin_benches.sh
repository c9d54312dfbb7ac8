#!/bin/bash
# closing bench lines (c3 p1 g2 g1 c4, CPU baselines) and rocprof kernel stats of c3 / p1 / g2 into OUTDIR
out=${1:-gpurun_out/fin}; mkdir -p "$out"
for q in c3 p1 g2 g1 c4; do
  timeout -k 10 300 python3 bench.py --query $q > "$out/bench_$q.json" 2> "$out/bench_$q.err" || exit 1
done
for q in c3 p1 g2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$q" -o run -- python3 bench.py --query $q --steps 10 --no-cpu-baseline --no-c-host --no-rccl-world1 > "$out/${q}_under_rocprof.json" 2> "$out/prof_$q.err" || exit 1
done
echo done
