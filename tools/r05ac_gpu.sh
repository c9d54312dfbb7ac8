#!/bin/bash
# the C3 line with the leaner timed step
out=gpurun_out/r05ac; mkdir -p $out
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-rccl-world1 > $out/bench_c3_$i.json 2> $out/bench_c3_$i.err || exit 1
done
echo done
