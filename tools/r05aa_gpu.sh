#!/bin/bash
# pool spin on/off for the C3 line's host time, alternating processes
out=gpurun_out/r05aa; mkdir -p $out
for i in 1 2 3; do
  for v in 1000 0; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-c-host --no-rccl-world1 --tune POOL_SPIN_US=$v > $out/bench_spin${v}_$i.json 2> $out/bench_spin${v}_$i.err || exit 1
  done
done
echo done
