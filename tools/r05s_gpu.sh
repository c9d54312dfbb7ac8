#!/bin/bash
# LIMIT latency against round 4: which round-5 change costs it
out=gpurun_out/r05s; mkdir -p $out
for v in "" "POOL_SPIN_US=0" "SELECT_VARIANT=1" "BLOCK_CACHE=0" ""; do
  timeout -k 10 200 python3 tools/limit_probe.py $v >> $out/limit_probe.txt 2>> $out/limit_probe.err || exit 1
done
echo done
