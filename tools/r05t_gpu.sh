#!/bin/bash
# LIMIT latency per commit (worktrees under bisect/, each with its own build), alternating
out=gpurun_out/r05t2; mkdir -p $out
for round in 1 2; do
  for c in 085a9e4 37f6c2d afb5ba4 HEAD; do
    d=bisect/$c; [ $c = HEAD ] && d=.
    echo "== $c" >> $out/limit_probe.txt
    timeout -k 10 200 python3 $d/tools/limit_probe.py >> $out/limit_probe.txt 2>> $out/limit_probe.err || exit 1
  done
done
echo done
