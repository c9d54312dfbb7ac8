#!/bin/bash
# Alternating A/B of g2's kernel set over one numbers_mt partition
# (tools/g2_random.py --narrow-iota, checked against numpy each run), then one
# rocprofv3 kernel-stats pass per configuration.
# usage: sweep_g2_shapes.sh OUTDIR ROUNDS "CFG1" "CFG2" ...   (a CFG is --tune args, "" = defaults)
out=$1; rounds=$2; shift 2
mkdir -p "$out"
for r in $(seq "$rounds"); do
  for cfg in "$@"; do
    timeout -k 10 120 python3 tools/g2_random.py --narrow-iota --reps 5 $cfg >> "$out/res.jsonl" 2>> "$out/err.log" || exit 1
  done
done
i=0
for cfg in "$@"; do
  i=$((i + 1))
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$i" -o run -- python3 tools/g2_random.py --narrow-iota --reps 3 $cfg > "$out/prof_$i.json" 2>> "$out/err.log" || exit 1
done
