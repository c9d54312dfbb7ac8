#!/bin/bash
# Alternating A/B of g2's kernel set between this tree and a second tree
# holding another build (its fuse-query_amd/{fq_amd,lib} and tools/g2_random.py),
# then one rocprofv3 kernel-stats pass of each.
# usage: ab_g2_trees.sh OUTDIR ROUNDS OTHER_TREE [g2_random args]
out=$1; rounds=$2; other=$3; shift 3
mkdir -p "$out"
for r in $(seq "$rounds"); do
  for t in . "$other"; do
    timeout -k 10 120 python3 "$t/tools/g2_random.py" --narrow-iota --reps 5 "$@" > "$out/tmp.json" 2>> "$out/err.log" || exit 1
    python3 -c "import json,sys; d=json.load(open('$out/tmp.json')); d['tree']='$t'; print(json.dumps(d))" >> "$out/res.jsonl" || exit 1
  done
done
for t in . "$other"; do
  n=$(basename "$t"); [ "$n" = . ] && n=new
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$n" -o run -- python3 "$t/tools/g2_random.py" --narrow-iota --reps 3 "$@" > /dev/null 2>> "$out/err.log" || exit 1
done
