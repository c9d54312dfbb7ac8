#!/bin/bash
# g2 kernel stats, narrow partition rows on and off (FQ_TUNE_GROUP_NARROW)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); OUT="$R/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
for nw in ${NARROWS:-0 1}; do
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_g2q$nw" -o run -- python3 "$R/bench.py" --query g2 --steps 5 --warmup 1 --no-cpu-baseline --tune GROUP_NARROW=$nw > "$OUT/prof_g2q$nw.json" 2> "$OUT/prof_g2q$nw.err") || exit $?
echo "narrow=$nw"; head -3 "$OUT/prof_g2q$nw/run_kernel_stats.csv" | tail -2 | cut -c1-100
done
