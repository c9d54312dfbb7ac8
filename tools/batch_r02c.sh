#!/bin/bash
# bench g2 (profile mode) under a kernel + HIP API trace: timeline of the last steps
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); OUT=$R/gpurun_out/r02c; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/tr -o run -- python3 $R/bench.py --query g2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err
rc=$?; cat $OUT/b.json; [ $rc -eq 0 ] || exit $rc
K=$(find $OUT/tr -name "*kernel_trace.csv" | head -1); A=$(find $OUT/tr -name "*hip_api_trace.csv" | head -1)
python3 $R/tools/trace_timeline.py $K $A 900 300 > $OUT/timeline.txt 2>&1; head -150 $OUT/timeline.txt
rm -rf $OUT/tr
