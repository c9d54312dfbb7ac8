#!/bin/bash
# g2 query: one execution under a kernel + HIP API trace, cut to its window
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); OUT=$R/gpurun_out/r02b; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/tr -o run -- python3 $R/tools/readme_window.py g2 > $OUT/win.txt 2> $OUT/win.err
rc=$?; cat $OUT/win.txt; [ $rc -eq 0 ] || exit $rc
K=$(find $OUT/tr -name "*kernel_trace.csv" | head -1); A=$(find $OUT/tr -name "*hip_api_trace.csv" | head -1)
python3 $R/tools/trace_window.py $OUT/win.txt $K $A > $OUT/summary.txt 2>&1; cat $OUT/summary.txt | head -80
rm -rf $OUT/tr
