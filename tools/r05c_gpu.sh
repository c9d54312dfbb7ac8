#!/bin/bash
# one C3 query traced (kernels + HIP API) in the engine's bench configuration
# (FQ_OPT_PROFILE 2), then the finalize-form A/B again
R=$(pwd); out=gpurun_out/r05c; mkdir -p $out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$R/$out/trace" -o run -- \
  python3 "$R/tools/readme_window.py" c3 2 > "$R/$out/window.txt" 2> "$R/$out/trace.err") || exit 1
K=$(find $out/trace -name "*kernel_trace.csv" | head -1); A=$(find $out/trace -name "*hip_api_trace.csv" | head -1)
python3 tools/window_timeline.py $out/window.txt "$K" "$A" > $out/c3_query_timeline.txt || exit 1
rm -rf $out/trace
timeout -k 10 300 python3 tools/scan_fin_ab.py 6 > $out/scan_fin_ab.json 2> $out/scan_fin_ab.err || exit 1
sleep 15  # the A/B process's 80 GB reclaimed before the next timed run
timeout -k 10 300 python3 bench.py --query p1 --no-cpu-baseline > $out/bench_p1.json 2> $out/bench_p1.err || exit 1
sleep 15
timeout -k 10 300 python3 bench.py > $out/bench_c3.json 2> $out/bench_c3.err || exit 1
echo done
