out=gpurun_out/r05b; mkdir -p $out
timeout -k 10 300 python3 tools/scan_fin_ab.py 6 > $out/scan_fin_ab.json 2> $out/scan_fin_ab.err || exit 1
bash tools/host_spread.sh $out/host_spread || exit 1
timeout -k 10 300 python3 bench.py > $out/bench_c3.json 2> $out/bench_c3.err || exit 1
echo done
