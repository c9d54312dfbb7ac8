cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/q
timeout -k 10 300 python -u tools/bench_kernels.py > gpurun_out/kernels.json 2> gpurun_out/kernels.err; rc=$?; cat gpurun_out/kernels.err | tail -30; [ $rc -eq 0 ] || exit $rc
for qq in c2 c3 c4 max max1 avg g1; do
timeout -k 10 300 python bench.py --query $qq --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/q/$qq.json 2> gpurun_out/q/$qq.err; rc=$?; python -c "import json,sys;d=json.load(open('gpurun_out/q/$qq.json'));print('$qq', round(d['value']/1e9,1), 'G rows/s', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['achieved']), 'GB/s', round(d['roofline']['frac'],3))"; [ $rc -eq 0 ] || exit $rc
done
