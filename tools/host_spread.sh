#!/bin/bash
# The C3 step from the two hosts of the C ABI, alternated in one box: the
# torch-hosted bench process (torch's ROCm 7.0 HIP runtime) and the C host
# (fq_c_client --bench: /opt/rocm 7.2 runtime, no torch), back to back and
# after 20 s pauses -- what separates their lines.
# usage: tools/host_spread.sh OUTDIR
out=${1:-gpurun_out/host_spread}
mkdir -p "$out"
B="timeout -k 10 240 python3 bench.py --no-c-host --no-rccl-world1 --no-cpu-baseline"
C="timeout -k 10 240 fuse-query_amd/lib/fq_c_client --bench 20 10000000000 3"
$B > "$out/1_torch.json" 2> "$out/1_torch.err" || exit 1
$C > "$out/2_c.json" 2> "$out/2_c.err" || exit 1
sleep 20
$B > "$out/3_torch_after_pause.json" 2> "$out/3_torch.err" || exit 1
sleep 20
$C > "$out/4_c_after_pause.json" 2> "$out/4_c.err" || exit 1
$C > "$out/5_c_back_to_back.json" 2> "$out/5_c.err" || exit 1
$B > "$out/6_torch_back_to_back.json" 2> "$out/6_torch.err" || exit 1
sleep 20
$B > "$out/7_torch_after_pause.json" 2> "$out/7_torch.err" || exit 1
echo done
