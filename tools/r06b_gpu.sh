#!/bin/bash
# round 6, second GPU call: C3 line on a fresh process, C1 CPU line, the rank rehearsal, a p1 kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u bench.py > gpurun_out/r06b_bench_c3.json 2> gpurun_out/r06b_bench_c3.err || exit $?
timeout -k 10 120 python -u bench.py --cpu-only --query c2 --rows-per-gpu 1e8 > gpurun_out/r06b_c1_cpu.json 2> gpurun_out/r06b_c1_cpu.err || exit $?
timeout -k 10 180 python -u tools/rank_rehearsal.py --rank 7 --world 8 --rows 1e10 --steps 40 > gpurun_out/r06b_rank7of8.json 2> gpurun_out/r06b_rank7of8.err || exit $?
timeout -k 10 180 python -u tools/rank_rehearsal.py --rank 0 --world 1 --rows 1e10 --steps 20 > gpurun_out/r06b_rank0of1.json 2> gpurun_out/r06b_rank0of1.err || exit $?
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06b_p1trace -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/p1_stage_ab.py 1 4 ENGINE_PROJECT_LAUNCH=1 ENGINE_PROJECT_LAUNCH=2 > $GRAFT_REPO_ROOT/gpurun_out/r06b_p1trace.json 2> $GRAFT_REPO_ROOT/gpurun_out/r06b_p1trace.err || exit $?
echo done
