#!/bin/bash
# p1 blocks per run with the staged kernel; the C3 tail split (states vs merge + final)
out=gpurun_out/r05l; mkdir -p $out
timeout -k 10 500 python3 tools/p1_stage_ab.py 4 8 SELECT_BLOCKS_RUN=1 SELECT_BLOCKS_RUN=2 SELECT_BLOCKS_RUN=4 \
  SELECT_BLOCKS_RUN=8 SELECT_BLOCKS_STAGE=1,SELECT_BLOCKS_ROWS=16,SELECT_BLOCKS_RUN=4 > $out/p1_run_ab.json 2> $out/p1_run_ab.err || exit 1
sleep 5
timeout -k 10 200 fuse-query_amd/lib/fq_c_client --bench 20 10000000000 3 > $out/c_client_bench.json 2> $out/c_client.err || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-c-host --no-rccl-world1 > $out/bench_c3.json 2> $out/bench_c3.err || exit 1
echo done
