#!/bin/bash
# round 6: p1 over 1 / 2 / 4 shared queues (kernel boundaries overlapped), one process, configs alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/p1_stage_ab.py 4 8 STREAMS=1 STREAMS=2 STREAMS=4 > gpurun_out/r06f_p1_streams_ab.json 2> gpurun_out/r06f_p1_streams_ab.err || exit $?
echo done
