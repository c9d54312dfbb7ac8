#!/bin/bash
# round 6: C3 and C4 over 1 / 2 shared queues, one process each, configs alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/streams_ab.py 6 20 c3 1 2 > gpurun_out/r06g_c3_streams_ab.json 2> gpurun_out/r06g_c3_streams_ab.err || exit $?
timeout -k 10 300 python -u tools/streams_ab.py 4 20 c4 1 2 > gpurun_out/r06g_c4_streams_ab.json 2> gpurun_out/r06g_c4_streams_ab.err || exit $?
echo done
