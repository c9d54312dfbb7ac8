#!/bin/bash
# round 6: p1 kernel + HIP runtime trace (where the gaps between projection launches come from)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace -d $GRAFT_REPO_ROOT/gpurun_out/r06c_p1trace -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/p1_stage_ab.py 1 2 ENGINE_PROJECT_LAUNCH=1 > $GRAFT_REPO_ROOT/gpurun_out/r06c_p1trace.json 2> $GRAFT_REPO_ROOT/gpurun_out/r06c_p1trace.err || exit $?
ls -la $GRAFT_REPO_ROOT/gpurun_out/r06c_p1trace
echo done
