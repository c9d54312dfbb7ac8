#!/bin/bash
# p1 through the engine: async path vs the launch path with the hand-off after the kernel / in it, one process
out=gpurun_out/r05ab; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_project_blocks_gpu.py -x -q --timeout 300 --timeout-method thread > $out/pytest.txt 2>&1 || exit 1
timeout -k 10 600 python3 tools/p1_stage_ab.py 4 8 ENGINE_PROJECT_LAUNCH=0 ENGINE_PROJECT_LAUNCH=1,PROJECT_HANDOFF=0 \
  ENGINE_PROJECT_LAUNCH=1,PROJECT_HANDOFF=1 > $out/p1_handoff_ab.json 2> $out/p1_handoff_ab.err || exit 1
echo done
