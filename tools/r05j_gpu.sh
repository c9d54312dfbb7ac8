#!/bin/bash
# how long a scan stays slow after another process freed its HBM (tools/reclaim_probe.py)
out=gpurun_out/r05j; mkdir -p $out
timeout -k 10 200 python3 tools/reclaim_probe.py none 0 12 > $out/probe_none_1.json 2> $out/probe_none_1.err || exit 1
timeout -k 10 300 python3 tools/reclaim_probe.py free 80 12 > $out/probe_free80.json 2> $out/probe_free80.err || exit 1
timeout -k 10 300 python3 tools/reclaim_probe.py free 160 12 > $out/probe_free160.json 2> $out/probe_free160.err || exit 1
sleep 30
timeout -k 10 200 python3 tools/reclaim_probe.py none 0 12 > $out/probe_none_2.json 2> $out/probe_none_2.err || exit 1
echo done
