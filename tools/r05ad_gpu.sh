#!/bin/bash
# flake hunt: the GPU suite twice in a row
out=gpurun_out/r05ad; mkdir -p $out
for i in 1 2; do
  timeout -k 10 560 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu_$i.txt 2>&1 || exit 1
done
echo done
