#!/bin/bash
# The whole GPU test suite into OUT (default gpurun_out/suite.txt), one process, per-test timeouts.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/suite.txt}; mkdir -p "$(dirname "$OUT")"
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT" 2>&1
rc=$?; tail -3 "$OUT"; exit $rc
