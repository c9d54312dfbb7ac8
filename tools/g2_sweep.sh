#!/bin/bash
# g2 (GROUP BY number%100000) launch knobs on one GPU: chunk rows, partition
# workgroups per CU; then a kernel-trace profile of the default.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$(pwd); OUT="$R/gpurun_out/g2s"; mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=() extra=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
  [ "$1" = "--" ] && shift
  extra=("$@")
  timeout -k 10 240 env "${envs[@]}" python -u bench.py --query g2 --steps 5 --warmup 2 --no-cpu-baseline "${extra[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    print("%-28s ms/step %7.2f  kernel %6.3f ms/10GB" % (sys.argv[2], d["ms_per_step"], d["kernel_ms_per_launch"]))
except Exception as e:
    print(sys.argv[2], "no result", e)
PY
  return $rc
}
run default FQ_X=0 && \
run bins2 FQ_GBINS_PER_CU=2 && \
run bins4 FQ_GBINS_PER_CU=4 && \
run default_b FQ_X=0 && \
run bins2_b FQ_GBINS_PER_CU=2 && \
run bins4_b FQ_GBINS_PER_CU=4 && \
true || (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --query g2 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof.json" 2> "$OUT/prof.err")
