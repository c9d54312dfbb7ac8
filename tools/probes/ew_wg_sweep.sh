for w in 1 2 4 8; do FQ_TUNE_EW_WG_PER_CU=$w timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/k_w$w.json 2>/dev/null || exit 1; done
python3 - <<'PY'
import json
for w in (1,2,4,8):
    d=json.load(open('gpurun_out/k_w%d.json'%w))
    print(w, [(k['kernel'][:28], round(k['ms'],3)) for k in d['kernels'] if k['kernel'].startswith(('compare','arith'))])
PY
