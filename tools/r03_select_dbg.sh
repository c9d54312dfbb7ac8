cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
for cfg in 3:32 3:16 1:32; do IFS=: read v rows <<< "$cfg"
FQ_TUNE_SELECT_VARIANT=$v FQ_TUNE_SELECT_ROWS=$rows KEEP=0.375 NOUT=2 FQ_TUNE_SELECT_DEBUG=1 timeout -k 10 120 python tools/select_probe.py 2>&1 | grep -E "select-debug|keep=" | tail -2 || exit $?
done
