set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rows_exceptional.py tests/test_gpu_parity.py -k "rows or armed or golden or crafted or certificate or qc or cu_yield or keeper or rekey" > gpurun_out/r06_t16.log 2>&1 || exit $?
bash tools/ab.sh gpurun_out/ab_poll 3 qc base env:PBFTV_QC_SPIN=999 > gpurun_out/ab_poll.log 2>&1 || exit $?
