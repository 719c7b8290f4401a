set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 ./tools/rows_probe > gpurun_out/rows_probe8.json 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rows_exceptional.py tests/test_gpu_parity.py -k "rows or armed or golden or crafted or wave or certificate or qc" > gpurun_out/r06_t14.log 2>&1 || exit $?
bash tools/ab.sh gpurun_out/ab_tail 3 qc base lib:oldtail > gpurun_out/ab_tail.log 2>&1 || exit $?
