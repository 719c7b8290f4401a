set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rows_exceptional.py > gpurun_out/r06_t10.log 2>&1 || exit $?
bash tools/ab.sh gpurun_out/ab_pf 3 qc base lib:nopf > gpurun_out/ab_pf.log 2>&1 || exit $?
