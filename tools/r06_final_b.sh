set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_rows_exceptional.py > gpurun_out/r06_t7.log 2>&1 || exit $?
bash tools/profile.sh gpurun_out/prof6 > gpurun_out/prof6.log 2>&1
