set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rows_exceptional.py tests/test_gpu_parity.py -k "wide or armed or split or rekey or qc or certificate" > gpurun_out/r06_t11.log 2>&1 || exit $?
WM_TOOL=numa_split.py WM_ARGS= WM_NT="1" bash tools/wm_numa.sh || exit $?
