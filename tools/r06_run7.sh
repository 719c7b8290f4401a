set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_t9.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r06_bench_7.json 2> gpurun_out/r06_bench_7.err || exit $?
