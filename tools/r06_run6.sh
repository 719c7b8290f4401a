set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 90 ./tools/divstep_lat > gpurun_out/divstep_lat4.json 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_t8.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r06_bench_6.json 2> gpurun_out/r06_bench_6.err || exit $?
