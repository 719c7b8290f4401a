set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_t13.log 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_smoke2.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r06_bench_9.json 2> gpurun_out/r06_bench_9.err || exit $?
