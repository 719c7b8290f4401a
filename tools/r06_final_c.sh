set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r06_final_tests_c.log 2>&1
rc=$?
echo "suite rc=$rc" >> gpurun_out/r06_final_tests_c.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_smoke_c.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r06_bench_final_c.json 2> gpurun_out/r06_bench_final_c.err || exit $?
exit $rc
