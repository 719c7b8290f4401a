set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r06_full4.log 2>&1
rc=$?
echo "suite rc=$rc" >> gpurun_out/r06_full4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u bench.py > gpurun_out/r06_bench4.json 2> gpurun_out/r06_bench4.err || exit $?
exit $rc
