set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r06_final_tests.log 2>&1
rc=$?
echo "suite rc=$rc" >> gpurun_out/r06_final_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_smoke.log 2>&1 || exit $?
PBFTV_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python -u bench.py --gpus 2 --no-extras --steps 20 > gpurun_out/r06_bench_gpus2_share.json 2> gpurun_out/r06_bench_gpus2_share.err || exit $?
exit $rc
