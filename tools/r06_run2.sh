set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r06_full2.log 2>&1
rc=$?
echo "suite rc=$rc" >> gpurun_out/r06_full2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 ./tools/fmul_alt_bench > gpurun_out/r06_fmul_alt.txt 2>&1 || exit $?
python tools/fmul_alt_check.py < gpurun_out/r06_fmul_alt.txt > gpurun_out/r06_fmul_alt_checked.txt 2>&1
timeout -k 10 240 python -u tools/armed_tax.py > gpurun_out/r06_armed_tax.json 2> gpurun_out/r06_armed_tax.err || exit $?
exit $rc
