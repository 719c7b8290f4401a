set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_wide_arming_is_kept_by_the_keeper" \
  "tests/test_gpu_parity.py::test_armed_kernel_does_not_hold_frees_or_other_contexts" \
  "tests/test_gpu_parity.py::test_certificates_beside_a_batch" \
  "tests/test_gpu_parity.py::test_armed_kernels_of_two_contexts_concurrent" \
  "tests/test_gpu_parity.py::test_armed_latency_path" \
  "tests/test_gpu_parity.py::test_sha256_small_calls_zero_copy" \
  tests/test_gpu_rows_exceptional.py > gpurun_out/r06_t3.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r06_t3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/armed_tax.py --streams 1 --arm-ms 100 --sizes 1048576 --configs none,rows_narrow_4,rows_wide --rounds 3 > gpurun_out/r06_armed_tax_s1_a100.json 2> gpurun_out/r06_armed_tax_s1_a100.err || exit $?
timeout -k 10 200 python -u tools/armed_tax.py --streams 1 --arm-ms 1000 --sizes 1048576 --configs none,rows_narrow_4,rows_wide --rounds 2 > gpurun_out/r06_armed_tax_s1_a1000.json 2> gpurun_out/r06_armed_tax_s1_a1000.err || exit $?
exit $rc
