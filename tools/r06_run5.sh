set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_parity.py::test_certificates_beside_a_batch" \
  "tests/test_gpu_parity.py::test_armed_kernels_of_two_contexts_concurrent" \
  "tests/test_gpu_parity.py::test_split_wide_certificates" > gpurun_out/r06_t5.log 2>&1 || exit $?
bash tools/ab.sh gpurun_out/ab_busy6 2 load base env:PBFTV_QC_BUSY_ONE_WAVE=0 env:PBFTV_QC_EXCLUSIVE_CU=narrow env:PBFTV_QC_EXCLUSIVE_CU=80 > gpurun_out/ab_busy6.log 2>&1
