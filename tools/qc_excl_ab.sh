#!/bin/bash
# QC latency under a concurrent 1M stream with and without PBFTV_QC_EXCLUSIVE_CU=1
# (armed workgroups take whole CUs): the armed tests with it on, then
# tools/qc_cadence.py --parts load alternating, 2 rounds.   bash tools/qc_excl_ab.sh
set -o pipefail
mkdir -p gpurun_out/r04ae
PBFTV_QC_EXCLUSIVE_CU=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k armed > gpurun_out/r04ae/tests_excl.log 2>&1 || { echo "excl tests failed"; tail -30 gpurun_out/r04ae/tests_excl.log; exit 1; }
tail -1 gpurun_out/r04ae/tests_excl.log
for r in 1 2; do
  timeout -k 10 200 python -u tools/qc_cadence.py --parts load > gpurun_out/r04ae/load_base_$r.jsonl 2> gpurun_out/r04ae/load_base_$r.err || exit 1
  PBFTV_QC_EXCLUSIVE_CU=1 timeout -k 10 200 python -u tools/qc_cadence.py --parts load > gpurun_out/r04ae/load_excl_$r.jsonl 2> gpurun_out/r04ae/load_excl_$r.err || exit 1
done
