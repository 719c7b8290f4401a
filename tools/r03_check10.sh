#!/bin/bash
# Armed latency kernel with waves past the slot lines (n <= 128 served without
# a launch): latency-path GPU tests, then fresh-certificate QC p50 for the new
# and the previous library, alternating, and the full GPU suite.
set -o pipefail
OUT=${1:-gpurun_out/r03c10q}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "armed or latency or qc or empty" -x -v --timeout 120 --timeout-method thread > "$OUT/armed_tests.log" 2>&1 || { echo "armed tests failed"; tail -40 "$OUT/armed_tests.log"; exit 1; }
tail -1 "$OUT/armed_tests.log"
for r in 1 2; do
  timeout -k 10 200 python -u tools/qc_fresh.py 3000 > "$OUT/new_$r.json" || { echo "qc new failed"; exit 1; }
  PBFTV_LIB=$PWD/exp/libpbftv_old.so timeout -k 10 200 python -u tools/qc_fresh.py 3000 > "$OUT/old_$r.json" || { echo "qc old failed"; exit 1; }
  echo "new $(cat $OUT/new_$r.json | cut -c1-160)"
  echo "old $(cat $OUT/old_$r.json | cut -c1-160)"
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
