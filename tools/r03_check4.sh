#!/bin/bash
# Armed latency path: armed-path test first, then the full GPU suite, fresh-certificate QC p50, QC probe.
set -o pipefail
OUT=${1:-gpurun_out/r03d}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k armed > "$OUT/armed_tests.log" 2>&1 || { echo "armed tests failed"; tail -40 "$OUT/armed_tests.log"; exit 1; }
tail -2 "$OUT/armed_tests.log"
timeout -k 10 300 python -u tools/qc_fresh.py 4000 > "$OUT/qc_fresh.json" || exit 1
cat "$OUT/qc_fresh.json"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
