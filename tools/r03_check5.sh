#!/bin/bash
# Armed latency path v2: armed + wave-path tests, fresh-certificate QC p50.
set -o pipefail
OUT=${1:-gpurun_out/r03e}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_messages.py -m gpu -x -v --timeout 120 --timeout-method thread -k "armed or qc or wave or flush" > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python -u tools/qc_fresh.py 4000 > "$OUT/qc_fresh.json" || exit 1
cat "$OUT/qc_fresh.json"
PBFTV_QC_ARM=0 timeout -k 10 300 python -u tools/qc_fresh.py 4000 > "$OUT/qc_fresh_noarm.json" || exit 1
cat "$OUT/qc_fresh_noarm.json"
