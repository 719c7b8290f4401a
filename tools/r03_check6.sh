#!/bin/bash
set -o pipefail
OUT=${1:-gpurun_out/r03g}
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/qc_fresh.py 4000 > "$OUT/qc_fresh.json" || exit 1
cat "$OUT/qc_fresh.json"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
