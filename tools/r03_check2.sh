#!/bin/bash
# Round-3 check 2: full GPU suite, latency-path stage probe, QC probe, small-shard A/B.
set -o pipefail
OUT=${1:-gpurun_out/r03b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 120 ./tools/wave_kernel_probe > "$OUT/wave_kernel_probe.json" || exit 1
cat "$OUT/wave_kernel_probe.json"
timeout -k 10 300 python -u tools/qc_probe.py > "$OUT/qc_probe.json" || exit 1
cat "$OUT/qc_probe.json"
timeout -k 10 600 bash tools/streams_ab.sh "$OUT/streams" 2 "131072 0" "131072 2" "1048576 2" || exit 1
timeout -k 10 300 ./tools/gather_comb 1048576 5 > "$OUT/gather_comb.txt" || exit 1
cat "$OUT/gather_comb.txt"
