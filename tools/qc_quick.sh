#!/bin/bash
# Quick latency-path GPU check: wave-path parity tests, stage probe, QC latency.
set -eo pipefail
OUT=${1:-gpurun_out/qcq}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_geometry.py -m gpu -x -v --timeout 200 \
  --timeout-method thread -k "wave or qc or small" > "$OUT/tests.log" 2>&1
timeout -k 10 120 ./tools/wave_kernel_probe > "$OUT/wave_kernel_probe.json"
timeout -k 10 300 python -u tools/qc_probe.py > "$OUT/qc_probe.json"
