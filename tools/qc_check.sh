#!/bin/bash
# One GPU call for the latency path: the full -m gpu suite, the in-kernel stage
# probe of the one-wave-per-signature kernel, and the QC latency split
# (tools/qc_probe.py).  Run on the GPU box from the repo root.
set -eo pipefail
OUT=${1:-gpurun_out/qc}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 120 ./tools/wave_kernel_probe > "$OUT/wave_kernel_probe.json" 2> "$OUT/wave_kernel_probe.err"
timeout -k 10 300 python -u tools/qc_probe.py > "$OUT/qc_probe.json" 2> "$OUT/qc_probe.err"
