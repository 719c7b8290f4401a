#!/bin/bash
# Latency-path check: wave-path parity tests, stage probe, fresh-certificate QC p50 (default, G24).
set -o pipefail
OUT=${1:-gpurun_out/r03c}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_geometry.py tests/test_gpu_parity.py tests/test_gpu_messages.py tests/test_gpu_keys_devices.py -m gpu -x -v --timeout 300 --timeout-method thread -k "wave or qc or geometry or width or crafted or flush or padding or caller" > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 120 ./tools/wave_kernel_probe > "$OUT/wave_kernel_probe.json" || exit 1
cat "$OUT/wave_kernel_probe.json"
timeout -k 10 300 python -u tools/qc_fresh.py 4000 > "$OUT/qc_default.json" || exit 1
cat "$OUT/qc_default.json"
PBFTV_GBITS=24 timeout -k 10 300 python -u tools/qc_fresh.py 4000 > "$OUT/qc_g24.json" || exit 1
cat "$OUT/qc_g24.json"
timeout -k 10 120 ./tools/launch_rt 5000 > "$OUT/launch_rt.json" || exit 1
cat "$OUT/launch_rt.json"
