#!/bin/bash
# GPU check of the device Go-JSON / pool-flush path: its parity tests and the
# config-1 end-to-end timing.  Run on the GPU box from the repo root.
set -eo pipefail
OUT=${1:-gpurun_out/msg}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_messages.py tests/test_gpu_parity.py -m gpu -x -v \
  --timeout 200 --timeout-method thread -k "gojson or flush or digest or hash or vote" > "$OUT/tests.log" 2>&1
timeout -k 10 200 python -u -c "
import bench, json
from simple_pbft_amd import Verifier
v = Verifier()
print(json.dumps(bench.run_config1(v)))
" > "$OUT/c1.json" 2> "$OUT/c1.err"
