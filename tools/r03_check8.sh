#!/bin/bash
# Host-path concurrency build: host-pipeline GPU tests (incl. concurrent
# callers), the full bench line (host_path.pageable_2_callers), then the
# scalar-stage K A/B under two-stream overlap.
set -o pipefail
OUT=${1:-gpurun_out/r03c8}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "host_pipeline" -x -v --timeout 300 --timeout-method thread > "$OUT/host_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/host_tests.log"; exit 1; }
tail -2 "$OUT/host_tests.log"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['value']/1e6, d['ms_per_step'], json.dumps(d.get('host_path')))"
timeout -k 10 900 bash tools/streams_ab.sh "$OUT/kab" 2 "1048576 2" "1048576 2 PBFTV_SCALAR_BATCH=8" "131072 2" "131072 2 PBFTV_SCALAR_BATCH=4" "131072 2 PBFTV_SCALAR_BATCH=1" || { echo "kab failed"; exit 1; }
