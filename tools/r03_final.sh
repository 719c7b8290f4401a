#!/bin/bash
# Round-3 final measurement on the final library: full GPU suite, smoke(),
# headline bench, fresh-certificate QC latency, rocprofv3 kernel trace of the
# bench (HIP-event kernel averages must agree) and the PMC passes.
set -o pipefail
OUT=${1:-gpurun_out/r03final}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
tail -c 600 "$OUT/bench.json"; echo
timeout -k 10 300 python -u tools/qc_fresh.py 4000 > "$OUT/qc_fresh.json" || { echo "qc failed"; exit 1; }
cat "$OUT/qc_fresh.json"
bash tools/r03_profile.sh "$OUT/prof" > "$OUT/profile.log" 2>&1 || { echo "profile failed"; tail -30 "$OUT/profile.log"; exit 1; }
tail -5 "$OUT/profile.log"
