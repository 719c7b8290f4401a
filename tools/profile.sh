#!/bin/bash
# Profiles of the current library: the headline bench under rocprofv3
# --kernel-trace --stats (its HIP-event kernel averages must agree with the
# trace), then PMC passes (one counter group per pass) over tools/pmc_workload.py.
set -o pipefail
OUT=${1:-gpurun_out/prof}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/trace" -o run -- python3 "$ROOT/bench.py" --no-extras \
  > "$ROOT/$OUT/bench_under_rocprof.json" 2> "$ROOT/$OUT/trace.log" || { echo "trace failed"; tail -20 "$ROOT/$OUT/trace.log"; exit 1; }
cat "$ROOT/$OUT/bench_under_rocprof.json"
cd "$ROOT"
timeout -k 10 900 bash tools/pmc_passes.sh "$OUT/pmc" > "$OUT/pmc_passes.log" 2>&1 || { echo "pmc failed"; tail -20 "$OUT/pmc_passes.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_summary.json" 2> "$OUT/pmc_summary.err" || { echo "summary failed"; cat "$OUT/pmc_summary.err"; exit 1; }
cat "$OUT/pmc_summary.json"
python3 tools/rocpd_stats.py "$OUT/trace/run_results.db" > "$OUT/kernel_stats.csv"  # rocpd SQLite output (ROCm 7)
head -20 "$OUT/kernel_stats.csv"
