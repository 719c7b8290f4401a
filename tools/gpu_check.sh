#!/bin/bash
# One GPU call: parity tests, headline bench (JSON line), rocprofv3 kernel
# stats of a short bench.  Run on the GPU box from the repo root:
#   bash tools/gpu_check.sh gpurun_out/check
set -eo pipefail
OUT=${1:-gpurun_out/check}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run \
  -- python3 "$ROOT/bench.py" --no-extras > "$ROOT/$OUT/prof_bench.json" 2> "$ROOT/$OUT/prof.log"
