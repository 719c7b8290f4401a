#!/bin/bash
# One GPU call after a comb-geometry change: all GPU parity tests (geometry
# module included), the headline bench, a rocprofv3 kernel-stats run and the
# PMC traffic passes.  Run on the GPU box from the repo root:
#   bash tools/gpu_geom.sh gpurun_out/geom
set -eo pipefail
OUT=${1:-gpurun_out/geom}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run \
  -- python3 "$ROOT/bench.py" --no-extras > "$ROOT/$OUT/prof_bench.json" 2> "$ROOT/$OUT/prof.log"
cd "$ROOT"
bash tools/pmc_passes.sh "$OUT/pmc"
python tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_traffic.json"
