#!/bin/bash
# One GPU call: the default bench line (JSON) and the rocprofv3 kernel stats of
# a short bench run (the profiled command is bench.py --no-extras).
#   bash tools/bench_check.sh gpurun_out/bench
set -eo pipefail
OUT=${1:-gpurun_out/bench}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run \
  -- python3 "$ROOT/bench.py" --no-extras > "$ROOT/$OUT/prof_bench.json" 2> "$ROOT/$OUT/prof.log"
