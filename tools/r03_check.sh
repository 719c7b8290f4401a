#!/bin/bash
# Round-3 GPU check: allotment probe, full GPU suite, headline bench.
set -o pipefail
OUT=${1:-gpurun_out/r03}
mkdir -p "$OUT"
export TMPDIR=/tmp
{ echo "nproc=$(nproc)"; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))';
  cat /sys/fs/cgroup/cpu.max 2>&1; cat /proc/self/cgroup; cat /sys/devices/system/cpu/smt/active; } > "$OUT/allot.txt" 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
