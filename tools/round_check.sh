#!/bin/bash
# One GPU call, any subset of the standard checks, in order, stopping at the
# first failure (each step under its own time limit).  Run on the GPU box from
# the repo root:
#   bash tools/round_check.sh OUT step [step ...]
# steps:
#   tests          the full -m gpu suite               -> OUT/gpu_tests.log
#   tests:EXPR     the -m gpu tests selected by -k EXPR -> OUT/gpu_tests_k.log
#   smoke          __graft_entry__.smoke()             -> OUT/smoke.log
#   bench          bench.py, default arguments         -> OUT/bench.json
#   qc             tools/qc_fresh.py 4000              -> OUT/qc_fresh.json
#   cadence[:P]    tools/qc_cadence.py --parts P       -> OUT/cadence.jsonl
#   profile        bench under rocprofv3 + PMC passes  -> OUT/prof/ (tools/profile.sh)
#   allot          the CPU allotment evidence          -> OUT/allot.txt
set -o pipefail
OUT=${1:?usage: round_check.sh OUT step...}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
      tail -1 "$OUT/gpu_tests.log" ;;
    tests:*)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${step#tests:}" \
        > "$OUT/gpu_tests_k.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests_k.log"; exit 1; }
      tail -1 "$OUT/gpu_tests_k.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
      tail -1 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
      tail -c 400 "$OUT/bench.json"; echo ;;
    qc)
      timeout -k 10 300 python -u tools/qc_fresh.py 4000 > "$OUT/qc_fresh.json" || { echo "qc failed"; exit 1; }
      cut -c1-300 "$OUT/qc_fresh.json" ;;
    cadence*)
      parts=${step#cadence}; parts=${parts#:}
      timeout -k 10 400 python -u tools/qc_cadence.py ${parts:+--parts $parts} >> "$OUT/cadence.jsonl" \
        2>> "$OUT/cadence.err" || { echo "cadence failed"; tail -20 "$OUT/cadence.err"; exit 1; } ;;
    profile)
      timeout -k 10 1500 bash tools/profile.sh "$OUT/prof" > "$OUT/profile.log" 2>&1 \
        || { echo "profile failed"; tail -30 "$OUT/profile.log"; exit 1; }
      tail -5 "$OUT/profile.log" ;;
    allot)
      { echo "nproc=$(nproc)"; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))';
        cat /sys/fs/cgroup/cpu.max; cat /sys/devices/system/cpu/smt/active; } > "$OUT/allot.txt" 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
