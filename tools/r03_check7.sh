#!/bin/bash
# Comb first-pair / fused-last-step build: GPU parity suite, same-box A/B
# against the previous library (exp/libpbftv_old.so), one PMC VALU pass.
set -o pipefail
OUT=${1:-gpurun_out/r03c7}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 900 bash tools/ab.sh 3 old || { echo "ab failed"; exit 1; }
python3 tools/ab_summary.py gpurun_out/ab 2>/dev/null || ls gpurun_out/ab
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/pmc/valu" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 "$ROOT/tools/pmc_workload.py" > "$ROOT/$OUT/pmc_valu.log" 2>&1 || { echo "pmc failed"; tail "$ROOT/$OUT/pmc_valu.log"; exit 1; }
echo pmc-ok
