#!/bin/bash
# PMC passes over tools/pmc_workload.py (config-4 verify, config-5 digests, one
# quorum certificate): one counter group per pass (<= 8 SQ, 1 GRBM, or one TCC
# size counter), --kernel-trace only, never combined with sys/runtime traces.
# Run on the GPU box from the repo root:  bash tools/pmc_passes.sh gpurun_out/pmc
# Summarise with:  python tools/pmc_summary.py gpurun_out/pmc
set -euo pipefail
OUT=${1:-gpurun_out/pmc}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  echo "pmc pass $name: $*"
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/$name" -o run --pmc "$@" \
    -- python3 "$ROOT/tools/pmc_workload.py" > "$ROOT/$OUT/$name.log" 2>&1
}
pass valu SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU \
  SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pass wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD \
  SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
