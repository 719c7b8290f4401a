#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, --kernel-trace
# only, never combined with sys/runtime traces).  Run on the GPU box from the
# repo root:  bash tools/pmc_passes.sh gpurun_out/pmc
set -euo pipefail
OUT=${1:-gpurun_out/pmc}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/$name" -o run --pmc "$@" \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-extras > "$ROOT/$OUT/$name.log" 2>&1
}
pass sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
pass sq2 SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC
pass fetch FETCH_SIZE
pass write WRITE_SIZE
