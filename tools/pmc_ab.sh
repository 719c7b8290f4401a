#!/bin/bash
# One PMC pass (cycles + VALU counts) over the config-4 verify for the in-tree
# library and experiment builds exp/libpbftv_<v>.so: do the variants differ in
# cycles, or only in clock?   bash tools/pmc_ab.sh OUT v1 [v2 ...]
set -euo pipefail
OUT=$1; shift
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for v in base "$@"; do
  L=""; [ "$v" = base ] || L=$ROOT/exp/libpbftv_$v.so
  PBFTV_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/$v" -o run \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -- python3 "$ROOT/tools/pmc_workload.py" comb > "$ROOT/$OUT/$v.log" 2>&1
done
