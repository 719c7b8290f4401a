#!/bin/bash
# Windowed SHA sort + XCD-local blocks (in-tree) vs exp/libpbftv_old.so: SHA tests, timings,
# SQ counters (tools/sha_lib_ab.sh) and the L2 fabric read requests per launch.
set -o pipefail
OUT=gpurun_out/r04ai
bash tools/sha_lib_ab.sh $OUT 2 old || exit 1
ROOT=$(pwd)
cd /tmp
for v in base old; do
  L=""; [ "$v" = base ] || L=$ROOT/exp/libpbftv_$v.so
  PBFTV_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/tcc_$v" -o run --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum \
    -- python3 "$ROOT/tools/pmc_workload.py" sha > "$ROOT/$OUT/tcc_$v.log" 2>&1 || { echo "tcc $v failed"; exit 1; }
done
echo done
