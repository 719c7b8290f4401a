#!/bin/bash
# Times experiment builds of libpbftv.so (exp/libpbftv_<v>.so; "base" = the
# in-tree library) with bench.py --no-extras.  On the GPU box:
#   bash tools/exp_variants.sh base w3 w4
set -euo pipefail
mkdir -p gpurun_out/exp
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L=$PWD/exp/libpbftv_$v.so; fi
  PBFTV_LIB=$L timeout -k 10 120 python bench.py --no-extras --steps 10 > gpurun_out/exp/$v.json 2>&1
done
