#!/bin/bash
# Same-box A/B of key registration (tools/reg_probe.py) for the in-tree library
# ("base") and experiment builds exp/libpbftv_<v>.so, R rounds each.
set -euo pipefail
R=$1; shift
mkdir -p gpurun_out/regab
for r in $(seq 1 "$R"); do
  for v in base "$@"; do
    L=""; [ "$v" = base ] || L=$PWD/exp/libpbftv_$v.so
    PBFTV_LIB=$L timeout -k 10 200 python tools/reg_probe.py > "gpurun_out/regab/${v}_$r.json"
  done
done
