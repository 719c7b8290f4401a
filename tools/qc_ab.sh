#!/bin/bash
# Same-box A/B of the latency path: alternates the in-tree library ("base") with
# experiment builds exp/libpbftv_<v>.so, R rounds each (tools/qc_ab.py).
#   bash tools/qc_ab.sh R v1 [v2 ...]     -> gpurun_out/qcab/<v>_<round>.json
set -euo pipefail
R=$1; shift
mkdir -p gpurun_out/qcab
for r in $(seq 1 "$R"); do
  for v in base "$@"; do
    L=""; [ "$v" = base ] || L=$PWD/exp/libpbftv_$v.so
    PBFTV_LIB=$L timeout -k 10 120 python tools/qc_ab.py > "gpurun_out/qcab/${v}_$r.json"
  done
done
