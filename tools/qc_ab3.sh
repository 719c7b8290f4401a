#!/bin/bash
# QC p50 (tools/qc_fresh.py) for the in-tree library and experiment builds, alternating:
#   bash tools/qc_ab3.sh OUT ROUNDS v1 [v2 ...]   (v = exp/libpbftv_<v>.so, "base" = in-tree)
set -o pipefail
OUT=$1; R=$2; shift 2
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for v in base "$@"; do
    L=""; [ "$v" = base ] || L=$PWD/exp/libpbftv_$v.so
    PBFTV_LIB=$L timeout -k 10 200 python -u tools/qc_fresh.py 3000 > "$OUT/${v}_$r.json" || { echo "qc $v failed"; exit 1; }
    echo "$v $(cut -c1-150 "$OUT/${v}_$r.json")"
  done
done
