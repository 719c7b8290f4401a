#!/bin/bash
# Same-box A/B of experiment builds exp/libpbftv_<v>.so ("base" = in-tree) at
# several batch sizes, R alternating rounds:
#   bash tools/lib_ab.sh OUT R "N1 N2" v1 [v2 ...]   -> OUT/<v>_<N>_<round>.json
set -euo pipefail
OUT=$1; R=$2; NS=$3; shift 3
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for n in $NS; do
    for v in base "$@"; do
      L=""; [ "$v" = base ] || L=$PWD/exp/libpbftv_$v.so
      PBFTV_LIB=$L timeout -k 10 150 python bench.py --no-extras --n "$n" --steps 30 > "$OUT/${v}_${n}_$r.json" 2> "$OUT/${v}_${n}_$r.err"
    done
  done
done
