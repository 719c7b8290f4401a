#!/bin/bash
# Same-box A/B of the latency path at the reference's cadence: the in-tree
# library against exp/libpbftv_<v>.so, tools/qc_cadence.py --parts tick,
# R alternating rounds.   bash tools/qc_tick_ab.sh OUT R v
set -euo pipefail
OUT=$1; R=$2; V=$3
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for v in base "$V"; do
    L=""; [ "$v" = base ] || L=$PWD/exp/libpbftv_$v.so
    PBFTV_LIB=$L timeout -k 10 200 python -u tools/qc_cadence.py --parts tick > "$OUT/${v}_$r.jsonl" 2> "$OUT/${v}_$r.err"
  done
done
