#!/bin/bash
# Small per-GPU batches (the strong-scaling shards of config 4: 1M / 8 = 131072,
# 1M / 4 = 262144): bench.py --no-extras --n N under env variants, same box.
#   bash tools/small_n_ab.sh OUT "N ENV=V ..." ...   -> OUT/<i>.json
set -euo pipefail
OUT=$1; shift
mkdir -p "$OUT"
i=0
for v in "$@"; do
  set -- $v
  N=$1; shift
  echo "$v" > "$OUT/$i.variant"
  env "$@" timeout -k 10 150 python bench.py --no-extras --n "$N" --steps 50 > "$OUT/$i.json" 2> "$OUT/$i.err"
  i=$((i + 1))
done
