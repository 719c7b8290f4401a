#!/bin/bash
# Strong-scaling shard sizes x stream overlap, same box, interleaved rounds:
#   bash tools/streams_ab.sh OUT ROUNDS "N STREAMS [ENV=V ...]" ...  -> OUT/summary.txt
set -euo pipefail
OUT=$1; ROUNDS=$2; shift 2
VARIANTS=("$@")
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for v in "${VARIANTS[@]}"; do
    set -- $v
    N=$1; S=$2; shift 2
    f="$OUT/r${r}_${i}.json"
    env "$@" timeout -k 10 150 python bench.py --no-extras --n "$N" --streams "$S" --steps 50 > "$f" 2> "$OUT/r${r}_${i}.err"
    python3 - "$f" "$v" >> "$OUT/summary.txt" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(f"{sys.argv[2]:<40} {d['value']/1e6:8.1f} M/s  step {d['ms_per_step']:.4f} ms  comb {k['ecdsa_comb']['avg_ms']:.4f}"
      f"  scal {k['ecdsa_scalars']['avg_ms']:.4f}  {d['check']}")
PY
    i=$((i + 1))
  done
done
cat "$OUT/summary.txt"
