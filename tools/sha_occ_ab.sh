#!/bin/bash
# SHA-256 L2-footprint A/B: blocks per CU capped by dynamic LDS padding
# (PBFTV_SHA_LDS_PAD), time (bench.py --sha-only) and FETCH_SIZE per variant.
set -o pipefail
OUT=${1:-gpurun_out/sha_occ}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
for pad in 0 49152 65536; do
  PBFTV_SHA_LDS_PAD=$pad timeout -k 10 200 python3 bench.py --sha-only > "$OUT/bench_$pad.json" 2> "$OUT/bench_$pad.err" || { echo "bench $pad failed"; tail "$OUT/bench_$pad.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$pad.json')); c=d['config5']; print('pad $pad', 'ms', round(c['ms'],3), 'kernel_ms', round(c['kernel_ms'],3), 'frac', round(c['roofline']['frac'],3))"
  (cd /tmp && PBFTV_SHA_LDS_PAD=$pad timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/fetch_$pad" -o run --pmc FETCH_SIZE -- python3 "$ROOT/tools/pmc_workload.py" sha > "$ROOT/$OUT/fetch_$pad.log" 2>&1) || { echo "pmc $pad failed"; tail "$OUT/fetch_$pad.log"; exit 1; }
done
