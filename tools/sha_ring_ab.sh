#!/bin/bash
# k_sha256_ring (line-aligned LDS staging) vs k_sha256 (dword windows): SHA
# parity tests on the ring kernel, then per variant (PBFTV_SHA_RING=1 / 0) the
# config-5 and PBFT-digest timings (bench.py --sha-only, alternating, 2 rounds)
# and the fabric read requests per launch (one PMC pass each).
set -o pipefail
OUT=${1:-gpurun_out/sha_ring}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "sha256 or digest or config5 or flush or gojson" \
  > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for r in 1 2; do
  for v in 1 0; do
    PBFTV_SHA_RING=$v timeout -k 10 200 python3 bench.py --sha-only > "$OUT/bench_${v}_$r.json" 2> "$OUT/bench_${v}_$r.err" || { echo "bench $v failed"; tail "$OUT/bench_${v}_$r.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); c=d['config5']; p=d['pbft_digests']; print('ring=$v', 'config5 kernel_ms', round(c['kernel_ms'],4), 'frac', round(c['roofline']['frac'],4), 'check', c['check'], '| pbft', round(p['kernel_ms'],4), p['check'])"
  done
done
for v in 1 0; do
  (cd /tmp && PBFTV_SHA_RING=$v timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/req_$v" -o run --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum -- python3 "$ROOT/tools/pmc_workload.py" sha > "$ROOT/$OUT/req_$v.log" 2>&1) || { echo "pmc $v failed"; tail "$OUT/req_$v.log"; exit 1; }
  python3 - "$OUT/req_$v/run_counter_collection.csv" $v <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "sha256" in r["Kernel_Name"]:
        v[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("ring=" + sys.argv[2], {k: round(sum(x) / len(x) / 1e6, 3) for k, x in v.items()}, "M requests per launch")
PY
done
