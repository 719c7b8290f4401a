#!/bin/bash
# SHA-256 kernel variants as library builds: SHA parity tests on the in-tree
# library, then config-5 / PBFT-digest timings (bench.py --sha-only) for the
# in-tree library ("base") and exp/libpbftv_<v>.so, R alternating rounds, then
# one PMC pass each (VALU busy, LDS stalls).
#   bash tools/sha_lib_ab.sh OUT R v1 [v2 ...]
set -o pipefail
OUT=$1; R=$2; shift 2
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "sha256 or digest or config5" \
  > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for r in $(seq 1 "$R"); do
  for v in base "$@"; do
    L=""; [ "$v" = base ] || L=$ROOT/exp/libpbftv_$v.so
    PBFTV_LIB=$L timeout -k 10 200 python3 bench.py --sha-only > "$OUT/${v}_$r.json" 2> "$OUT/${v}_$r.err" || { echo "bench $v failed"; tail "$OUT/${v}_$r.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_$r.json')); c=d['config5']; p=d['pbft_digests']; print('$v', 'config5 kernel_ms', round(c['kernel_ms'],4), 'frac', round(c['roofline']['frac'],4), 'check', c['check'], '| pbft', round(p['kernel_ms'],4), p['check'])"
  done
done
cd /tmp
for v in base "$@"; do
  L=""; [ "$v" = base ] || L=$ROOT/exp/libpbftv_$v.so
  PBFTV_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/pmc_$v" -o run \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    -- python3 "$ROOT/bench.py" --sha-only > "$ROOT/$OUT/pmc_$v.log" 2>&1 || { echo "pmc $v failed"; exit 1; }
done
