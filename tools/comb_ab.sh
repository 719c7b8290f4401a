#!/bin/bash
# Comb change check on the GPU box: the comb/geometry parity tests, then a
# same-box A/B of the in-tree library against exp/libpbftv_<v>.so at 1M and
# 131k (R alternating rounds), then one PMC pass each.
#   bash tools/comb_ab.sh OUT R v
set -euo pipefail
OUT=$1; R=$2; V=$3
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_geometry.py tests/test_gpu_parity.py tests/test_gpu_configs.py \
  > "$OUT/tests.log" 2>&1
bash tools/lib_ab.sh "$OUT/ab" "$R" "1048576 131072" "$V"
bash tools/pmc_ab.sh "$OUT/pmc" "$V"
