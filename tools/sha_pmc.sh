#!/bin/bash
# SHA-256 memory counters (config-5 workload, tools/pmc_workload.py sha), one
# TCC group per pass: what the L2 asks the fabric for, by request size, and
# its hit/miss counts -- to calibrate FETCH_SIZE for the lane-per-message
# pattern before reading it as over-fetch.  Also lists the TCC counters.
set -o pipefail
OUT=${1:-gpurun_out/sha_pmc}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
pass() {
  local name=$1; shift
  PBFTV_SHA_LDS_PAD=${PAD:-0} timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/$name" -o run --pmc "$@" \
    -- python3 "$ROOT/tools/pmc_workload.py" sha > "$ROOT/$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -5 "$ROOT/$OUT/$name.log"; return 1; }
}
pass req TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum || exit 1
pass size TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum || exit 1
pass hit TCC_HIT_sum TCC_MISS_sum || exit 1
pass dram TCC_EA0_RDREQ_DRAM_sum || exit 1
echo ok
