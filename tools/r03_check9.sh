#!/bin/bash
# fs_is_zero without the canonical subtract: ECDSA GPU parity (lane + wave
# paths, geometries, configs), same-box A/B against exp/libpbftv_old.so, one
# PMC VALU pass.
set -o pipefail
OUT=${1:-gpurun_out/r03c9}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_geometry.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
rm -rf gpurun_out/ab
timeout -k 10 900 bash tools/ab.sh 3 old || { echo "ab failed"; exit 1; }
python3 tools/ab_summary.py gpurun_out/ab
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/pmc/valu" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 "$ROOT/tools/pmc_workload.py" > "$ROOT/$OUT/pmc_valu.log" 2>&1 || { echo "pmc failed"; tail "$ROOT/$OUT/pmc_valu.log"; exit 1; }
cd "$ROOT" && python3 tools/pmc_summary.py "$OUT/pmc" 2>/dev/null | python3 -c "
import json,sys
j=json.load(sys.stdin)
for k in ('ecdsa_comb','ecdsa_wave','ecdsa_scalars'):
    v=j['kernels'].get(k)
    if v: print(k, 'valu/wave %.0f issue %.3f'%(v['valu_insts_per_wave'], v['valu_issue_frac']))
"
