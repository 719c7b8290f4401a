#!/bin/bash
# Same-box A/B on the GPU box: every VARIANT runs every WORKLOAD, in
# alternating rounds, each run a fresh process under its own time limit.
#
#   bash tools/ab.sh OUT ROUNDS WORKLOADS VARIANT [VARIANT ...]
#
# WORKLOADS: comma-separated, each one of
#   bench:N     bench.py --no-extras --n N --steps 30  (verifies/s, comb/scalar ms)
#   streams:N:S the same with --streams S
#   sha         bench.py --sha-only                      (config 5 + PBFT digests)
#   qc          tools/qc_ab.py      (QC p50, fresh certificates)
#   tick        tools/qc_cadence.py --parts tick        (QC at the reference's 1-s tick)
#   load        tools/qc_load_ab.py (QC p50 idle / beside a 1M stream, stream rates)
#   idle        tools/qc_idle_cost.py (the stream's rate with an armed kernel serving nothing)
#   reg         tools/reg_probe.py  (key registration phases)
#   pmc         one rocprofv3 --pmc pass (cycles, VALU) over tools/pmc_workload.py comb
# VARIANT: "base" (the in-tree library), or any "+"-joined mix of
#   lib:V              exp/libpbftv_V.so (an experiment build) instead of the in-tree library
#   env:A=1,B=2        environment variables for the run
# e.g.  bash tools/ab.sh gpurun_out/ab 3 bench:1048576,bench:131072 base lib:nt
#       bash tools/ab.sh gpurun_out/ab 2 load base env:PBFTV_QC_EXCLUSIVE_CU=0
# Output: OUT/<workload>__<variant>__<round>.json (+ .err); then a summary per
# workload and variant (tools/ab_summary.py OUT).  A run that fails or times
# out stops the script (no GPU step after a failure).
set -euo pipefail
OUT=$1; ROUNDS=$2; WORKLOADS=$3; shift 3
ROOT=$(pwd)
mkdir -p "$OUT"
run() {  # run WORKLOAD VARIANT FILE
  local w=$1 v=$2 f=$3 lib="" envs=() part
  for part in ${v//+/ }; do
    case "$part" in
      base) ;;
      lib:*) lib=$ROOT/exp/libpbftv_${part#lib:}.so ;;
      env:*) local e=${part#env:}; envs+=(${e//,/ }) ;;
      *) echo "bad variant part: $part" >&2; return 2 ;;
    esac
  done
  local cmd
  case "$w" in
    bench:*) cmd=(python3 bench.py --no-extras --n "${w#bench:}" --steps 30) ;;
    streams:*) local a=${w#streams:}; cmd=(python3 bench.py --no-extras --n "${a%%:*}" --streams "${a##*:}" --steps 50) ;;
    sha) cmd=(python3 bench.py --sha-only) ;;
    qc) cmd=(python3 tools/qc_ab.py) ;;
    tick) cmd=(python3 -u tools/qc_cadence.py --parts tick) ;;
    load) cmd=(python3 -u tools/qc_load_ab.py) ;;
    idle) cmd=(python3 -u tools/qc_idle_cost.py) ;;
    reg) cmd=(python3 tools/reg_probe.py) ;;
    pmc) (cd /tmp && env TMPDIR=/tmp PBFTV_LIB="$lib" "${envs[@]}" timeout -s KILL 240 rocprofv3 --kernel-trace \
            --output-format csv -d "$ROOT/${f%.json}" -o run \
            --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
            -- python3 "$ROOT/tools/pmc_workload.py" comb > "$ROOT/${f%.json}.log" 2>&1)
         return ;;
    *) echo "bad workload: $w" >&2; return 2 ;;
  esac
  env PBFTV_LIB="$lib" "${envs[@]}" timeout -k 10 300 "${cmd[@]}" > "$f" 2> "${f%.json}.err"
}
for r in $(seq 1 "$ROUNDS"); do
  for w in ${WORKLOADS//,/ }; do
    for v in "$@"; do
      f="$OUT/${w//:/-}__${v//[:=,+\/]/-}__$r.json"
      run "$w" "$v" "$f" || { echo "FAILED: $w $v round $r (see ${f%.json}.err)"; exit 1; }
    done
  done
done
python3 tools/ab_summary.py "$OUT"
