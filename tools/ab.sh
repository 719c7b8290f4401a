#!/bin/bash
# A/B timing on one GPU box: alternates the in-tree library ("base") with
# experiment builds exp/libpbftv_<v>.so, R rounds each (bench.py --no-extras).
#   bash tools/ab.sh R v1 [v2 ...]     -> gpurun_out/ab/<v>_<round>.json
set -euo pipefail
R=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 "$R"); do
  for v in base "$@"; do
    # v = a library exp/libpbftv_<v>.so, or env:NAME=VALUE[,NAME=VALUE...] (same library, variables set)
    L=""; E=""
    case "$v" in
      base) ;;
      env:*) E=${v#env:}; E=${E//,/ } ;;
      *) L=$PWD/exp/libpbftv_$v.so ;;
    esac
    env PBFTV_LIB=$L $E timeout -k 10 120 python bench.py --no-extras --steps 20 > "gpurun_out/ab/${v//[:=,]/_}_$r.json" 2>&1
  done
done
