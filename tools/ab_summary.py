"""Summarise tools/ab.sh output: per variant, comb/scalar kernel ms and value (median over rounds)."""
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
res = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    v = os.path.basename(f).rsplit("_", 1)[0]
    try:
        j = json.load(open(f))
    except Exception:
        print(v, "FAILED", open(f).read()[-300:])
        continue
    res[v].append((j["value"] / 1e6, j["kernels"]["ecdsa_comb"]["avg_ms"], j["kernels"]["ecdsa_scalars"]["avg_ms"], j["check"]))
for v, rs in res.items():
    print(f"{v:12s} Mverif/s {statistics.median(r[0] for r in rs):7.1f}  comb {statistics.median(r[1] for r in rs):.4f} ms"
          f"  scalars {statistics.median(r[2] for r in rs):.4f} ms  checks {[r[3] for r in rs]}")
