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
    res[v].append((j["value"] / 1e6, {k: x["avg_ms"] for k, x in j["kernels"].items()}, j["check"]))
for v, rs in res.items():
    ks = {k: statistics.median(r[1][k] for r in rs) for k in rs[0][1]}
    print(f"{v:12s} Mverif/s {statistics.median(r[0] for r in rs):7.1f}  " +
          "  ".join(f"{k} {t:.4f} ms" for k, t in ks.items()) + f"  checks {[r[2] for r in rs]}")
