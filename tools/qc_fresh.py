"""QC p50 on FRESH certificates (bench.py's qc_latency: a different
certificate every call, table entries cold) for n = 4 / 3 signatures and
n = 100 / 67, plus the same-certificate figure.  One JSON line.
    python tools/qc_fresh.py [calls]"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    ver = Verifier(device_mask=1)
    q4 = bench.qc_latency(ver, 4, 3, calls, 11)
    q100 = bench.qc_latency(ver, 100, 67, max(500, calls // 5), 12)
    out = {"p50_n4_3sigs": q4["p50"], "p99_n4_3sigs": q4["p99"], "p50_n100_67sigs": q100["p50"],
           "p99_n100_67sigs": q100["p99"], "n4": q4, "n100": q100,
           "table_config": ver.table_config()[:2], "env": {k: v for k, v in os.environ.items() if k.startswith("PBFTV")}}
    print(json.dumps(out), flush=True)
    ver.close()


if __name__ == "__main__":
    main()
