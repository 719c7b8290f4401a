"""Same-box A/B of the latency path: p50 of pbftv_qc_verify (one n = 4
certificate of 3 signatures, pre-marshalled call) for the library given by
PBFTV_LIB.  tools/ab.sh (workload qc) alternates builds.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402
import bench  # noqa: E402
from simple_pbft_amd.pbftv import K_ECDSA_WAVE  # noqa: E402

pin = bench.pin_to_gpu_node(0)  # as bench.py: the 67-vote p50 follows the caller's socket
ver = Verifier()
out = {"lib": os.environ.get("PBFTV_LIB") or "base", "affinity": pin}
for n_keys, sigs in ((4, 3), (100, 67)):
    pub, H, S, K = synth.qc(n_keys, sigs, 5)
    ver.register_keys(pub)
    call = ver.qc_verify_prepared(H, S, K, quorum=sigs)
    for _ in range(50):
        call()
    ts = []
    for _ in range(1500):
        t0 = time.perf_counter()
        acc, ok = call()
        ts.append(time.perf_counter() - t0)
        assert ok and acc == sigs
    ver.set_kernel_timing(True)
    ver.reset_kernel_times()
    for _ in range(300):
        call()
    ms, cnt = ver.kernel_time_ms(0, K_ECDSA_WAVE)
    ver.set_kernel_timing(False)
    # (launched kernels only: an armed serve records no event)
    out[f"{sigs}sigs"] = {"p50_us": float(np.percentile(ts, 50) * 1e6), "p90_us": float(np.percentile(ts, 90) * 1e6),
                          "kernel_us": ms * 1e3 / cnt if cnt else None}
print(json.dumps(out))
