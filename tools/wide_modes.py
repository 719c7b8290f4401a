"""The 67-vote certificate's p50 over several fresh contexts in one process
(each context allocates its own mailbox, relay word and tables): whether
the slow runs (~36 vs ~31 us across tools/ab.sh rounds) follow an
allocation.  Prints one JSON line per context."""
import json
import os
import sys
import time

import ctypes

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

pub, H, S, K = synth.qc(100, 67, 5)
pub4, H4, S4, K4 = synth.qc(4, 3, 5)
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    ver = Verifier()
    ver.register_keys(pub)
    call = ver.qc_verify_prepared(H, S, K, quorum=67)
    for _ in range(50):
        call()
    ts = []
    for _ in range(600):
        t0 = time.perf_counter()
        acc, ok = call()
        ts.append(time.perf_counter() - t0)
        assert ok and acc == 67
    call4 = None
    ver4 = Verifier()
    ver4.register_keys(pub4)
    call4 = ver4.qc_verify_prepared(H4, S4, K4, quorum=3)
    for _ in range(50):
        call4()
    t4 = []
    for _ in range(600):
        t0 = time.perf_counter()
        acc, ok = call4()
        t4.append(time.perf_counter() - t0)
        assert ok and acc == 3
    ver4.close()
    c = ver.qc_counters(0)
    print(json.dumps({"context": it, "cpu": ctypes.CDLL(None).sched_getcpu(), "p50_us": float(np.percentile(ts, 50) * 1e6),
                      "p50_3sigs_us": float(np.percentile(t4, 50) * 1e6),
                      "p10_us": float(np.percentile(ts, 10) * 1e6), "p90_us": float(np.percentile(ts, 90) * 1e6),
                      "armed_frac": c["armed"] / max(c["calls"], 1), "armed_waves": c["armed_waves"],
                      "rotations": c["rotations"]}), flush=True)
    ver.close()
