"""What an armed latency kernel that serves nothing costs a concurrent batch
stream: the 1M stream's rate with nothing armed, then with the keeper holding
an armed kernel (one certificate call arms it; no call during the timing), in
alternating segments.  One JSON line; knobs from the environment
(PBFTV_QC_ARM_MS, PBFTV_QC_SPIN, PBFTV_QC_EXCLUSIVE_CU, PBFTV_QC_WIDE)."""
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

n = 1 << 20
pub, H, S, K, ok = synth.config4(n, n_keys=100, seed=0x50424654)
_, h3, s3, k3 = synth.certs(100, 3, 64, 0x50424654)
ver = Verifier(device_mask=1)
ver.register_keys(pub)
dh, ds, dk = ver.to_device(0, H), ver.to_device(0, S), ver.to_device(0, K)
st = ver.stream_create(0)
db = ver.alloc(0, n // 8 + 1)


def rate(seconds):
    stop = threading.Event()
    done = [0]

    def run():
        while not stop.is_set():
            ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr, stream=st)
            ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr, stream=st)
            ver.stream_wait(0, st)
            done[0] += 2
    th = threading.Thread(target=run)
    th.start()
    time.sleep(0.05)
    t0, b0 = time.perf_counter(), done[0]
    time.sleep(seconds)
    r = (done[0] - b0) * n / (time.perf_counter() - t0)
    stop.set()
    th.join()
    return r


out = {"env": {k: v for k, v in os.environ.items() if k.startswith("PBFTV_QC")}, "alone": [], "armed": []}
os.environ["PBFTV_QC_KEEP_MS"] = "2500"  # the keeper holds it for 2.5 s after a call, then nothing is armed
for seg in range(3):
    time.sleep(3.0)  # the previous arming ran out
    out["alone"].append(rate(0.5))
    assert ver.qc_verify(h3[3 * seg:3 * seg + 3], s3[3 * seg:3 * seg + 3], k3[3 * seg:3 * seg + 3], 3)[2]
    out["armed"].append(rate(0.5))
out["ratio"] = float(np.mean(out["armed"]) / np.mean(out["alone"]))
out["check"] = bool((np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool) == ok).all())
print(json.dumps(out))
