"""Host-buffer verify at 1M signatures (config 4) for the pipeline's full chunk
size (PBFTV_HOST_CHUNK is read per call): pinned and pageable
inputs, best of 5.  One JSON line per setting; tools/ for DESIGN.md."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

pub, H, S, K, ok = synth.config4(1 << 20, n_keys=100)
ver = Verifier()
ver.register_keys(pub)
pins = [ver.pinned(a) for a in (H, S, K)]
VARIANTS = [  # (full chunk, last chunk, PBFTV_HOST_KEYS_FIRST, PBFTV_HOST_2COMPUTE)
    (262144, 65536, 0, 0), (262144, 65536, 1, 0), (262144, 65536, 1, 1), (262144, 32768, 1, 1),
    (262144, 131072, 1, 1), (131072, 65536, 1, 1)]
for rnd in range(2):
    for chunk, last, kf, two in VARIANTS:
        os.environ["PBFTV_HOST_CHUNK"] = str(chunk)
        os.environ["PBFTV_HOST_LAST"] = str(last)
        os.environ["PBFTV_HOST_KEYS_FIRST"] = str(kf)
        os.environ["PBFTV_HOST_2COMPUTE"] = str(two)
        r = {"round": rnd, "chunk": chunk, "last": last, "keys_first": kf, "two_compute": two}
        for label, arrays in (("pinned", tuple(p.a for p in pins)), ("pageable", (H, S, K))):
            got = ver.verify_batch(*arrays)
            ts = []
            for _ in range(7):
                t0 = time.perf_counter()
                ver.verify_batch(*arrays)
                ts.append(time.perf_counter() - t0)
            r[label + "_ms"] = round(min(ts) * 1e3, 3)
            r[label + "_check"] = bool((got == ok).all())
        print(json.dumps(r), flush=True)
