"""Three host-buffer verifies of the config-4 batch (pinned inputs) for a
rocprofv3 --kernel-trace --memory-copy-trace timeline of the chunk pipeline;
with an argument C, C caller threads doing three verifies each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

pub, H, S, K, ok = synth.config4(1 << 20, n_keys=100)
ver = Verifier()
ver.register_keys(pub)
pins = [ver.pinned(a) for a in (H, S, K)]
callers = int(sys.argv[1]) if len(sys.argv) > 1 else 1
res = []


import time
t00 = time.perf_counter()
stamps = []


def run():
    for _ in range(3):
        t = time.perf_counter()
        got = ver.verify_batch(*(p.a for p in pins))
        stamps.append((round((t - t00) * 1e3, 3), round((time.perf_counter() - t00) * 1e3, 3)))
    res.append(bool((got == ok).all()))


if callers == 1:
    run()
else:
    import threading
    th = [threading.Thread(target=run) for _ in range(callers)]
    for x in th:
        x.start()
    for x in th:
        x.join()
assert all(res) and len(res) == callers
print("call start/end ms:", sorted(stamps))
