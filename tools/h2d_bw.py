"""Raw host->device copy bandwidth through the library (pinned vs pageable, 100/25/6 MB): the PCIe ceiling of the host-buffer verify path."""
import time, numpy as np, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simple_pbft_amd import Verifier
v = Verifier()
n = 100 << 20
src = v.pinned(np.zeros(n, np.uint8))
pg = np.zeros(n, np.uint8)
dst = v.alloc(0, n)
for label, p in (("pinned", src.ptr), ("pageable", pg.ctypes.data)):
    for sz in (100 << 20, 25 << 20, 6 << 20):
        ts = []
        for _ in range(7):
            t0 = time.perf_counter(); v._L.pbftv_memcpy_h2d(v._h, 0, dst.ptr, p, sz); ts.append(time.perf_counter() - t0)
        print(label, sz >> 20, "MB", round(sz / min(ts) / 1e9, 1), "GB/s")
