"""bench.qc_under_load alone (QC p50 idle and beside a 1M stream, per
certificate size, and the stream's rate alone and meanwhile), one JSON line:
the same-box A/B driver for the armed kernel's CU options.

    PBFTV_QC_EXCLUSIVE_CU=0|narrow|1 python tools/qc_load_ab.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

n = 1 << 20
pub, H, S, K, ok = synth.config4(n, n_keys=100, seed=0x50424654)
pin = bench.pin_to_gpu_node(0)  # as bench.py
ver = Verifier(device_mask=1)
ver.register_keys(pub)
dh, ds, dk = ver.to_device(0, H), ver.to_device(0, S), ver.to_device(0, K)
out = bench.qc_under_load(ver, dh, ds, dk, n, ok, seed=0x50424654)
out["env"] = {k: v for k, v in os.environ.items() if k.startswith("PBFTV_QC")}
for b in (dh, ds, dk):
    b.free()
ver.close()
print(json.dumps(out))
