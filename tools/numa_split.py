"""Where a remote-socket caller's extra time goes (tools/wm_numa.sh runs it
on each NUMA node): bench.qc_latency for 3- and 67-vote certificates with
the GPU's serve stamps (PBFTV_QC_STAMPS=1) -- host time to the doorbell, the
GPU's serve time, and the rest (doorbell -> GPU sees it, verdict -> host).
One JSON line per size."""
import ctypes
import json
import os
import sys

os.environ["PBFTV_QC_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

ver = Verifier()
for keys, sigs in ((4, 3), (100, 67)):
    r = bench.qc_latency(ver, keys, sigs, 1000, 7)
    keep = ("p50", "in_library_us_p50", "in_library_handover_us_p50", "in_library_slots_in_us_p50",
            "gpu_serve_us_p50", "gpu_sclk_mhz_p50", "armed_frac")
    print(json.dumps({"sigs": sigs, "cpu": ctypes.CDLL(None).sched_getcpu(), **{k: r.get(k) for k in keep}}), flush=True)
ver.close()
