"""Where the 1-s tick's extra QC time goes: bench.qc_latency for a 3-vote
certificate back to back and at the reference's 1-s cadence, with the GPU's
serve stamps (PBFTV_QC_STAMPS=1), on the GPU's NUMA node.  One JSON line per
cadence."""
import json
import os
import sys

os.environ["PBFTV_QC_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

print(json.dumps(bench.pin_to_gpu_node(0)), flush=True)
ver = Verifier()
keep = ("p50", "p90", "min", "in_library_us_p50", "in_library_handover_us_p50", "in_library_to_lock_us_p50",
        "in_library_slots_in_us_p50", "gpu_serve_us_p50", "gpu_sclk_mhz_p50", "armed_frac")
if os.environ.get("TICK_ONE_CORE") == "1":
    # the keeper thread first (it inherits the creating thread's mask), then
    # this thread alone on one core of the GPU's node
    bench.qc_latency(ver, 4, 3, 20, 22)
    core = min(os.sched_getaffinity(0))
    os.sched_setaffinity(0, {core})
    print(json.dumps({"one_core": core}), flush=True)
for gap, calls in ((0.0, 2000), (1.0, 40), (0.1, 100)):
    r = bench.qc_latency(ver, 4, 3, calls, 21, gap_s=gap, warm=3 if gap else 20)
    print(json.dumps({"gap_s": gap, **{k: r.get(k) for k in keep}}), flush=True)
ver.close()
