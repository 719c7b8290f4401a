"""Pinned host memory on the GPU's NUMA node (PBFTV_HOST_NUMA, default on)
or where the runtime puts it (=0), for the caller's CPU as launched (taskset
by tools/wm_numa.sh): the host-buffer batch path at 1M (pinned and pageable
inputs, best of 5) and the 3- / 67-vote certificate p50, one fresh context per
setting and round.  One JSON line each."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

pub, H, S, K, ok = synth.config4(1 << 20, n_keys=100, seed=0x50424654)
q100 = synth.qc(100, 67, 5)
q4 = synth.qc(4, 3, 5)


def qc_p50(ver, q, sigs, reps=600):
    ver.register_keys(q[0])
    call = ver.qc_verify_prepared(q[1], q[2], q[3], quorum=sigs)
    for _ in range(50):
        call()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        acc, good = call()
        ts.append(time.perf_counter() - t0)
        assert good and acc == sigs
    return float(np.percentile(ts, 50) * 1e6)


for rnd in range(2):
    for setting in ("1", "0"):
        os.environ["PBFTV_HOST_NUMA"] = setting
        ver = Verifier()
        ver.register_keys(pub)
        hp = bench.host_path(ver, H, S, K, ok)
        out = {"round": rnd, "PBFTV_HOST_NUMA": setting, "cpu": ctypes.CDLL(None).sched_getcpu(),
               "host_pinned_Mps": hp["pinned"]["verifies_per_s"] / 1e6,
               "host_pageable_Mps": hp["pageable"]["verifies_per_s"] / 1e6,
               "checks": [hp["pinned"]["check"], hp["pageable"]["check"]],
               "qc67_p50_us": qc_p50(ver, q100, 67), "qc3_p50_us": qc_p50(ver, q4, 3)}
        ver.close()
        print(json.dumps(out), flush=True)
