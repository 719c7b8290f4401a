"""What a resident latency server costs a concurrent batch stream, by server
shape: the 1M device-resident stream's rate with nothing
armed, and with the keeper holding each kind of armed kernel while no
certificate arrives -- the row schedule's narrow kernel at 4 and at 1 slot,
its wide kernel (72 workgroups, after 67-vote certificates), the quad
schedule's narrow kernel (PBFTV_QC_ROWS=0) -- in alternating rounds, at
the full batch (1,048,576: exactly 4 comb blocks per slot of every CU) and
at batches a little smaller, whose last comb round is partial anyway.  Also
the batch cost of the policy knobs (PBFTV_QC_YIELD).

    python tools/armed_tax.py [--rounds 2] [--seconds 0.4]

One JSON line.  Measurement tool (not product)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=0.4)
    ap.add_argument("--sizes", default="1048576,1032192,983040")
    ap.add_argument("--streams", type=int, default=2,
                    help="2: four batches alternating over two library streams per sync (bench.py's step); "
                         "1: two batches on one stream per sync (bench.py qc_under_load's stream)")
    ap.add_argument("--arm-ms", default="200", help="PBFTV_QC_ARM_MS (the keeper rotates every half of it)")
    ap.add_argument("--configs", default="none,rows_narrow_4,rows_narrow_1,rows_wide,quad_narrow")
    a = ap.parse_args()
    os.environ["PBFTV_QC_KEEP_MS"] = str(max(1200, 3 * int(a.arm_ms)))  # the keeper drops the server after this
    os.environ["PBFTV_QC_ARM_MS"] = a.arm_ms
    import synth  # noqa: E402
    from simple_pbft_amd import Verifier  # noqa: E402
    n = 1 << 20
    pub, H, S, K, ok = synth.config4(n, n_keys=100, seed=0x50424654)
    _, h3, s3, k3 = synth.certs(100, 3, 200, 0x50424654)
    _, h67, s67, k67 = synth.certs(100, 67, 20, 0x50424654)
    ver = Verifier(device_mask=1)
    ver.register_keys(pub)
    dh, ds, dk = ver.to_device(0, H), ver.to_device(0, S), ver.to_device(0, K)
    sts = [ver.stream_create(0) for _ in range(2)]
    dbs = [ver.alloc(0, n // 8 + 1) for _ in range(2)]
    sizes = [int(x) for x in a.sizes.split(",")]
    cert = [0]

    def qc(kind):
        c = cert[0]
        cert[0] += 1
        if kind == 67:
            i = c % 20
            sl = slice(67 * i, 67 * i + 67)
            return ver.qc_verify(h67[sl], s67[sl], k67[sl], 67)
        i = c % 200
        sl = slice(3 * i, 3 * i + 3)
        return ver.qc_verify(h3[sl], s3[sl], k3[sl], 3)

    def rate(m, seconds):
        """m-signature batches alternating over two library streams (bench.py's step)"""
        stop = threading.Event()
        done = [0]

        def run():
            j = 0
            per = 4 if a.streams == 2 else 2
            while not stop.is_set():
                for _ in range(per):
                    k = j & 1 if a.streams == 2 else 0
                    ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, m, dbs[k].ptr, stream=sts[k])
                    j += 1
                for st in sts:
                    ver.stream_wait(0, st)
                done[0] += per
        th = threading.Thread(target=run)
        th.start()
        time.sleep(0.08)
        t0, b0 = time.perf_counter(), done[0]
        time.sleep(seconds)
        r = (done[0] - b0) * m / (time.perf_counter() - t0)
        stop.set()
        th.join()
        return r

    def set_env(kv):
        for k in ("PBFTV_QC_SLOTS", "PBFTV_QC_ROWS", "PBFTV_QC_WIDE", "PBFTV_QC_YIELD"):
            os.environ.pop(k, None)
        os.environ.update(kv)

    def arm(cfg):
        """make the keeper hold the kernel of this configuration, then no call"""
        set_env(cfg["env"])
        time.sleep(int(os.environ["PBFTV_QC_KEEP_MS"]) * 1e-3 + 2 * int(a.arm_ms) * 1e-3 + 0.2)  # the last arming ran out
        if cfg["cert"] == 0:
            return {}
        for _ in range(3):
            qc(cfg["cert"])
        c = ver.qc_counters(0)
        return {"armed_waves": c["armed_waves"], "armed_wide": c["armed_wide"]}

    configs = [
        {"name": "none", "env": {}, "cert": 0},
        {"name": "rows_narrow_4", "env": {"PBFTV_QC_SLOTS": "4", "PBFTV_QC_WIDE": "0"}, "cert": 3},
        {"name": "rows_narrow_1", "env": {"PBFTV_QC_SLOTS": "1", "PBFTV_QC_WIDE": "0"}, "cert": 3},
        {"name": "rows_wide", "env": {}, "cert": 67},
        {"name": "quad_narrow", "env": {"PBFTV_QC_ROWS": "0", "PBFTV_QC_WIDE": "0"}, "cert": 3},
    ]
    want = a.configs.split(",")
    configs = [c for c in configs if c["name"] in want]
    res = {c["name"]: {str(m): [] for m in sizes} for c in configs}
    shape = {}
    rate(n, 0.3)  # warm
    for rnd in range(a.rounds):
        for cfg in configs:
            shape[cfg["name"]] = arm(cfg)
            for m in sizes:
                res[cfg["name"]][str(m)].append(rate(m, a.seconds))
            print(json.dumps({"round": rnd, "cfg": cfg["name"], "rates": {m: res[cfg["name"]][str(m)][-1]
                                                                           for m in map(str, sizes)}}),
                  file=sys.stderr, flush=True)
    out = {"rates": {k: {m: float(np.mean(v)) for m, v in d.items()} for k, d in res.items()}, "shape": shape,
           "streams": a.streams, "arm_ms": a.arm_ms}
    base = out["rates"]["none"]
    out["ratio_to_none"] = {k: {m: out["rates"][k][m] / base[m] for m in base} for k in out["rates"]}
    out["check"] = all(bool((np.unpackbits(db.to_host(), bitorder="little")[:sizes[-1]].astype(bool) ==
                             ok[:sizes[-1]]).all()) for db in dbs[:a.streams])
    print(json.dumps(out), flush=True)
    ver.close()


if __name__ == "__main__":
    main()
