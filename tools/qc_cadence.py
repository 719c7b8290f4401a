"""QC latency at the reference's call cadence, under load, and the CPU beside it.

    python tools/qc_cadence.py [--quick] [--parts a,b,...]

Parts (one JSON object per part on stdout, flushed as it completes):
  b2b      back-to-back fresh certificates (bench.py qc_latency), n4/3 and n100/67
  tick     fresh certificates with an idle gap before each: 1 s (the reference's
           alarm, pbft/network/node.go:44, :513-518), 100 ms, 10 ms
  free     hipFree / hipHostFree right after a latency-path call (does the armed
           kernel hold them?)
  load     QC p50 (2 ms gaps) with and without a 1M-signature stream running on
           another library stream of the same context
  host     host_path (pageable, pinned) with and without an armed kernel polling
  cpu      OpenSSL stand-in QC latency on 1 / 3 threads (3 sigs) and on the
           allotment (67 sigs)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

SEED4 = 0x50424654  # config 4's key set (synth.config4): QC certificates of the same committee


def pct(ts):
    a = np.asarray(ts) * 1e6
    return {"p50": float(np.percentile(a, 50)), "p90": float(np.percentile(a, 90)),
            "p99": float(np.percentile(a, 99)), "min": float(a.min()), "calls": len(a)}


def fresh_calls(ver, n_keys, sigs, count, seed, register=True):
    pub, H, S, K = synth.certs(n_keys, sigs, count, seed)
    if register:
        ver.register_keys(pub)
    return [ver.qc_verify_prepared(H[c * sigs:(c + 1) * sigs], S[c * sigs:(c + 1) * sigs],
                                   K[c * sigs:(c + 1) * sigs], quorum=sigs) for c in range(count)]


def timed_calls(calls, sigs, gap_s=0.0, ver=None, serve=None, clk=None):
    ts = []
    for call in calls:
        if gap_s:
            time.sleep(gap_s)
        t0 = time.perf_counter()
        acc, ok = call()
        ts.append(time.perf_counter() - t0)
        assert ok and acc == sigs, (acc, sigs)
        if serve is not None:  # the armed slot-0 wave's GPU serve time (PBFTV_QC_STAMPS=1)
            st = ver.qc_stamps(0)
            if "gpu_serve_us" in st:
                serve.append(st["gpu_serve_us"])
            if clk is not None and "sclk_mhz" in st:  # the mean shader clock over that serve
                clk.append(st["sclk_mhz"])
    return ts


def part_b2b(ver, quick):
    out = {}
    for nk, sg, cnt in ((4, 3, 2000 if quick else 10000), (100, 67, 500 if quick else 2000)):
        calls = fresh_calls(ver, nk, sg, cnt + 20, 11 + nk)
        timed_calls(calls[:20], sg)
        out[f"n{nk}_{sg}sigs"] = pct(timed_calls(calls[20:], sg))
    return out


def part_tick(ver, quick):
    """bench.qc_latency (the C caller loop) at idle gaps before every call."""
    out = {}
    plan = [(4, 3, 0.0, 2000), (4, 3, 1.0, 12 if quick else 30), (4, 3, 0.1, 30), (4, 3, 0.01, 100),
            (100, 67, 0.0, 500), (100, 67, 1.0, 8 if quick else 20)]
    reg = None
    for nk, sg, gap, cnt in plan:
        out[f"n{nk}_{sg}sigs_gap{int(gap * 1000)}ms"] = bench.qc_latency(ver, nk, sg, cnt, 101 + nk, gap_s=gap,
                                                                          warm=3, register=(reg != nk))
        reg = nk
    return out


def part_stamps(ver, quick):
    """Where the time goes after an idle gap (pbftv_qc_stamps per call): host
    hand-over, total, and for armed serves the GPU's serve time and shader clock."""
    out = {}
    calls = fresh_calls(ver, 4, 3, 400, 203)
    timed_calls(calls[:5], 3)
    i = 5
    for gap, cnt in ((0.0, 150), (0.002, 50), (0.01, 50), (0.1, 30), (1.0, 10 if quick else 20)):
        rows = []
        for call in calls[i:i + cnt]:
            if gap:
                time.sleep(gap)
            t0 = time.perf_counter()
            acc, ok = call()
            t = time.perf_counter() - t0
            assert ok and acc == 3
            st = ver.qc_stamps(0)
            st["wall_us"] = t * 1e6
            rows.append(st)
        i += cnt
        agg = {"armed_frac": float(np.mean([r["armed"] for r in rows]))}
        for k in ("wall_us", "total_us", "handover_us", "gpu_serve_us", "sclk_mhz"):
            v = [r[k] for r in rows if k in r]
            if v:
                agg[k + "_p50"] = float(np.median(v))
        out[f"gap{int(gap * 1000)}ms"] = agg
    return out


def part_wide(ver, quick):
    """Where a 67-signature certificate's time goes on the wide armed kernel
    (pbftv_qc_stamps_all): helper start and finish relative to slot 0 seeing
    the request, GPU wall-clock us."""
    calls = fresh_calls(ver, 100, 67, 120, 307)
    timed_calls(calls[:20], 67)
    rows = []
    for call in calls[20:]:
        t0 = time.perf_counter()
        acc, ok = call()
        wall = (time.perf_counter() - t0) * 1e6
        st = ver.qc_stamps_all(67).astype(np.int64)
        s0 = ver.qc_stamps(0)
        if not s0["armed"] or st[0, 0] == 0:
            continue
        khz = 100000.0
        rel_seen = (st[:, 0] - st[0, 0]) / khz * 1e3
        rel_done = (st[:, 2] - st[0, 0]) / khz * 1e3
        dur = (st[:, 2] - st[:, 0]) / khz * 1e3
        rows.append({"wall": wall, "lib": s0["total_us"], "lib_slots_in": s0["slots_in_us"],
                     "lib_handover": s0["handover_us"], "slot_seen_max": float(rel_seen[:8].max()),
                     "helper_seen_med": float(np.median(rel_seen[8:])), "helper_seen_max": float(rel_seen[8:].max()),
                     "slot_done_max": float(rel_done[:8].max()), "helper_done_max": float(rel_done[8:].max()),
                     "slot_dur_med": float(np.median(dur[:8])), "helper_dur_med": float(np.median(dur[8:])),
                     "helper_dur_max": float(dur[8:].max())})
    out = {"calls": len(rows)}
    for k in (rows[0].keys() if rows else []):
        out[k + "_p50"] = float(np.median([r[k] for r in rows]))
    return out


def part_free(ver, quick):
    calls = fresh_calls(ver, 4, 3, 8, 7)
    res = {}
    for label in ("dev_free", "host_free"):
        timed_calls(calls[:2], 3)
        if label == "dev_free":
            b = ver.alloc(0, 1 << 20)
            t0 = time.perf_counter()
            b.free()
        else:
            p = ver.pinned(np.zeros(1 << 20, np.uint8))
            t0 = time.perf_counter()
            p.free()
        res[label + "_ms_after_qc"] = (time.perf_counter() - t0) * 1e3
    return res


def part_load(ver, quick):
    n = 1 << 20
    pub, H, S, K, ok = synth.config4(n, n_keys=100, seed=SEED4)
    ver.register_keys(pub)
    calls = fresh_calls(ver, 100, 3, 620, SEED4, register=False)  # the config-4 committee's keys
    calls67 = fresh_calls(ver, 100, 67, 220, SEED4, register=False)
    dh, ds, dk = ver.to_device(0, H), ver.to_device(0, S), ver.to_device(0, K)
    st = ver.stream_create(0)
    db = ver.alloc(0, n // 8 + 1)
    out = {}
    timed_calls(calls[:20], 3)
    si3, si67, ci3, cv3 = [], [], [], []
    out["idle_3sigs_gap2ms"] = pct(timed_calls(calls[20:320], 3, 0.002, ver, si3, ci3))
    timed_calls(calls67[:10], 67)
    out["idle_67sigs_gap2ms"] = pct(timed_calls(calls67[10:110], 67, 0.002, ver, si67))
    out["idle_gpu_serve_us_p50"] = {"3sigs": float(np.median(si3)) if si3 else None,
                                    "67sigs": float(np.median(si67)) if si67 else None}
    stop = threading.Event()
    done = [0]

    def stream():
        while not stop.is_set():
            ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr, stream=st)
            ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr, stream=st)
            ver.stream_wait(0, st)
            done[0] += 2
    th = threading.Thread(target=stream)
    th.start()
    time.sleep(0.05)
    t0 = time.perf_counter()
    sv3, sv67 = [], []
    out["loaded_3sigs_gap2ms"] = pct(timed_calls(calls[320:620], 3, 0.002, ver, sv3, cv3))
    out["loaded_67sigs_gap2ms"] = pct(timed_calls(calls67[110:220], 67, 0.002, ver, sv67))
    out["loaded_gpu_serve_us_p50"] = {"3sigs": float(np.median(sv3)) if sv3 else None,
                                      "67sigs": float(np.median(sv67)) if sv67 else None}
    # serve time = cycles / clock: how much of the loaded penalty is the clock
    if si3 and sv3 and ci3 and cv3:
        ki, kl = float(np.median(ci3)), float(np.median(cv3))
        out["sclk_mhz_p50_3sigs"] = {"idle": ki, "loaded": kl}
        out["serve_kcycles_p50_3sigs"] = {"idle": float(np.median(si3)) * ki * 1e-3,
                                          "loaded": float(np.median(sv3)) * kl * 1e-3}
    dt = time.perf_counter() - t0
    b0 = done[0]
    stop.set()
    th.join()
    out["stream_batches_during"] = b0
    out["stream_verifies_per_s_during"] = b0 * n / dt
    got = np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool)
    out["stream_check"] = bool((got == ok).all())
    # the stream alone, same loop
    t0 = time.perf_counter()
    for _ in range(20):
        ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr, stream=st)
    ver.stream_wait(0, st)
    out["stream_alone_verifies_per_s"] = 20 * n / (time.perf_counter() - t0)
    for b in (dh, ds, dk, db):
        b.free()
    ver.stream_destroy(0, st)
    return out


def part_host(ver, quick):
    n = 1 << 20
    pub, H, S, K, ok = synth.config4(n, n_keys=100, seed=SEED4)
    ver.register_keys(pub)
    calls = fresh_calls(ver, 100, 3, 40, SEED4, register=False)
    out = {}
    for label, arm in (("no_armed_kernel", "0"), ("armed_kernel_polling", "1")):
        os.environ["PBFTV_QC_ARM"] = arm
        if arm == "0":
            timed_calls(calls[:2], 3)  # a launched call: nothing stays armed
        res = {}
        for kind in ("pageable", "pinned"):
            pins = None
            arrays = (H, S, K)
            if kind == "pinned":
                pins = [ver.pinned(a) for a in (H, S, K)]
                arrays = tuple(p.a for p in pins)
            best = 1e9
            for _ in range(5):
                if arm == "1":
                    timed_calls(calls[2:4], 3)  # arms the next kernel (500 ms budget): polling during the batch
                t0 = time.perf_counter()
                got = ver.verify_batch(*arrays)
                best = min(best, time.perf_counter() - t0)
            res[kind] = {"verifies_per_s": n / best, "ms": best * 1e3, "check": bool((got == ok).all())}
            if pins:
                for p in pins:
                    p.free()
        out[label] = res
    os.environ.pop("PBFTV_QC_ARM", None)
    return out


def part_cpu(ver, quick):
    so = os.path.join(ROOT, "oracle", "libopenssl_standin.so")
    L = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    L.standin_qc_latency.restype = ctypes.c_int64
    L.standin_qc_latency.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_uint32, ctypes.c_int,
                                     ctypes.c_double, vp, vp]
    thr = bench.cpu_allotment()["threads"]
    out = {"allotment_threads": thr}
    for nk, sg, threads, cnt, gap in ((4, 3, 1, 400, 0.0), (4, 3, 3, 400, 0.0), (100, 67, thr, 200, 0.0),
                                      (100, 67, 1, 50, 0.0), (4, 3, 1, 12 if quick else 30, 1.0),
                                      (4, 3, 3, 12 if quick else 30, 1.0)):
        pub, H, S, K = synth.certs(nk, sg, cnt, 11 + nk)
        us = np.zeros(cnt)
        bm = np.zeros((cnt * sg + 7) // 8, np.uint8)
        acc = L.standin_qc_latency(H.ctypes.data, S.ctypes.data, K.ctypes.data, cnt, sg, pub.ctypes.data, len(pub),
                                   threads, gap * 1e6, us.ctypes.data, bm.ctypes.data)
        assert acc == cnt * sg
        out[f"n{nk}_{sg}sigs_{threads}thr_gap{int(gap * 1000)}ms"] = pct(us * 1e-6)
    return out


PARTS = {"wide": part_wide, "stamps": part_stamps, "b2b": part_b2b, "tick": part_tick, "free": part_free, "load": part_load, "host": part_host,
         "cpu": part_cpu}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--parts", default="cpu,b2b,free,tick,load,host")
    a = ap.parse_args()
    if os.environ.get("PBFTV_QC_STAMPS") is None and any(p in a.parts for p in ("wide", "stamps", "load")):
        os.environ["PBFTV_QC_STAMPS"] = "1"  # the armed kernels write their GPU timestamps (diagnostics)
    ver = Verifier(device_mask=1)
    for p in a.parts.split(","):
        t0 = time.perf_counter()
        r = PARTS[p](ver, a.quick)
        print(json.dumps({"part": p, "seconds": time.perf_counter() - t0,
                          "env": {k: v for k, v in os.environ.items() if k.startswith("PBFTV")}, **r}), flush=True)
    ver.close()


if __name__ == "__main__":
    main()
