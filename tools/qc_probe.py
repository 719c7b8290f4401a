"""Where does quorum-certificate latency go?  Times, for a 3-sig and a 67-sig
certificate: pbftv_qc_verify end to end, the device-resident verify (+sync),
each kernel (HIP events), and a bare H2D+D2H round trip."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402
from simple_pbft_amd.pbftv import K_ECDSA_COMB, K_ECDSA_SCALARS, K_ECDSA_WAVE  # noqa: E402


def p50(f, iters=500):
    for _ in range(20):
        f()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.percentile(ts, 50) * 1e6)


def main():
    ver = Verifier()
    out = {}
    for n_keys, sigs in ((4, 3), (100, 67)):
        pub, H, S, K = synth.qc(n_keys, sigs, 5)
        ver.register_keys(pub)
        r = {"qc_verify_us": p50(lambda: ver.qc_verify(H, S, K, quorum=sigs)),
             "qc_verify_prepared_us": p50(ver.qc_verify_prepared(H, S, K, quorum=sigs))}
        dh, ds, dk = ver.to_device(0, H), ver.to_device(0, S), ver.to_device(0, K)
        db = ver.alloc(0, 64)

        def dev():
            ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, sigs, db.ptr)
            ver.sync(0)
        r["dev_verify_sync_us"] = p50(dev)
        small = ver.alloc(0, 4096)
        hb = np.zeros(4096, np.uint8)

        def rt():
            ver._L.pbftv_memcpy_h2d(ver._h, 0, small.ptr, hb.ctypes.data, 32 * sigs)
            ver._L.pbftv_memcpy_d2h(ver._h, 0, hb.ctypes.data, small.ptr, 8)
        r["h2d_d2h_roundtrip_us"] = p50(rt)
        ver.set_kernel_timing(True)
        ver.reset_kernel_times()
        for _ in range(200):
            dev()
        for name, k in (("scalars_kernel_us", K_ECDSA_SCALARS), ("comb_kernel_us", K_ECDSA_COMB),
                        ("wave_kernel_us", K_ECDSA_WAVE)):
            ms, cnt = ver.kernel_time_ms(0, k)
            if cnt:
                r[name] = ms * 1e3 / cnt
        ver.set_kernel_timing(False)
        out[f"{sigs}sigs"] = r
        for b in (dh, ds, dk, db, small):
            b.free()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
