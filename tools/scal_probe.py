"""Stage timing inside k_ecdsa_scalars (experiment build with -DPBFTV_SCAL_PROBE):

    make -C simple_pbft_amd OBJ=/tmp/probe_build LIB=$PWD/exp/libpbftv_probe.so EXTRA=-DPBFTV_SCAL_PROBE
    PBFTV_LIB=$PWD/exp/libpbftv_probe.so python tools/scal_probe.py [N ...]

One verify of N config-4 signatures (100 keys) after warm-up, then lane 0 of
every wave's wall_clock64() stamps (100 MHz) at the stage boundaries:
  0 start, 1 key starts, 2 forward products, 3 lane total + claims,
  4 wave inversion, 5 backward pass + records; inside the inversion
  (wave_batch_inv_n, K <= 2): 6 scans done, 7 safegcd done.
Prints the median / p90 of each stage over the waves and the spread of the
waves' start and end times."""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402
from simple_pbft_amd import pbftv  # noqa: E402

NAMES = ["key starts", "forward", "total+claims", "inversion", "backward+records"]


def probe(ver, n, reps=5):
    pub, H, S, K, ok = synth.config4(n, n_keys=100, seed=0x50424654)
    ver.register_keys(pub)
    dh, ds, dk = ver.to_device(0, H), ver.to_device(0, S), ver.to_device(0, K)
    db = ver.alloc(0, (n + 7) // 8)
    ver.reserve(n)
    f = pbftv.lib().pbftv_debug_scal_probe
    f.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]
    buf = np.zeros(8192 * 8, dtype=np.uint64)
    rows = []
    for r in range(reps + 2):
        buf[:] = 0
        ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr)
        ver.sync(0)
        assert f(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), buf.size) == 0
        if r < 2:
            continue
        t = buf.reshape(8192, 8).astype(np.int64)
        t = t[t[:, 0] != 0]
        rows.append(t)
    got = np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool)
    assert (got == ok).all(), "verify mismatch"
    for b in (dh, ds, dk, db):
        b.free()
    print(f"n = {n}: {rows[0].shape[0]} waves, {reps} launches (us, 100 MHz stamps)")
    for t in rows:
        d = np.diff(t[:, :6], axis=1) * 0.01
        span = (t[:, 5] - t[:, 0]) * 0.01
        start = (t[:, 0] - t[:, 0].min()) * 0.01
        end = (t[:, 5].max() - t[:, 0].min()) * 0.01
        parts = "  ".join(f"{nm} {np.median(d[:, i]):.1f}/{np.percentile(d[:, i], 90):.1f}" for i, nm in enumerate(NAMES))
        print(f"  first->last {end:.1f}  wave span med {np.median(span):.1f} max {span.max():.1f}  "
              f"start spread {start.max():.1f}  | {parts}")
        if (t[:, 6] != 0).all():
            sc, sg, tl = (t[:, 6] - t[:, 3]) * 0.01, (t[:, 7] - t[:, 6]) * 0.01, (t[:, 4] - t[:, 7]) * 0.01
            print(f"    inversion = scans {np.median(sc):.1f}/{np.percentile(sc, 90):.1f} + safegcd "
                  f"{np.median(sg):.1f}/{np.percentile(sg, 90):.1f} + tail {np.median(tl):.1f}/{np.percentile(tl, 90):.1f}")


def main():
    ns = [int(a) for a in sys.argv[1:]] or [131072, 1 << 20]
    ver = Verifier(device_mask=1)
    for n in ns:
        probe(ver, n)
    ver.close()


if __name__ == "__main__":
    main()
