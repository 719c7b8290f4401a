"""Short workload for rocprofv3 --pmc passes (tools/pmc_passes.sh): every
kernel the roofline claims rest on, each launched a few times --
  * config 4 verify (1M signatures, 100 keys): k_key_*, k_ecdsa_scalars, k_ecdsa_comb;
  * config 5 digests (1M messages, 256 B..4 KiB): k_sha256;
  * one quorum certificate (n = 4, 3 signatures) through the latency path: k_ecdsa_wave.
Not a benchmark: the numbers come from the counters."""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402


def main():
    which = sys.argv[1:] or ["comb", "sha", "wave"]
    ver = Verifier(device_mask=1)
    if "comb" in which:
        n = 1 << 20
        pub, H, S, K, ok = synth.config4(n, n_keys=100, seed=0x50424654)
        ver.register_keys(pub)
        dh, ds, dk = ver.to_device(0, H), ver.to_device(0, S), ver.to_device(0, K)
        db = ver.alloc(0, (n + 7) // 8)
        ver.reserve(n)
        for _ in range(3):
            ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr)
        ver.sync(0)
        got = np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool)
        assert (got == ok).all()
        for b in (dh, ds, dk, db):
            b.free()
    if "sha" in which:
        n = 1_000_000
        data, off, ln = synth.sha_config5(n)
        dd = ver.to_device(0, data, pad=64)
        do, dl = ver.to_device(0, off), ver.to_device(0, ln)
        dord, dg = ver.alloc(0, 4 * n), ver.alloc(0, 32 * n)
        ver.sha256_order_dev(0, dl.ptr, n, dord.ptr)
        for _ in range(3):
            ver.sha256_batch_dev(0, dd.ptr, do.ptr, dl.ptr, dord.ptr, n, dg.ptr)
        ver.sync(0)
        for b in (dd, do, dl, dord, dg):
            b.free()
    if "wave" in which:
        pub, H, S, K = synth.qc(4, 3, 11)
        ver.register_keys(pub)
        for _ in range(50):
            _, acc, q = ver.qc_verify(H, S, K, quorum=3)
            assert q and acc == 3
    ver.close()
    print("pmc workload done:", " ".join(which))


if __name__ == "__main__":
    main()
