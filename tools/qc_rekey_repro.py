"""Replays the round-4 r04a sequence that returned 0 of 67 on hardware
(gpurun_out/r04a/cadence.err: tools/qc_cadence.py parts cpu,b2b,free,tick,load
on the round-3 library), with corrupted votes in every certificate so that an
all-reject AND an all-accept answer both fail, and classifies every wrong
bitmap:

  register key set A (100 keys) -> 67-signature certificates back to back and
  at 1-s gaps (the armed kernel runs out) -> ~2 s of host work -> register key
  set B (100 keys: same geometry, the key-table slots are reused) -> 3-signature
  certificates (armed) back to back and at 2-ms gaps -> 67- and 129-signature
  certificates.

For a wrong bitmap it reports whether it equals the previous call's inputs
verified under the current keys (stale inputs), the previous call's answer
(stale verdict bytes), all zeros or something else.

    python tools/qc_rekey_repro.py [--lib-root DIR] [--rounds R] [--quick]

--lib-root: directory holding the simple_pbft_amd package to test (default:
this repo; exp/r3 holds the round-3 library for the before/after check).
Prints one JSON line per round and a summary line.  Test infrastructure: the
oracle (oracle/liboracle.so) is the checker.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def oracle():
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    vp = ctypes.c_void_p
    L.oracle_ecdsa_p256_verify_batch.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint32, vp, ctypes.c_int]
    return L


def expect(L, pub, H, S, K):
    n = len(K)
    bm = np.zeros((n + 7) // 8, np.uint8)
    L.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, n, pub.ctypes.data, len(pub),
                                     bm.ctypes.data, 8)
    return np.unpackbits(bm, bitorder="little")[:n].astype(bool)


def make_certs(synth, L, seed, sigs, count, rng):
    """count certificates of `sigs` votes by a 100-key committee; in every one
    1-3 votes corrupted (r, s or hash byte flipped): expected bits from the oracle."""
    pub, H, S, K = synth.certs(100, sigs, count, seed)
    H = H.copy()
    for c in range(count):
        for j in rng.choice(sigs, int(rng.integers(1, min(3, sigs) + 1)), replace=False):
            i = c * sigs + int(j)
            which = int(rng.integers(0, 3))
            if which == 0:
                S[i, int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
            elif which == 1:
                S[i, 32 + int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
            else:
                H[i, int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
    want = expect(L, pub, H, S, K)
    calls = [(H[c * sigs:(c + 1) * sigs], S[c * sigs:(c + 1) * sigs], K[c * sigs:(c + 1) * sigs],
              want[c * sigs:(c + 1) * sigs]) for c in range(count)]
    return pub, calls


class Runner:
    def __init__(self, ver, L):
        self.ver, self.L = ver, L
        self.pub = None
        self.prev = None  # (H, S, K, got) of the previous call
        self.calls = 0
        self.bad = []

    def run(self, phase, calls, gap=0.0):
        for i, (H, S, K, want) in enumerate(calls):
            if gap:
                time.sleep(gap)
            got = np.asarray(self.ver.verify_batch(H, S, K), bool)
            self.calls += 1
            if not (got == want).all():
                cls = "other"
                if not got.any():
                    cls = "all_zero"
                elif got.all():
                    cls = "all_one"
                if self.prev is not None and len(self.prev[2]) >= len(K):
                    pH, pS, pK, pgot = self.prev
                    n = len(K)
                    stale = expect(self.L, self.pub, pH[:n].copy(), pS[:n].copy(), pK[:n].copy())
                    if (got == stale).all():
                        cls += "+prev_inputs_under_current_keys"
                    if (got == pgot[:n]).all():
                        cls += "+prev_answer"
                self.bad.append({"phase": phase, "call": i, "n": len(K), "wrong": int((got != want).sum()),
                                 "accepted": int(got.sum()), "expected_accepted": int(want.sum()), "class": cls})
            self.prev = (H, S, K, got)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib-root", default=ROOT)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth  # noqa: E402
    sys.path.insert(0, os.path.abspath(a.lib_root))
    from simple_pbft_amd import Verifier  # noqa: E402
    L = oracle()
    rng = np.random.default_rng(5)
    ticks = 3 if a.quick else 6
    A = [make_certs(synth, L, 201 + 2 * r, 67, 60 + ticks, rng) for r in range(a.rounds)]
    B3 = [make_certs(synth, L, 0x50424654 + r, 3, 320, rng) for r in range(a.rounds)]
    B67 = [make_certs(synth, L, 0x50424654 + r, 67, 60, rng) for r in range(a.rounds)]
    # 129 signatures (past the armed kernel's 128 waves): two certificates' votes in one call
    B129 = [(B67[r][0], [tuple(np.concatenate([x[j], y[j][:62]]) for j in range(4))
                         for x, y in zip(B67[r][1][:40:2], B67[r][1][1:40:2])]) for r in range(a.rounds)]
    total_bad = 0
    with Verifier(device_mask=1) as ver:
        R = Runner(ver, L)
        for r in range(a.rounds):
            t0 = time.perf_counter()
            R.bad = []
            pubA, ca = A[r]
            ver.register_keys(pubA)
            R.pub = pubA
            R.prev = None
            R.run("A67_b2b", ca[:60])
            R.run("A67_tick1s", ca[60:], gap=1.0)
            time.sleep(2.0)  # the host work before the next registration (synth.config4 in r04a)
            pubB, c3 = B3[r]
            assert (B67[r][0] == pubB).all() and (B129[r][0] == pubB).all()
            ver.register_keys(pubB)
            R.pub = pubB
            R.run("B3_b2b", c3[:20])
            R.run("B3_gap2ms", c3[20:], gap=0.002)
            R.run("B67_first", B67[r][1][:10])
            R.run("B67_gap2ms", B67[r][1][10:], gap=0.002)
            R.run("B129", B129[r][1])
            R.run("B3_after", c3[:20])
            total_bad += len(R.bad)
            print(json.dumps({"round": r, "seconds": time.perf_counter() - t0, "calls": R.calls, "bad": R.bad[:20],
                              "bad_count": len(R.bad)}), flush=True)
    print(json.dumps({"summary": True, "lib_root": a.lib_root, "rounds": a.rounds, "bad_total": total_bad}),
          flush=True)
    sys.exit(1 if total_bad else 0)


if __name__ == "__main__":
    main()
