"""Concurrency stress of the library on one GPU, every answer checked: the
class of fault behind round 4's unexplained 0-of-67 --
a key change, a free or a rotation racing a certificate -- looked for by
running them all at once for a while.

Two contexts on GPU 0 (--contexts N: more; a third one finds the GPU's
high-priority stream pairs taken and waits for an idle holder to hand one
over, pbftv_api.cpp qc_streams_ready, so idle gaps are mixed in and pairs
change hands while certificates race).  Worker threads (each on its own
context) submit, at
random: certificates of 3 / 8 / 67 / 129 signatures through pbftv_qc_verify
(armed narrow / wide kernels, launches past 128), host-buffer lane batches,
and device-resident batches on library streams.  A control thread every
0.2-0.6 s does one of: switch a context's whole key set (A <-> B, same
geometry: slots rewritten in place), set_key a key to itself, allocate and
free device memory (a GPU-wide quiesce of every armed kernel), a pinned
alloc/free.  PBFTV_QC_ARM_MS=30 makes the keepers rotate every 15 ms.
Every certificate carries corrupted votes, so all-accept and all-reject
answers both fail; every bitmap is compared with the oracle's.

    python tools/stress.py [--seconds S] [--gbits 24 --qbits 16]

One JSON line: counts per operation, wrong answers (with details), errors.
Test infrastructure (the oracle is the checker)."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import random
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def oracle_bits(L, pub, H, S, K):
    n = len(K)
    bm = np.zeros((n + 7) // 8, np.uint8)
    L.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, n, pub.ctypes.data, len(pub),
                                     bm.ctypes.data, 8)
    return np.unpackbits(bm, bitorder="little")[:n].astype(bool)


def corrupt(rng, H, S, frac):
    idx = rng.choice(len(S), max(1, int(frac * len(S))), replace=False)
    for i in idx:
        col = int(rng.integers(0, 96))
        if col < 64:
            S[i, col] ^= np.uint8(1 << int(rng.integers(0, 8)))
        else:
            H[i, col - 64] ^= np.uint8(1 << int(rng.integers(0, 8)))


def make_set(synth, L, seed, rng):
    """100 keys; certificates of 3, 8, 67 and 129 signatures (the 129 ones from
    two 67-signature certificates), ~5 % of the votes corrupted; a pool for
    batches.  Expected bits from the oracle."""
    certs = {}
    pub = None
    for per, cnt in ((3, 60), (8, 40), (67, 40)):
        p, H, S, K = synth.certs(100, per, cnt, seed)
        pub = p if pub is None else pub
        assert (p == pub).all()
        H = H.copy()
        corrupt(rng, H, S, 0.05)
        want = oracle_bits(L, pub, H, S, K)
        certs[per] = [(H[c * per:(c + 1) * per], S[c * per:(c + 1) * per], K[c * per:(c + 1) * per],
                       want[c * per:(c + 1) * per]) for c in range(cnt)]
    certs[129] = [tuple(np.concatenate([x[j], y[j][:62]]) for j in range(4))
                  for x, y in zip(certs[67][0::2], certs[67][1::2])]
    _, H, S, K = synth.certs(100, 64, 512, seed + 1)  # 32,768 signatures for batches
    H = H.copy()
    corrupt(rng, H, S, 0.01)
    pool = (H, S, K, oracle_bits(L, pub, H, S, K))
    return pub, certs, pool


class RWLock:
    """Many workers (shared) or the control thread alone (exclusive)."""

    def __init__(self):
        self.c = threading.Condition()
        self.readers = 0
        self.writer = False

    def shared(self):
        lock = self

        class _S:
            def __enter__(self):
                with lock.c:
                    while lock.writer:
                        lock.c.wait()
                    lock.readers += 1

            def __exit__(self, *a):
                with lock.c:
                    lock.readers -= 1
                    lock.c.notify_all()
        return _S()

    def exclusive(self):
        lock = self

        class _X:
            def __enter__(self):
                with lock.c:
                    while lock.writer:
                        lock.c.wait()
                    lock.writer = True
                    while lock.readers:
                        lock.c.wait()

            def __exit__(self, *a):
                with lock.c:
                    lock.writer = False
                    lock.c.notify_all()
        return _X()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--gbits", default="24")
    ap.add_argument("--qbits", default="16")
    ap.add_argument("--contexts", type=int, default=2)
    a = ap.parse_args()
    nctx = max(2, a.contexts)
    os.environ.setdefault("PBFTV_GBITS", a.gbits)
    os.environ.setdefault("PBFTV_QBITS", a.qbits)
    os.environ.setdefault("PBFTV_QC_ARM_MS", "30")
    import synth  # noqa: E402
    from simple_pbft_amd import Verifier  # noqa: E402
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    vp = ctypes.c_void_p
    L.oracle_ecdsa_p256_verify_batch.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint32, vp, ctypes.c_int]
    rng = np.random.default_rng(20261018)
    sets = [make_set(synth, L, 0x50424654 + 17 * k, rng) for k in range(2)]
    ctxs = [Verifier(device_mask=1) for _ in range(nctx)]
    cur = [c % 2 for c in range(nctx)]  # key set of each context
    locks = [RWLock() for _ in range(nctx)]  # workers shared; the control thread alone while it changes a context's keys
    for c in range(nctx):
        ctxs[c].register_keys(sets[cur[c]][0])
    stop = threading.Event()
    counts, wrong, errors = {}, [], []
    cl = threading.Lock()

    def note(key, ok=True, detail=None):
        with cl:
            counts[key] = counts.get(key, 0) + 1
            if not ok:
                wrong.append(detail)

    def worker(c, seed, kinds):
        r = random.Random(seed)
        v = ctxs[c]
        streams = [v.stream_create(0) for _ in range(2)]
        dev = None
        try:
            while not stop.is_set():
                kind = r.choice(kinds)
                if kind == "idle":  # (a holder idle for 0.2 s hands its pair to a waiting context)
                    time.sleep(r.uniform(0.1, 0.5))
                    note(kind)
                    continue
                with locks[c].shared():
                    s = cur[c]
                    pub, certs, pool = sets[s]
                    if kind.startswith("cert"):
                        per = int(kind[4:])
                        H, S, K, want = r.choice(certs[per])
                        bm, acc, okq = v.qc_verify(H, S, K, quorum=len(K))
                        good = (bm == want).all() and acc == int(want.sum())
                        note(kind, good, None if good else {"kind": kind, "ctx": c, "set": s, "acc": int(acc),
                                                            "want": int(want.sum()), "armed": v.qc_stamps(0)["armed"]})
                    elif kind == "host_batch":
                        H, S, K, want = pool
                        lo = r.randrange(0, 16384)
                        n = r.choice([2049, 5000, 16384])
                        got = v.verify_batch(H[lo:lo + n], S[lo:lo + n], K[lo:lo + n])
                        good = (got == want[lo:lo + n]).all()
                        note(kind, good, None if good else {"kind": kind, "ctx": c, "set": s, "n": n,
                                                            "wrong": int((got != want[lo:lo + n]).sum())})
                    else:  # device-resident batch on a library stream
                        H, S, K, want = pool
                        if dev is None or dev[0] != s:
                            if dev is not None:
                                for b in dev[1]:
                                    b.free()
                            dev = (s, [v.to_device(0, H), v.to_device(0, S), v.to_device(0, K),
                                       v.alloc(0, len(K) // 8 + 1)])
                        dh, ds, dk, db = dev[1]
                        st = r.choice(streams)
                        v.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, len(K), db.ptr, stream=st)
                        v.stream_wait(0, st)
                        got = np.unpackbits(db.to_host(), bitorder="little")[:len(K)].astype(bool)
                        good = (got == want).all()
                        note(kind, good, None if good else {"kind": kind, "ctx": c, "set": s,
                                                            "wrong": int((got != want).sum())})
        except Exception as e:  # noqa: BLE001 -- reported
            errors.append(f"worker {c}/{seed}: {e!r}")
        finally:
            if dev is not None:
                for b in dev[1]:
                    b.free()
            for st in streams:
                v.stream_destroy(0, st)

    def control():
        r = random.Random(7)
        try:
            while not stop.is_set():
                time.sleep(r.uniform(0.2, 0.6))
                op = r.choice(["switch", "switch", "set_key", "dev_free", "host_free"])
                c = r.randrange(nctx)
                if op == "switch":
                    with locks[c].exclusive():
                        cur[c] ^= 1
                        valid = ctxs[c].register_keys(sets[cur[c]][0])
                        assert valid.all()
                elif op == "set_key":
                    with locks[c].exclusive():
                        k = r.randrange(100)
                        assert ctxs[c].set_key(k, sets[cur[c]][0][k])
                elif op == "dev_free":
                    ctxs[c].alloc(0, 1 << 20).free()
                else:
                    ctxs[c].pinned(np.zeros(1 << 16, np.uint8)).free()
                note("ctl_" + op)
        except Exception as e:  # noqa: BLE001
            errors.append(f"control: {e!r}")

    ths = [threading.Thread(target=worker, args=(0, 1, ["cert3", "cert3", "cert8", "cert67", "cert129"])),
           threading.Thread(target=worker, args=(0, 2, ["host_batch", "dev_batch", "cert3"])),
           threading.Thread(target=worker, args=(1, 3, ["cert3", "cert67", "cert8", "dev_batch"]
                                                 + (["idle"] if nctx > 2 else []))),
           threading.Thread(target=control)]
    ths += [threading.Thread(target=worker, args=(c, 10 + c, ["cert3", "cert3", "cert8", "cert67", "idle"]))
            for c in range(2, nctx)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    last = t0
    while time.perf_counter() - t0 < a.seconds and not errors:
        time.sleep(1.0)
        if time.perf_counter() - last > 30:  # progress for the run's watchdog
            last = time.perf_counter()
            with cl:
                print(json.dumps({"progress_s": round(last - t0), "counts": dict(counts), "wrong": len(wrong)}),
                      file=sys.stderr, flush=True)
    stop.set()
    for t in ths:
        t.join(timeout=60)
    hung = [i for i, t in enumerate(ths) if t.is_alive()]
    qc = [{k: int(v.qc_counters(0)[k]) for k in ("calls", "armed", "launches", "armings")} for v in ctxs]
    for v in ctxs:
        v.close()
    out = {"seconds": time.perf_counter() - t0, "contexts": nctx, "qc_counters": qc, "counts": counts, "wrong": len(wrong), "wrong_detail": wrong[:20],
           "errors": errors[:10], "hung_threads": hung,
           "env": {k: v for k, v in os.environ.items() if k.startswith("PBFTV")}}
    print(json.dumps(out), flush=True)
    sys.exit(0 if not wrong and not errors and not hung else 1)


if __name__ == "__main__":
    main()
