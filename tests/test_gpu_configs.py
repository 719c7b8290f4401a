"""The SURVEY.md §8(d) configurations at full size as GPU parity tests (until
round 2 they were checked only inside bench.py):

  config 4  1,048,576 signatures over a 100-key table, 1 % corrupted evenly
            over the 8 classes -- every class checked on its own, on the
            device-resident path and on the host-buffer path (pageable and
            pinned), and a sample plus every corrupted index against the oracle;
  config 3  10,000 certificates of 67 signatures (n = 100, 2f + 1 = 67), 1 % of
            the certificates carrying one bad vote: the quorum must fail
            exactly there;
  config 2  20,000 certificates of 3 signatures (n = 4) in one launch, 1 % with
            one bad vote and 0.5 % with two: QC and the reference's 2f count
            must fail exactly there;
  config 1  the 4-node, 1000-request pattern with every message signed and
            2 % of each kind corrupted, through the four flushes
            (bench.run_config1's flow and check), against the oracle.

Signatures come from OpenSSL (tools/synth.py), an implementation independent of
both the product and the oracle.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

pytestmark = pytest.mark.gpu

N4 = 1 << 20
SEED = 0x50424654


@pytest.fixture(scope="module")
def ver():
    v = Verifier(device_mask=1)
    yield v
    v.close()


@pytest.fixture(scope="module")
def cfg4():
    return synth.config4(N4, n_keys=100, seed=SEED)


def corruption_classes(n, frac=0.01, seed=SEED):
    """index -> class (synth.corrupt draws the corrupted indices first, then
    assigns class t % 8 to the t-th)."""
    rng = np.random.default_rng(seed ^ 0x5A5A)
    idx = rng.choice(n, int(round(n * frac)), replace=False)
    return idx, np.arange(len(idx)) % 8


def test_config4_full_size_every_class(ver, cfg4, oracle_lib):
    pub, H, S, K, ok = cfg4
    valid = ver.register_keys(pub)
    assert valid.all()
    dh, ds, dk = ver.to_device(0, H), ver.to_device(0, S), ver.to_device(0, K)
    db = ver.alloc(0, (N4 + 7) // 8)
    try:
        ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, N4, db.ptr)
        ver.sync(0)
        got = np.unpackbits(db.to_host(), bitorder="little")[:N4].astype(bool)
    finally:
        for b in (dh, ds, dk, db):
            b.free()
    assert (got == ok).all(), f"{int((got != ok).sum())} signatures differ from the construction"
    idx, cls = corruption_classes(N4)
    for c, name in enumerate(synth.CLASSES):
        sel = idx[cls == c]
        assert len(sel) > 1000 and not got[sel].any(), name
    # the oracle on every corrupted index and a sample of the rest
    sample = np.unique(np.concatenate([idx, np.arange(0, N4, 97)]))
    h, s, k = (np.ascontiguousarray(a[sample]) for a in (H, S, K))
    bm = np.zeros((len(sample) + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(h.ctypes.data, s.ctypes.data, k.ctypes.data, len(sample),
                                              pub.ctypes.data, len(pub), bm.ctypes.data, 16)
    assert (np.unpackbits(bm, bitorder="little")[:len(sample)].astype(bool) == got[sample]).all()


def test_config4_full_size_host_path(ver, cfg4):
    pub, H, S, K, ok = cfg4
    ver.register_keys(pub)
    assert (ver.verify_batch(H, S, K) == ok).all()  # pageable (Go heap)
    pins = [ver.pinned(a) for a in (H, S, K)]
    assert (ver.verify_batch(*(p.a for p in pins)) == ok).all()


def test_config3_full_size_quorum(ver):
    per, n_certs = 67, 10000
    pub, H, S, K = synth.certs(100, per, n_certs, seed=per * 7 + 100)  # 670k distinct signatures
    rng = np.random.default_rng(3)
    bad_certs = rng.choice(n_certs, n_certs // 100, replace=False)
    bad_sig = bad_certs * per + rng.integers(0, per, len(bad_certs))
    S[bad_sig, 40] ^= 0x10  # one flipped bit of s in one vote of each bad certificate
    ver.register_keys(pub)
    got = ver.verify_batch(H, S, K).reshape(n_certs, per)
    want = np.ones(n_certs * per, bool)
    want[bad_sig] = False
    assert (got.reshape(-1) == want).all()
    quorum = got.sum(1) >= per  # 2f + 1 = 67 of n = 100
    assert not quorum[bad_certs].any() and quorum.sum() == n_certs - len(bad_certs)


def test_config2_full_size_quorum(ver, oracle_lib):
    """configs[1] at its workload: n = 4 keys, 10k requests x (prepare QC +
    commit QC) = 20,000 certificates x 3 distinct signatures = 60,000 in ONE
    verify_batch_dev launch (<= 8 keys: the lane path without the key sort).
    1 % of the certificates carry one bad vote, 0.5 % two, over the 8 classes
    (synth.corrupt_certs).  Every bit equals the construction; the 2f+1 = 3 QC
    fails exactly where a vote is bad and the reference's 2f = 2 count
    (pbft_impl.go:212,227) exactly where two are; the oracle agrees on every
    corrupted index and a sample."""
    import bench
    out = {}
    r = bench.run_certs(ver, 4, 3, 20000, "config2", outputs=out)
    assert r["check"], r
    assert len(out["K"]) == 60000 and r["rejected"] == 200 + 2 * 100
    want, bits = out["want"], out["bits"]
    sample = np.union1d(np.nonzero(~want)[0], np.arange(0, 60000, 13))
    h, s, k = (np.ascontiguousarray(out[x][sample]) for x in ("H", "S", "K"))
    bm = np.zeros((len(sample) + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(h.ctypes.data, s.ctypes.data, k.ctypes.data, len(sample),
                                              out["pub"].ctypes.data, 4, bm.ctypes.data, 16)
    assert (np.unpackbits(bm, bitorder="little")[:len(sample)].astype(bool) == bits[sample]).all()
    # the same certificates one at a time through pbftv_qc_verify (the latency path)
    for c in list(out["bad_two"][:3]) + list(np.setdiff1d(out["bad_any"], out["bad_two"])[:3]) + [0, 1, 2]:
        sl = slice(3 * int(c), 3 * int(c) + 3)
        got, acc, ok3 = ver.qc_verify(out["H"][sl], out["S"][sl], out["K"][sl], quorum=3)
        assert (got == want[sl]).all() and acc == int(want[sl].sum())
        assert ok3 == (c not in out["bad_any"])
        _, _, ok2 = ver.qc_verify(out["H"][sl], out["S"][sl], out["K"][sl], quorum=2)
        assert ok2 == (c not in out["bad_two"])


def test_config1_every_message_signed(ver, oracle_lib):
    """configs[0] through the four flushes with 2 % of each message kind
    corrupted (bad signatures; validly signed pre-prepares/votes with a wrong
    digest, wrong view or stale sequence ID): every bit equals the
    construction (bench.check_config1) and the oracle -- oracle/gojson.py
    preimages + the oracle verify + oracle_verify_msg against each receipt's
    State -- and the StartConsensus digests equal the oracle's."""
    import bench
    import hashlib
    from test_synth import _config1_oracle
    out = {}
    r = bench.run_config1(ver, outputs=out)
    assert r["check"], r
    assert "29000 signature checks" in r["workload"]
    c, got, idx = out["cluster"], out["got"], out["index"]
    want = _config1_oracle(oracle_lib, c)
    for k in ("request_sig", "preprepare_sig", "preprepare_msg", "vote_sig", "vote_msg", "reply_sig"):
        kind = k.split("_")[0]
        assert (np.asarray(got[k]) == want[k][idx[kind]]).all(), k
    from oracle import gojson
    req_d = [hashlib.sha256(gojson.request(q[0], q[1], q[2], int(a))).digest()
             for q, a in zip(c["requests"], c["assigned_seqs"])]
    assert [bytes(x) for x in got["request_digests"]] == [req_d[j] for j in idx["request"]]


def _openssl_sha256(data, off, ln):
    """The checker: OpenSSL 3 EVP SHA-256 on host threads
    (oracle/openssl_standin.c, built by __graft_entry__.build())."""
    import ctypes
    so = os.path.join(ROOT, "oracle", "libopenssl_standin.so")
    L = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    L.standin_sha256_batch.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_int]
    n = len(ln)
    out = np.zeros((n, 32), np.uint8)
    assert L.standin_sha256_batch(data.ctypes.data, off.ctypes.data, ln.ctypes.data, n, out.ctypes.data, 16) == 0
    return out


def test_config5_full_size_sha256(ver):
    """configs[4] at its full size through the device API: 1,000,000 messages
    of 256-4096 B (2.18 GB, so the last ~1.5 % start past 2^31 and their
    offsets need all 64 bits) in ONE pbftv_sha256_batch_dev call, every digest
    against OpenSSL (and a sample against hashlib), then 1 % of the expected
    digests flipped and the match bitmap checked bit for bit."""
    import hashlib
    data, off, ln = synth.sha_config5(1_000_000)
    n = len(ln)
    assert int(off[-1]) + int(ln[-1]) > 2 ** 31 and (off >= 2 ** 31).sum() > 10_000
    want = _openssl_sha256(data, off, ln)
    rng = np.random.default_rng(5)
    for i in list(rng.integers(0, n, 200)) + list(np.nonzero(off >= 2 ** 31)[0][[0, -1]]):
        assert want[i].tobytes() == hashlib.sha256(data[off[i]:off[i] + ln[i]].tobytes()).digest()
    exp = want.copy()
    flip = rng.choice(n, n // 100, replace=False)
    exp[flip, rng.integers(0, 32, len(flip))] ^= np.uint8(0x10)
    dd = ver.to_device(0, data, pad=64)
    do, dl, de = ver.to_device(0, off), ver.to_device(0, ln), ver.to_device(0, exp)
    dord, dg, db = ver.alloc(0, 4 * n), ver.alloc(0, 32 * n), ver.alloc(0, (n + 31) // 32 * 4)
    try:
        ver.sha256_order_dev(0, dl.ptr, n, dord.ptr)
        ver.sha256_batch_dev(0, dd.ptr, do.ptr, dl.ptr, dord.ptr, n, dg.ptr, de.ptr, db.ptr)
        ver.sync(0)
        got = dg.to_host().reshape(n, 32)
        bad = np.nonzero((got != want).any(1))[0]
        assert len(bad) == 0, (len(bad), bad[:10], off[bad[:10]])
        bits = np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool)
        ok = np.ones(n, bool)
        ok[flip] = False
        assert (bits == ok).all()
    finally:
        for b in (dd, do, dl, de, dord, dg, db):
            b.free()
