"""Key-table management and the in-context multi-device path on hardware.

* pbftv_add_keys / pbftv_set_key: keys appended or replaced one at a time at
  the registered geometry, each checked against the oracle's verify.
* PBFTV_ALIAS_DEVICES=2 maps two logical context devices onto GPU 0, so the
  paths a multi-GPU context takes -- per-device registration, contiguous
  shards of 512-aligned items, per-shard pipelines / flushes, and the bitmap
  concatenation at s.lo / 8 -- run here against the oracle, with batch sizes
  that are not multiples of 512."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import fixture_arrays, oracle_sign_pool
from oracle import gojson

pytestmark = pytest.mark.gpu


def _oracle_bits(oracle_lib, H, S, K, keys):
    n = len(K)
    want = np.zeros((n + 7) // 8 + 1, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, n, keys.ctypes.data,
                                              len(keys), want.ctypes.data, 8)
    return np.unpackbits(want, bitorder="little")[:n].astype(bool)


@pytest.fixture(params=["wave", "lane"])
def path(request, monkeypatch):
    monkeypatch.setenv("PBFTV_WAVE_MAX", "100000000" if request.param == "wave" else "0")
    return request.param


def test_add_and_set_keys(oracle_lib, path, monkeypatch):
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_GBITS", "24")  # small tables: this test is about key bookkeeping
    monkeypatch.setenv("PBFTV_QBITS", "16")
    keys, H, S, K = oracle_sign_pool(oracle_lib, 6, 40, seed=71)
    with Verifier() as v:
        assert v.register_keys(keys[:3]).all()
        assert v.table_config()[:2] == (24, 16)
        # signatures under keys 3..5 fail while those keys are unknown (index out of range)
        got = v.verify_batch(H, S, K)
        assert got.tolist() == (K < 3).tolist()
        assert v.add_keys(keys[3:5]).all()
        got = v.verify_batch(H, S, K)
        assert got.tolist() == (K < 5).tolist()
        assert v.add_keys(keys[5:]).all()
        assert v.verify_batch(H, S, K).all()
        assert v.table_config()[2] > 0
        # replace key 1 by key 4: key 1's signatures now fail, key 4's verify under index 1
        assert v.set_key(1, keys[4])
        K2 = K.copy()
        K2[K == 4] = 1
        want = _oracle_bits(oracle_lib, H, S, K2, np.concatenate([keys[:1], keys[4:5], keys[2:]]))
        assert v.verify_batch(H, S, K2).tolist() == want.tolist()
        assert not v.verify_batch(H[K == 1], S[K == 1], K[K == 1]).any()
        # an invalid key is reported and its signatures fail
        bad = keys[0].copy()
        bad[63] ^= 1
        assert not v.set_key(2, bad)
        assert not v.verify_batch(H[K == 2], S[K == 2], K[K == 2]).any()
        with pytest.raises(Exception):
            v.set_key(99, keys[0])


@pytest.fixture
def two_devices(monkeypatch):
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_ALIAS_DEVICES", "2")
    monkeypatch.setenv("PBFTV_GBITS", "24")
    monkeypatch.setenv("PBFTV_QBITS", "16")
    v = Verifier()
    assert v.device_count() == 2 and v.device_id(0) == v.device_id(1)
    yield v
    v.close()


@pytest.mark.parametrize("n", [2049, 5000, 70001])
def test_two_device_shards_vs_oracle(two_devices, oracle_lib, n):
    """Host-buffer verify split over two logical devices (pipelined shards,
    key order in both at 70001), bitmap joined at the 512-aligned boundary."""
    v = two_devices
    keys, h, s, k = oracle_sign_pool(oracle_lib, 10, 30, seed=n)
    assert v.register_keys(keys).all()
    rng = np.random.default_rng(n)
    idx = rng.integers(0, len(k), n)
    H, S, K = h[idx].copy(), s[idx].copy(), k[idx].copy()
    bad = rng.choice(n, n // 50, replace=False)
    S[bad, 5] ^= 0x10
    got = v.verify_batch(H, S, K)
    want = np.ones(n, bool)
    want[bad] = False
    assert got.tolist() == want.tolist()
    sample = rng.choice(n, 300, replace=False)
    assert got[sample].tolist() == _oracle_bits(oracle_lib, H[sample], S[sample], K[sample], keys).tolist()


def test_two_device_fixtures_and_flush(two_devices, oracle_lib, ecdsa_fixtures):
    """Golden vectors tiled past one shard, and a vote flush + SHA batch split
    over the two devices."""
    from simple_pbft_amd.pbftv import VoteColumns
    v = two_devices
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    v.register_keys(keys)
    reps = 3000 // len(kidx) + 1
    H, S, K = np.tile(hashes, (reps, 1)), np.tile(sigs, (reps, 1)), np.tile(kidx, reps)
    assert v.verify_batch(H, S, K).tolist() == np.tile(expect, reps).tolist()
    n = 3333
    votes = [(7, i, b"%064x" % (i * 977), b"node%d" % (i % 4), i % 2) for i in range(n)]
    dg, _, _ = v.flush_votes(VoteColumns(votes))
    assert [x.tobytes() for x in dg] == [hashlib.sha256(gojson.vote(*x)).digest() for x in votes]
    msgs = [bytes([i % 251]) * (i % 300) for i in range(n)]
    data, off, ln = v.pack(msgs)
    assert [x.tobytes() for x in v.sha256_batch(data, off, ln)] == [hashlib.sha256(m).digest() for m in msgs]


def test_two_device_registration_geometry(two_devices, oracle_lib):
    v = two_devices
    keys, H, S, K = oracle_sign_pool(oracle_lib, 3, 4, seed=5)
    assert v.register_keys(keys).all()
    g, q, b = v.table_config()
    assert (g, q) == (24, 16) and b > 0
    assert v.add_keys(keys[:1]).all()          # both logical devices get the new table
    K2 = np.concatenate([K, np.full(4, 3, np.uint32)])
    assert v.verify_batch(np.concatenate([H, H[:4]]), np.concatenate([S, S[:4]]), K2).all()


def ctypes_void(p):
    import ctypes
    return ctypes.c_void_p(p)


def _foreign_stream():
    """A HIP stream the library did not create (hipStreamCreateWithFlags,
    non-blocking), as a caller that owns its streams would pass one."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    st = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(st), ctypes.c_uint(1)) == 0
    return hip, st.value


@pytest.mark.parametrize("stream_kind", ["library", "foreign"])
@pytest.mark.parametrize("path_n", [64, 40_000])  # the wave kernel (<= 2048) and the lane path
def test_set_key_waits_for_caller_stream_verifies(oracle_lib, path_n, stream_kind, monkeypatch):
    """a verify enqueued on a CALLER stream (pbftv_stream_create +
    verify_batch_dev, or a stream the caller made itself) must still see the
    old key table when pbftv_set_key replaces that key right after the
    enqueue: set_key waits for every stream this context was given before it
    rewrites the table in place (round 4: only this context's work, not the
    whole device)."""
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_GBITS", "24")
    monkeypatch.setenv("PBFTV_QBITS", "16")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, 4, 16, seed=73)
    rng = np.random.default_rng(74)
    o = rng.integers(0, len(kidx), path_n)
    H, S, K = hashes[o].copy(), sigs[o].copy(), kidx[o].copy()
    with Verifier(device_mask=1) as v:
        assert v.register_keys(keys).all()
        bufs = [v.to_device(0, H), v.to_device(0, S), v.to_device(0, K), v.alloc(0, (path_n + 7) // 8)]
        hip = None
        if stream_kind == "library":
            side = v.stream_create(0)
        else:
            hip, side = _foreign_stream()
        # a queue of verifies several ms long, so the rewrite would overlap it
        deep = 40 if path_n <= 2048 else 8
        outs = [v.alloc(0, (path_n + 7) // 8) for _ in range(deep)]
        bufs += outs
        try:
            for _ in range(3):
                for o in outs:
                    o.zero()
                for o in outs:
                    v.verify_batch_dev(0, bufs[0].ptr, bufs[1].ptr, bufs[2].ptr, path_n, o.ptr, stream=side)
                assert v.set_key(0, keys[1])  # key 0 now holds key 1's point
                v.stream_wait(0, side)
                for j, o in enumerate(outs):
                    got = np.unpackbits(o.to_host(), bitorder="little")[:path_n].astype(bool)
                    assert got.all(), f"verify {j} queued before set_key saw the new table"
                assert v.set_key(0, keys[0])
            # after the change, key-0 signatures fail under index 0
            v.set_key(0, keys[1])
            got = v.verify_batch(H, S, K)
            assert got.tolist() == (K != 0).tolist()
        finally:
            if hip is None:
                v.stream_destroy(0, side)
            else:
                v.stream_wait(0, side)
                hip.hipStreamDestroy(ctypes_void(side))
            for b in bufs:
                b.free()


def test_bitmap_padding_bits_are_zero(oracle_lib, monkeypatch):
    """bits past n in the last bitmap byte are 0 on every path, even
    when the buffer held ones before: the wave kernel on a device buffer, and
    the host pipeline whose chunks take the wave kernel (PBFTV_HOST_CHUNK=512,
    a ragged last chunk after a batch that set those bits)."""
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_GBITS", "24")
    monkeypatch.setenv("PBFTV_QBITS", "16")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, 3, 8, seed=75)
    with Verifier(device_mask=1) as v:
        assert v.register_keys(keys).all()
        for n in (1, 5, 13, 24):
            dh, ds, dk = v.to_device(0, hashes[:n]), v.to_device(0, sigs[:n]), v.to_device(0, kidx[:n])
            db = v.alloc(0, 4)
            v._L.pbftv_memset_dev(v._h, 0, db.ptr, 0xFF, 4)
            v.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr)
            v.sync(0)
            raw = db.to_host()
            bits = np.unpackbits(raw, bitorder="little")
            nb = (n + 7) // 8
            assert bits[:n].all() and not bits[n:8 * nb].any(), (n, raw)
            assert (raw[nb:] == 0xFF).all()  # bytes past the bitmap untouched
            for b in (dh, ds, dk, db):
                b.free()
        monkeypatch.setenv("PBFTV_HOST_CHUNK", "512")
        # n > 2048: the call takes the pipeline, whose 512-signature chunks take the wave kernel
        reps = 3000 // len(kidx) + 1
        H, S, K = np.tile(hashes, (reps, 1)), np.tile(sigs, (reps, 1)), np.tile(kidx, reps)
        assert v.verify_batch(H[:3000], S[:3000], K[:3000]).all()
        L = v._L
        for n in (2999, 2993):
            bm = np.zeros((n + 7) // 8 + 1, np.uint8)
            rc = L.pbftv_ecdsa_p256_verify_batch(v._h, np.ascontiguousarray(H[:n]).ctypes.data,
                                                 np.ascontiguousarray(S[:n]).ctypes.data,
                                                 np.ascontiguousarray(K[:n]).ctypes.data, n, bm.ctypes.data)
            assert rc == 0
            bits = np.unpackbits(bm[:(n + 7) // 8], bitorder="little")
            assert bits[:n].all() and not bits[n:].any(), n


def test_latency_path_goes_to_least_loaded_device(oracle_lib, monkeypatch):
    """in a multi-device context a certificate goes to the
    device with the least lane-path work queued (pbftv_api.cpp
    latency_device), not always to device 0.  Two logical devices on GPU 0
    (PBFTV_ALIAS_DEVICES=2): with a 1M batch just enqueued on device 0, the
    next certificate is served on device 1 (its pbftv_qc_stamps record the
    call); with nothing queued it goes to device 0.  Every bitmap against the
    oracle."""
    import time
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_ALIAS_DEVICES", "2")
    monkeypatch.setenv("PBFTV_GBITS", "24")
    monkeypatch.setenv("PBFTV_QBITS", "16")
    keys, H, S, K = oracle_sign_pool(oracle_lib, 4, 16, seed=73)
    S[::5, 11] ^= 0x10
    want = _oracle_bits(oracle_lib, H, S, K, keys)
    n = 1 << 20
    reps = n // len(K)
    with Verifier(device_mask=1) as v:
        assert v.device_count() == 2
        v.register_keys(keys)
        dh, ds, dk = (v.to_device(0, np.tile(a, (reps, 1)) if a.ndim > 1 else np.tile(a, reps)) for a in (H, S, K))
        db = v.alloc(0, n // 8 + 1)
        try:
            for i in range(0, 12, 3):  # idle: device 0 serves
                assert (v.verify_batch(H[i:i + 3], S[i:i + 3], K[i:i + 3]) == want[i:i + 3]).all()
            before = v.qc_stamps(1)["total_us"]
            assert v.qc_stamps(0)["total_us"] > 0 and before == 0
            time.sleep(0.01)
            v.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr)  # ~1 ms of device 0 queued
            got = v.verify_batch(H[12:15], S[12:15], K[12:15])
            assert (got == want[12:15]).all()
            assert v.qc_stamps(1)["total_us"] > 0  # served by device 1
            v.sync(0)
            bm = np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool)
            assert (bm == np.tile(want, reps)).all()
        finally:
            for b in (dh, ds, dk, db):
                b.free()
