"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the
committed golden fixtures.  Bit-exact for every digest and every accept bit."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import fixture_arrays, oracle_sign_pool

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ver():
    from simple_pbft_amd import Verifier
    v = Verifier()
    yield v
    v.close()


# Two ECDSA paths: "wave" (one wave per signature, batches <= PBFTV_WAVE_MAX)
# and "lane" (one signature per lane: scalars + comb kernels).  Parity tests
# run through both by moving the threshold.
@pytest.fixture(params=["wave", "lane"])
def path(request, monkeypatch):
    monkeypatch.setenv("PBFTV_WAVE_MAX", "100000000" if request.param == "wave" else "0")
    return request.param


# ------------------------------------------------------------------ SHA-256
def test_sha256_fixtures(ver, sha_fixtures):
    msgs, want = [], []
    for v in sha_fixtures:
        if "msg" in v:
            msgs.append(bytes.fromhex(v["msg"]))
        else:
            msgs.append(bytes.fromhex(v["msg_repeat"]["byte"]) * v["msg_repeat"]["count"])
        want.append(v["digest"])
    blob, off, ln = ver.pack(msgs)
    got = ver.sha256_batch(blob, off, ln)
    assert [g.tobytes().hex() for g in got] == want


def test_sha256_random_unaligned(ver):
    rng = np.random.default_rng(7)
    n = 3000
    lengths = rng.integers(0, 8193, n).astype(np.uint32)
    lengths[:130] = np.arange(130)  # every tail shape
    gaps = rng.integers(0, 7, n)
    offsets = np.zeros(n, np.uint64)
    pos = 0
    for i in range(n):
        pos += int(gaps[i])
        offsets[i] = pos
        pos += int(lengths[i])
    data = np.frombuffer(rng.bytes(pos + 16), np.uint8).copy()
    got = ver.sha256_batch(data, offsets, lengths)
    for i in range(n):
        m = data[offsets[i]:offsets[i] + lengths[i]].tobytes()
        assert got[i].tobytes() == hashlib.sha256(m).digest(), (i, lengths[i], offsets[i])


def test_sha256_empty_batch_and_empty_message(ver):
    assert ver.sha256_batch(np.zeros(1, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32)).shape == (0, 32)
    assert ver.hash_hex(b"") == hashlib.sha256(b"").hexdigest()


def test_sha256_empty_messages_on_line_boundaries(ver):
    """Empty messages at 128-B-aligned offsets (the ring kernel reads no line
    for them), one at the very end of the data, among 1..300-B neighbours
    that end exactly on line boundaries."""
    rng = np.random.default_rng(19)
    lens, offs, pos = [], [], 0
    for i in range(600):
        if i % 3 == 0:
            pos = (pos + 127) // 128 * 128  # an empty message on a line boundary
            lens.append(0)
        else:
            lens.append(int(rng.integers(1, 300)))
            if i % 3 == 2:  # ends exactly on a line boundary
                lens[-1] = (pos + lens[-1] + 127) // 128 * 128 - pos
        offs.append(pos)
        pos += lens[-1]
    pos = (pos + 127) // 128 * 128
    lens.append(0)
    offs.append(pos)  # empty, at the end of the data
    data = np.frombuffer(rng.bytes(pos), np.uint8).copy()
    lengths = np.array(lens, np.uint32)
    offsets = np.array(offs, np.uint64)
    got = ver.sha256_batch(data, offsets, lengths)
    for i in range(len(lens)):
        m = data[offs[i]:offs[i] + lens[i]].tobytes()
        assert got[i].tobytes() == hashlib.sha256(m).digest(), (i, lens[i], offs[i])


def test_digest_check(ver):
    rng = np.random.default_rng(3)
    msgs = [rng.bytes(int(l)) for l in rng.integers(0, 300, 777)]
    blob, off, ln = ver.pack(msgs)
    exp = np.array([list(hashlib.sha256(m).digest()) for m in msgs], np.uint8)
    flip = rng.random(len(msgs)) < 0.3
    exp[flip, 5] ^= 0x40
    got = ver.digest_check_batch(blob, off, ln, exp)
    assert (got == ~flip).all()


def test_sha256_small_calls_zero_copy(ver):
    """Digest calls of <= 64 messages and <= 64 KiB (pbftv_hash_hex, a few
    requests) take the zero-copy path: the messages packed into pinned
    coherent host memory that k_sha256 reads over the bus, digests written
    back the same way, one launch.  Every size class, offsets at every byte
    alignment, empty messages, the 64-message / 64-KiB limits and one past
    each (the DMA path) against hashlib."""
    rng = np.random.default_rng(23)
    for n, maxlen in [(1, 0), (1, 1), (1, 55), (1, 56), (1, 64), (1, 99), (1, 4096), (1, 65536), (1, 65537),
                      (2, 300), (7, 1000), (33, 130), (64, 1024), (64, 1025), (65, 200)]:
        lens = rng.integers(0, maxlen + 1, n).astype(np.uint32)
        lens[0] = maxlen
        gaps = rng.integers(0, 9, n)
        offs = np.zeros(n, np.uint64)
        pos = int(rng.integers(0, 200))
        for i in range(n):
            offs[i] = pos
            pos += int(lens[i]) + int(gaps[i])
        data = np.frombuffer(rng.bytes(pos + 8), np.uint8).copy()
        got = ver.sha256_batch(data, offs, lens)
        want = [hashlib.sha256(data[int(o):int(o) + int(l)].tobytes()).digest() for o, l in zip(offs, lens)]
        assert [g.tobytes() for g in got] == want, (n, maxlen)
    for m in (b"", b"a", bytes(range(99)), rng.bytes(1 << 16)):
        assert ver.hash_hex(m) == hashlib.sha256(m).hexdigest()


def test_hash_hex_and_request_digests(ver, digest_kats):
    """utils.Hash / digest(*RequestMsg) on the reference's own logged requests."""
    reqs = []
    for r in digest_kats["requests"] + digest_kats["escapes"]:
        pre = bytes.fromhex(r["preimage"])
        assert ver.hash_hex(pre) == r["digest"]
        reqs.append((r["timestamp"], bytes.fromhex(r["clientID"]), bytes.fromhex(r["operation"]), r["sequenceID"]))
    got = ver.digest_request_batch(reqs)
    want = [r["digest"] for r in digest_kats["requests"] + digest_kats["escapes"]]
    assert [g.tobytes().hex() for g in got] == want


def test_vote_and_reply_digests(ver, digest_kats):
    votes = [(v["viewID"], v["sequenceID"], bytes.fromhex(v["digest"]), bytes.fromhex(v["nodeID"]), v["msgType"])
             for v in digest_kats["votes"]]
    got = ver.digest_vote_batch(votes)
    assert [g.tobytes().hex() for g in got] == [v["digest_of_preimage"] for v in digest_kats["votes"]]
    reps = [(r["viewID"], r["timestamp"], bytes.fromhex(r["clientID"]), bytes.fromhex(r["nodeID"]),
             bytes.fromhex(r["result"])) for r in digest_kats["replies"]]
    got = ver.digest_reply_batch(reps)
    assert [g.tobytes().hex() for g in got] == [r["digest_of_preimage"] for r in digest_kats["replies"]]


def test_sha256_dev_api(ver):
    rng = np.random.default_rng(11)
    msgs = [rng.bytes(int(l)) for l in rng.integers(256, 4097, 2048)]
    blob, off, ln = ver.pack(msgs)
    n = len(msgs)
    d_data = ver.to_device(0, blob, pad=16)
    d_off = ver.to_device(0, off)
    d_len = ver.to_device(0, ln)
    d_ord = ver.alloc(0, 4 * n)
    d_dig = ver.alloc(0, 32 * n)
    exp = np.array([list(hashlib.sha256(m).digest()) for m in msgs], np.uint8)
    exp[::3, 0] ^= 1
    d_exp = ver.to_device(0, exp)
    d_bm = ver.alloc(0, (n + 31) // 32 * 4)
    ver.sha256_order_dev(0, d_len.ptr, n, d_ord.ptr)
    ver.sha256_batch_dev(0, d_data.ptr, d_off.ptr, d_len.ptr, d_ord.ptr, n, d_dig.ptr, d_exp.ptr, d_bm.ptr)
    ver.sync(0)
    order = d_ord.to_host(dtype=np.uint32)
    assert sorted(order.tolist()) == list(range(n))
    nb = (ln.astype(np.int64) + 8) // 64 + 1
    assert (np.diff(nb[order]) <= 0).all(), "order must group by descending block count"
    got = d_dig.to_host().reshape(-1, 32)
    for i, m in enumerate(msgs):
        assert got[i].tobytes() == hashlib.sha256(m).digest()
    bits = np.unpackbits(d_bm.to_host(), bitorder="little")[:n].astype(bool)
    assert (bits == (np.arange(n) % 3 != 0)).all()
    for b in (d_data, d_off, d_len, d_ord, d_dig, d_exp, d_bm):
        b.free()


# ------------------------------------------------------------------ ECDSA
def test_ecdsa_empty_batches(ver, ecdsa_fixtures):
    """n = 0 on every signature entry point: an empty bitmap, no error, no
    launch; the quorum check counts 0 accepted (quorum 1 fails, quorum 0
    holds); a following batch is unaffected."""
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    ver.register_keys(keys)
    z32, z64, zk = np.zeros((0, 32), np.uint8), np.zeros((0, 64), np.uint8), np.zeros(0, np.uint32)
    assert ver.verify_batch(z32, z64, zk).shape == (0,)
    bm, acc, ok = ver.qc_verify(z32, z64, zk, quorum=1)
    assert bm.shape == (0,) and acc == 0 and not ok
    assert ver.qc_verify(z32, z64, zk, quorum=0)[2]
    d = ver.alloc(0, 64)
    try:
        ver.verify_batch_dev(0, d.ptr, d.ptr, d.ptr, 0, d.ptr)
        ver.sync(0)
    finally:
        d.free()
    assert (ver.verify_batch(hashes, sigs, kidx) == expect).all()


def test_register_keys_validity(ver, ecdsa_fixtures):
    keys, *_ = fixture_arrays(ecdsa_fixtures)
    valid = ver.register_keys(keys)
    assert valid.tolist() == [k["valid"] for k in ecdsa_fixtures["keys"]]


def test_ecdsa_fixtures(ver, ecdsa_fixtures, path):
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    ver.register_keys(keys)
    got = ver.verify_batch(hashes, sigs, kidx)
    bad = [(ecdsa_fixtures["vectors"][i]["kind"], bool(got[i])) for i in np.nonzero(got != expect)[0]]
    assert not bad, bad


def test_ecdsa_fixtures_every_alignment(ver, ecdsa_fixtures, path):
    """Same vectors at every position of a wave / bitmap byte."""
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    ver.register_keys(keys)
    for shift in (1, 7, 63):
        h = np.concatenate([hashes[:shift], hashes])
        s = np.concatenate([sigs[:shift], sigs])
        k = np.concatenate([kidx[:shift], kidx])
        e = np.concatenate([expect[:shift], expect])
        assert (ver.verify_batch(h, s, k) == e).all()


def test_ecdsa_random_vs_oracle(ver, oracle_lib, path):
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=16, per_key=64, seed=99)
    rng = np.random.default_rng(5)
    n = len(kidx)
    # corrupt a third of them in assorted ways
    c = rng.integers(0, 6, n)
    sel = rng.random(n) < 0.33
    for i in np.nonzero(sel)[0]:
        kind = c[i]
        if kind == 0:
            sigs[i, rng.integers(0, 32)] ^= 1 << rng.integers(0, 8)
        elif kind == 1:
            sigs[i, 32 + rng.integers(0, 32)] ^= 1 << rng.integers(0, 8)
        elif kind == 2:
            hashes[i, rng.integers(0, 32)] ^= 1 << rng.integers(0, 8)
        elif kind == 3:
            kidx[i] = (kidx[i] + 1) % 16
        elif kind == 4:
            sigs[i, :32] = 0
        else:
            sigs[i, 32:] = 0xFF
    ver.register_keys(keys)
    got = ver.verify_batch(hashes, sigs, kidx)
    want = np.zeros((n + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n].astype(bool)
    assert (got == want).all()
    assert want.sum() > n // 2


@pytest.mark.parametrize("k", [1, 2, 4, 8, 16])
def test_ecdsa_scalar_batch_sizes(ver, oracle_lib, ecdsa_fixtures, k, monkeypatch):
    """The batched-inversion scalar kernel for every K (signatures per lane),
    with valid / corrupted / out-of-range signatures mixed inside each batch."""
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    reps = 9
    H, S, K, E = (np.tile(hashes, (reps, 1)), np.tile(sigs, (reps, 1)), np.tile(kidx, reps), np.tile(expect, reps))
    monkeypatch.setenv("PBFTV_SCALAR_BATCH", str(k))
    monkeypatch.setenv("PBFTV_WAVE_MAX", "0")
    ver.register_keys(keys)
    got = ver.verify_batch(H, S, K)
    assert (got == E).all()


def test_ecdsa_large_tiled_property(ver, oracle_lib):
    """262,144 signatures (tiles of an oracle-signed pool) with 1 % corrupted at
    known positions: the accept bitmap must be exactly the complement of the
    corruption mask (size-independent property; multi-shard / many waves)."""
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=8, per_key=64, seed=123)
    reps = 262144 // len(kidx)
    H = np.tile(hashes, (reps, 1))
    S = np.tile(sigs, (reps, 1))
    K = np.tile(kidx, reps)
    rng = np.random.default_rng(8)
    bad = rng.random(len(K)) < 0.01
    idx = np.nonzero(bad)[0]
    S[idx, 63] ^= 1
    ver.register_keys(keys)
    got = ver.verify_batch(H, S, K)
    assert (got == ~bad).all()


@pytest.mark.parametrize("sort", ["0", "1"])
def test_ecdsa_key_order(ver, oracle_lib, sort, monkeypatch):
    """The lane path with and without the key-order stage (k_key_* + k_pack_bits):
    shuffled signatures of 24 keys, a ragged count, corruptions, out-of-range
    key indices and an invalid registered key, against the oracle."""
    monkeypatch.setenv("PBFTV_WAVE_MAX", "0")
    monkeypatch.setenv("PBFTV_KEY_SORT", sort)
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=24, per_key=125, seed=77)
    rng = np.random.default_rng(78)
    o = rng.permutation(len(kidx))[:2999]
    hashes, sigs, kidx = hashes[o].copy(), sigs[o].copy(), kidx[o].copy()
    n = len(kidx)
    sel = rng.random(n) < 0.2
    sigs[sel, 40] ^= 0x08
    kidx[rng.random(n) < 0.02] = 24 + rng.integers(0, 1000)   # no such key
    keys = keys.copy()
    keys[5, 63] ^= 1                                           # key 5 off the curve: its signatures fail
    ver.register_keys(keys)
    got = ver.verify_batch(hashes, sigs, kidx)
    want = np.zeros((n + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n].astype(bool)
    assert (got == want).all()
    assert want.sum() > n // 2


def test_ecdsa_key_order_large_property(ver, oracle_lib):
    """The default large-batch path (key order on: > 8 keys, n >= 32768): 131,072
    tiled signatures of 100 keys in random order, 1 % corrupted at known
    positions -- the bitmap must be the complement of the corruption mask."""
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=100, per_key=8, seed=321)
    reps = 131072 // len(kidx) + 1
    rng = np.random.default_rng(9)
    o = rng.permutation(reps * len(kidx))[:131072] % len(kidx)
    H, S, K = hashes[o], sigs[o].copy(), kidx[o]
    bad = rng.random(len(K)) < 0.01
    S[np.nonzero(bad)[0], 31] ^= 2
    ver.register_keys(keys)
    got = ver.verify_batch(H, S, K)
    assert (got == ~bad).all()


def test_ecdsa_no_keys_and_out_of_range(ecdsa_fixtures):
    from simple_pbft_amd import PBFTV_ENOKEYS, PbftvError, Verifier
    with Verifier() as v:
        keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
        with pytest.raises(PbftvError) as ei:
            v.verify_batch(hashes[:3], sigs[:3], kidx[:3])
        assert ei.value.code == PBFTV_ENOKEYS
        v.register_keys(keys[:2])
        k = np.full(len(kidx), 5, np.uint32)
        assert not v.verify_batch(hashes, sigs, k).any()


def test_qc_verify(ver, oracle_lib, path):
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=4, per_key=3, seed=4)
    ver.register_keys(keys)
    bm, acc, ok = ver.qc_verify(hashes, sigs, kidx, quorum=3)
    assert bm.all() and acc == 12 and ok
    sigs[:10, 40] ^= 1
    bm, acc, ok = ver.qc_verify(hashes, sigs, kidx, quorum=3)
    assert acc == 2 and not ok and bm.tolist() == [False] * 10 + [True] * 2


def test_ecdsa_dev_api(ver, ecdsa_fixtures, path):
    from simple_pbft_amd.pbftv import K_ECDSA_COMB, K_ECDSA_WAVE
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    ver.register_keys(keys)
    n = len(kidx)
    dh = ver.to_device(0, hashes)
    ds = ver.to_device(0, sigs)
    dk = ver.to_device(0, kidx)
    db = ver.alloc(0, (n + 7) // 8)
    ver.set_kernel_timing(True)
    ver.reset_kernel_times()
    ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr)
    ver.sync(0)
    ms, cnt = ver.kernel_time_ms(0, K_ECDSA_WAVE if path == "wave" else K_ECDSA_COMB)
    ver.set_kernel_timing(False)
    assert cnt == 1 and ms > 0
    got = np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool)
    assert (got == expect).all()
    for b in (dh, ds, dk, db):
        b.free()


def test_ecdsa_wave_path_edge_counts(ver, oracle_lib, monkeypatch):
    """The wave path at batch sizes around its 8-signature blocks and at the
    default threshold, against the oracle (1 in 5 corrupted)."""
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=6, per_key=400, seed=31)
    sigs[::5, 33] ^= 0x40
    ver.register_keys(keys)
    n_all = len(kidx)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n_all,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)
    for n in (1, 2, 7, 8, 9, 15, 16, 17, 67, 2047, 2048, 2049, 2400):
        got = ver.verify_batch(hashes[:n], sigs[:n], kidx[:n])
        assert (got == want[:n]).all(), n


# ---- host-buffer pipeline (pbftv_api.cpp verify_host_pipelined) ------------
@pytest.mark.parametrize("chunk", ["512", "4096", "262144"])
@pytest.mark.parametrize("layout", ["default", "one_stream", "short_tail"])
def test_host_pipeline_chunks_pageable_and_pinned(ver, oracle_lib, chunk, layout, monkeypatch):
    """The chunked host-buffer path (DMA into device slots -> verify, even and
    odd chunks on two verify streams, key indices copied up front) at chunk
    sizes that give 1, a few and many chunks, a ragged tail, from pageable numpy
    memory and from pbftv_host_alloc memory, against the corruption mask (1 %)
    and the oracle on a sample.  one_stream: the round-2 layout (one verify
    stream, keys copied per chunk); short_tail: a 1024-signature last chunk."""
    monkeypatch.setenv("PBFTV_HOST_CHUNK", chunk)
    if layout == "one_stream":
        monkeypatch.setenv("PBFTV_HOST_2COMPUTE", "0")
        monkeypatch.setenv("PBFTV_HOST_KEYS_FIRST", "0")
    if layout == "short_tail":
        monkeypatch.setenv("PBFTV_HOST_LAST", "1024")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=16, per_key=32, seed=55)
    n = 40_000 + 123
    rng = np.random.default_rng(56)
    o = rng.integers(0, len(kidx), n)
    H, S, K = hashes[o].copy(), sigs[o].copy(), kidx[o].copy()
    bad = rng.random(n) < 0.01
    S[np.nonzero(bad)[0], 50] ^= 4
    ver.register_keys(keys)
    got = ver.verify_batch(H, S, K)
    assert (got == ~bad).all()
    pins = [ver.pinned(a) for a in (H, S, K)]
    try:
        got2 = ver.verify_batch(*(p.a for p in pins))
        assert (got2 == got).all()
    finally:
        for p in pins:
            p.free()
    m = 3000
    want = np.zeros((m + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, m, keys.ctypes.data,
                                              len(keys), want.ctypes.data, 8)
    assert (np.unpackbits(want, bitorder="little")[:m].astype(bool) == got[:m]).all()


@pytest.mark.parametrize("chunk", ["4096", "262144"])
def test_host_pipeline_concurrent_callers(ver, oracle_lib, chunk, monkeypatch):
    """Concurrent host-buffer calls on one context (a Go node's pools flushing
    at once; the cgo pattern of tests/cpp/test_cgo_pattern.cpp, here on the
    chunked large-batch path): three threads, different batch sizes and
    corruption masks, pageable and pinned inputs, many chunks (4096) and few
    (262144), so device slots, key and bitmap buffers are reused call after
    call: every call's bitmap must be its own batch's."""
    import threading
    monkeypatch.setenv("PBFTV_HOST_CHUNK", chunk)
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=16, per_key=32, seed=61)
    ver.register_keys(keys)
    rng = np.random.default_rng(62)
    jobs = []
    for t, n in enumerate((30_000 + 77, 52_224, 12_289)):
        o = rng.integers(0, len(kidx), n)
        H, S, K = hashes[o].copy(), sigs[o].copy(), kidx[o].copy()
        bad = rng.random(n) < (0.01, 0.2, 0.5)[t]
        S[np.nonzero(bad)[0], 33] ^= 8
        jobs.append((H, S, K, ~bad))
    pins = [ver.pinned(a) for a in jobs[1][:3]]
    jobs[1] = (*(p.a for p in pins), jobs[1][3])
    errors = []

    def run(job):
        try:
            for _ in range(6):
                got = ver.verify_batch(*job[:3])
                if not (got == job[3]).all():
                    errors.append(int((got != job[3]).sum()))
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append(repr(e))

    try:
        th = [threading.Thread(target=run, args=(j,)) for j in jobs]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=120)
        assert not any(x.is_alive() for x in th)
        assert errors == []
    finally:
        for p in pins:
            p.free()


def test_dev_calls_on_two_streams_share_scratch(ver, oracle_lib, monkeypatch):
    """*_dev calls on a caller stream and on the context stream reuse
    the device scratch (scalars, flags, key order); the scratch event orders
    them.  Two different batches enqueued back to back on two streams must both
    come out right."""
    monkeypatch.setenv("PBFTV_WAVE_MAX", "0")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=12, per_key=16, seed=57)
    ver.register_keys(keys)
    n = 65536
    rng = np.random.default_rng(58)
    bufs, masks = [], []
    for t in range(2):
        o = rng.integers(0, len(kidx), n)
        H, S, K = hashes[o].copy(), sigs[o].copy(), kidx[o].copy()
        bad = rng.random(n) < (0.02 if t == 0 else 0.3)
        S[np.nonzero(bad)[0], 20] ^= 1
        bufs.append((ver.to_device(0, H), ver.to_device(0, S), ver.to_device(0, K), ver.alloc(0, n // 8)))
        masks.append(~bad)
    side = ver.stream_create(0)
    try:
        for _ in range(3):
            (h0, s0, k0, b0), (h1, s1, k1, b1) = bufs
            ver.verify_batch_dev(0, h0.ptr, s0.ptr, k0.ptr, n, b0.ptr, stream=side)
            ver.verify_batch_dev(0, h1.ptr, s1.ptr, k1.ptr, n, b1.ptr)
            ver.sync(0)
            ver.stream_wait(0, side)
            for (_, _, _, b), want in zip(bufs, masks):
                got = np.unpackbits(b.to_host(), bitorder="little")[:n].astype(bool)
                assert (got == want).all()
    finally:
        ver.stream_destroy(0, side)
        for tup in bufs:
            for b in tup:
                b.free()


# ---- the armed latency kernel (pbftv_api.cpp qc_arm / k_ecdsa_wave_armed) ----
def test_armed_path_golden_and_crafted(ecdsa_fixtures):
    """Every golden vector (valid, high-S, the corruption classes, e >= n,
    R.x >= n, invalid keys, the crafted doubling / cancellation sums) and the
    chosen-scalar exceptional sums, served in calls of 1-8 signatures (the
    armed kernel's mailbox slots) and of 9-128 (one launch of the latency
    kernel reading the mailbox arrays) -- against the fixtures' expected bits."""
    from conftest import crafted_exceptional
    from simple_pbft_amd import Verifier
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    rng = np.random.default_rng(79)
    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        o = rng.permutation(len(kidx))
        at = 0
        while at < len(o):
            m = int(rng.choice([1, 2, 3, 5, 8, 9, 13, 24, 67, 128]))
            sel = o[at:at + m]
            got = v.verify_batch(hashes[sel], sigs[sel], kidx[sel])
            bad = [ecdsa_fixtures["vectors"][i]["kind"] for i, g in zip(sel, got) if g != expect[i]]
            assert not bad, bad
            at += m
        key, H, S, K, E = crafted_exceptional()
        v.register_keys(key)
        for a in range(0, len(K), 4):
            assert (v.verify_batch(H[a:a + 4], S[a:a + 4], K[a:a + 4]) == E[a:a + 4]).all(), a
        assert (v.verify_batch(H, S, K) == E).all()  # all of them in one call (past the slots when > 8)



@pytest.mark.parametrize("mode", ["keeper", "expiring"])
def test_armed_latency_path(oracle_lib, mode, monkeypatch):
    """Small host-buffer batches are served by the persistent armed kernel
    (doorbell in host memory).  Consecutive calls of every size up to the
    mailbox capacity and past it, a key change while armed, and pauses longer
    than the armed kernel's budget: with the keeper (mode "keeper", 20 ms
    budget) the kernel is replaced before it runs out and every small call is
    still served armed; without it (PBFTV_QC_KEEP_MS=0, 1 ms budget) the armed
    kernel expires during each pause and the request must fall back to a
    launch (pbftv_qc_stamps says which served it).  Every bitmap against the
    oracle."""
    import time
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_ARM_MS", "20" if mode == "keeper" else "1")
    if mode == "expiring":
        monkeypatch.setenv("PBFTV_QC_KEEP_MS", "0")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=5, per_key=60, seed=77)
    sigs[::7, 45] ^= 0x20
    n_all = len(kidx)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n_all,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)
    rng = np.random.default_rng(78)
    served = []
    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        for it, n in enumerate([1, 3, 3, 67, 128, 129, 300, 2, 64, 5, 127, 1, 3, 8, 4, 7]):
            o = rng.choice(n_all, n, replace=False)
            got = v.verify_batch(hashes[o], sigs[o], kidx[o])
            assert (got == want[o]).all(), (it, n)
            if (n <= 8 and it > 0) or (8 < n <= 128 and it > 3):
                served.append((it, n, v.qc_stamps(0)["armed"]))
            time.sleep(0.06)  # three budgets (keeper) / sixty (expiring)
        if mode == "keeper":
            # the keeper kept one armed through every pause -- after the first
            # 67-signature call a WIDE one, with a workgroup per signature of
            # the largest wide certificate so far (rounded up to 8): a larger
            # one is launched once and the next arming is wider
            wide_max, expect = 67, []
            for it, n, a in served:
                if 8 < n <= 128 and n > (wide_max + 7) // 8 * 8:
                    expect.append((it, n, False))
                else:
                    expect.append((it, n, True))
                if 8 < n <= 128:
                    wide_max = max(wide_max, n)
            assert served == expect, [(x, y) for x, y in zip(served, expect) if x != y]
        else:
            assert not any(a for _, _, a in served), served  # every one expired: launched instead
        # a key change while a kernel is armed: it is cancelled first
        assert v.set_key(0, keys[0])
        o = rng.choice(n_all, 3, replace=False)
        assert (v.verify_batch(hashes[o], sigs[o], kidx[o]) == want[o]).all()
        armed = 0
        for _ in range(200):  # back to back, the quorum count too
            o = rng.choice(n_all, 3, replace=False)
            bm, acc, ok = v.qc_verify(hashes[o], sigs[o], kidx[o], quorum=3)
            assert (bm == want[o]).all() and acc == int(want[o].sum()) and ok == bool(want[o].all())
            armed += v.qc_stamps(0)["armed"]
        assert armed >= (190 if mode == "keeper" else 0)


def test_armed_slots_follow_certificate_size(oracle_lib, monkeypatch):
    """The narrow row-schedule server arms one workgroup per slot: as many
    slots as the largest certificate of the last period, at least 4.  A
    7-signature certificate after 3-signature ones is served by a launch (the
    armed kernel has 4 slots) and re-arms with 7 at once, so the next 7s are
    armed; every bitmap and quorum count against the oracle, with corrupted
    votes in every certificate."""
    import time
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_WIDE", "0")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=8, per_key=12, seed=91)
    sigs[::4, 50] ^= 0x04
    n_all = len(kidx)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n_all,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)
    rng = np.random.default_rng(92)
    served = []
    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        for it, n in enumerate([3, 3, 3, 7, 7, 7, 7, 2, 8, 8, 1]):
            o = rng.choice(n_all, n, replace=False)
            bm, acc, ok = v.qc_verify(hashes[o], sigs[o], kidx[o], quorum=n)
            assert (bm == want[o]).all() and acc == int(want[o].sum()), (it, n)
            served.append((it, n, v.qc_stamps(0)["armed"]))
            time.sleep(0.005)
    armed = {it: a for it, _, a in served}
    assert all(armed[it] for it in (1, 2)), served        # 3 <= 4 slots
    assert not armed[3], served                             # 7 > 4: launched, re-armed wider
    assert all(armed[it] for it in (4, 5, 6, 7)), served  # 7 slots now
    assert not armed[8] and armed[9] and armed[10], served  # 8 > 7: once launched


def test_wide_arming_is_kept_by_the_keeper(oracle_lib, monkeypatch):
    """a wide arming takes as many workgroups as the
    largest recent wide certificate (72 for 67 votes), and the keeper used to
    compare that SIZE with 128 to decide whether to reshape -- so it rotated
    a freshly armed wide server at once and on every wake.  The keeper now
    compares the SHAPE.  Right after the call that armed the wide kernel, wide
    certificates back to back are served by it (once all its workgroups are
    resident) with no further arming or rotation; every bit vs the oracle."""
    import time
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_ARM_MS", "4000")  # (no timed rotation within the test)
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=5, per_key=30, seed=93)
    sigs[::6, 44] ^= 0x10
    n_all = len(kidx)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n_all,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)
    rng = np.random.default_rng(94)

    def call(n):
        o = rng.choice(n_all, n, replace=False)
        assert (v.verify_batch(hashes[o], sigs[o], kidx[o]) == want[o]).all()
        return v.qc_stamps(0)["armed"]

    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        call(3)
        call(3)
        assert not call(67)  # launched; the call path arms the wide kernel
        c0 = v.qc_counters(0)
        assert c0["armed_wide"] and c0["armed_waves"] == 72, c0
        t0 = time.monotonic()
        while not call(67):  # launched until every workgroup is resident
            assert time.monotonic() - t0 < 2.0, v.qc_counters(0)
        time.sleep(0.02)     # the keeper has woken since
        for _ in range(2):
            assert call(67)
        c1 = v.qc_counters(0)
        assert (c1["armings"], c1["rotations"]) == (c0["armings"], c0["rotations"]), (c0, c1)
        assert c1["armed_wide"] and c1["armed_waves"] == 72


def test_split_wide_certificates(oracle_lib, monkeypatch):
    """PBFTV_QC_WIDE=split: no wide server is armed; a certificate of 9..128
    signatures puts its first signatures into the armed narrow slots and the
    rest into one launch beside them (pbftv_qc_counters: served armed, one
    launch, no rerun), and the narrow server stays armed.  Corrupted votes in
    every certificate; every bit against the oracle."""
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_WIDE", "split")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=5, per_key=60, seed=95)
    sigs[::5, 33] ^= 0x02
    n_all = len(kidx)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n_all,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)
    rng = np.random.default_rng(96)
    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        for n in (3, 3):
            o = rng.choice(n_all, n, replace=False)
            assert (v.verify_batch(hashes[o], sigs[o], kidx[o]) == want[o]).all()
        for n in (9, 20, 67, 67, 128, 100):
            o = rng.choice(n_all, n, replace=False)
            c0 = v.qc_counters(0)
            assert (v.verify_batch(hashes[o], sigs[o], kidx[o]) == want[o]).all(), n
            c1 = v.qc_counters(0)
            assert c1["armed"] - c0["armed"] == 1, (n, c0, c1)
            assert c1["launches"] - c0["launches"] == (1 if n > c0["armed_waves"] else 0), (n, c0, c1)
            assert c1["reruns"] == c0["reruns"] and not c1["armed_wide"], (n, c0, c1)


def test_armed_kernel_does_not_hold_frees_or_other_contexts(oracle_lib, monkeypatch):
    """An armed kernel with a 5-s budget stays resident between calls.  A
    device free and a pinned-host free neither wait for it nor stop it
    (VERDICT r5 item 6): pbftv_dev_alloc memory comes from a stream-ordered
    pool and its free is queued behind the context's streams (no hipFree),
    pinned blocks go back to a cache (no hipHostFree) -- so both contexts'
    servers keep serving right after (pbftv_qc_counters).  Another context's
    key change waits only for its OWN work (ctx_quiesce)."""
    import time
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_ARM_MS", "5000")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=4, per_key=20, seed=81)
    sigs[::5, 40] ^= 0x08
    n_all = len(kidx)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n_all,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)

    def call(v, i):
        assert (v.verify_batch(hashes[i:i + 3], sigs[i:i + 3], kidx[i:i + 3]) == want[i:i + 3]).all(), i
        return v.qc_stamps(0)["armed"]

    with Verifier(device_mask=1) as a, Verifier(device_mask=1) as b:
        a.register_keys(keys)
        b.register_keys(keys)
        for v in (a, b):
            for i in range(0, 12, 3):
                call(v, i)
            # (another context of this process -- the module's `ver` -- may hold
            # a high-priority stream pair; it gives it up within ~0.2 s of idling)
            t_end = time.perf_counter() + 3.0
            while not call(v, 0) and time.perf_counter() < t_end:
                time.sleep(0.01)
            assert call(v, 0)
        c0 = {id(v): v.qc_counters(0) for v in (a, b)}
        for it in range(20):
            t0 = time.perf_counter()
            buf = a.alloc(0, 1 << 20)
            assert time.perf_counter() - t0 < 0.05, ("alloc", it)
            t0 = time.perf_counter()
            buf.free()
            assert time.perf_counter() - t0 < 0.05, ("free", it)
            t0 = time.perf_counter()
            pin = a.pinned(np.zeros(1 << 16, np.uint8))
            assert time.perf_counter() - t0 < 0.05, ("pinned", it)
            t0 = time.perf_counter()
            pin.free()
            assert time.perf_counter() - t0 < 0.05, ("pinned free", it)
            for v in (a, b):  # served by the same armed servers, right after the frees
                t0 = time.perf_counter()
                assert call(v, 12), (it, v is a, time.perf_counter() - t0, v.qc_counters(0))
        for v in (a, b):
            c1 = v.qc_counters(0)
            assert c1["armed"] - c0[id(v)]["armed"] == 20 and c1["launches"] == c0[id(v)]["launches"], (c0[id(v)], c1)
        t0 = time.perf_counter()
        assert b.set_key(1, keys[1])  # b's key change with a's kernel armed (b waits for b's work only)
        assert time.perf_counter() - t0 < 2.0
        assert call(a, 15)  # (a's server was not stopped by it)
        for i in range(24, n_all - 3, 3):
            for v in (a, b):
                call(v, i)


def test_armed_stream_pairs_shared_out(oracle_lib, monkeypatch):
    """The runtime keeps GPU_MAX_HW_QUEUES (4) high-priority hardware queues
    per GPU: a fifth high-priority stream shares one, and a kernel launched
    there waits for the resident armed kernel's whole budget
    (profiles/r06_hiq_share.txt; before the fix, a third armed context in one
    process made certificates wait seconds).  Three contexts (beside the
    module's) with 5-s budgets: no certificate waits, every bitmap is right,
    at most GPU_MAX_HW_QUEUES / 2 contexts are armed at once, and the one that
    keeps calling is served armed once the idle ones give a pair up."""
    import os
    import time
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_ARM_MS", "5000")
    cap = int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) // 2
    if cap == 0:
        pytest.skip("GPU_MAX_HW_QUEUES < 2: the library arms no server")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=3, per_key=12, seed=83)
    sigs[::4, 45] ^= 0x20
    n_all = len(kidx)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n_all,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)

    def call(v, i):
        t0 = time.perf_counter()
        assert (v.verify_batch(hashes[i:i + 3], sigs[i:i + 3], kidx[i:i + 3]) == want[i:i + 3]).all(), i
        dt = time.perf_counter() - t0
        assert dt < 0.5, (i, dt)  # (a queue shared with a resident 5-s kernel: seconds)
        return v.qc_stamps(0)["armed"]

    with Verifier(device_mask=1) as a, Verifier(device_mask=1) as b, Verifier(device_mask=1) as c:
        ctxs = (a, b, c)
        for v in ctxs:
            v.register_keys(keys)
        for rnd in range(8):
            for j, v in enumerate(ctxs):
                call(v, 3 * ((rnd + j) % (n_all // 3)))
            assert sum(v.qc_counters(0)["armed_waves"] > 0 for v in ctxs) <= cap
        # a and b idle, c keeps calling: an idle holder gives its pair up
        t_end = time.perf_counter() + 3.0
        while not call(c, 0) and time.perf_counter() < t_end:
            time.sleep(0.01)
        assert call(c, 3)
        assert sum(v.qc_counters(0)["armed_waves"] > 0 for v in ctxs) <= cap
        for v in ctxs:  # every context still right, armed or launched
            for i in range(0, n_all - 2, 3):
                call(v, i)


def test_armed_kernels_of_two_contexts_concurrent(oracle_lib):
    """Two contexts on one GPU, each with its own armed server and keeper,
    called from two threads at once with certificates of 1-129 signatures
    (narrow, wide and launched), while a third thread runs lane-path batches
    on the first context: every bitmap against the oracle, and both contexts
    served most certificates armed (pbftv_qc_stamps)."""
    import threading
    from simple_pbft_amd import Verifier
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=6, per_key=100, seed=91)
    sigs[::9, 50] ^= 0x04
    n_all = len(kidx)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n_all,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)
    errors, armed = [], {}
    with Verifier(device_mask=1) as a, Verifier(device_mask=1) as b:
        a.register_keys(keys)
        b.register_keys(keys)

        def certs(name, v, seed):
            rng = np.random.default_rng(seed)
            got_armed = 0
            try:
                for it in range(150):
                    n = int(rng.choice([1, 3, 3, 4, 8, 67, 100, 129]))
                    o = rng.choice(n_all, n, replace=False)
                    got = v.verify_batch(hashes[o], sigs[o], kidx[o])
                    if not (got == want[o]).all():
                        errors.append((name, it, n))
                    got_armed += v.qc_stamps(0)["armed"]
            except Exception as e:  # noqa: BLE001 -- reported by the main thread
                errors.append((name, repr(e)))
            armed[name] = got_armed

        def lanes():
            rng = np.random.default_rng(7)
            try:
                for it in range(6):
                    o = rng.choice(n_all, 4096, replace=True)
                    with_path = a.verify_batch(hashes[o], sigs[o], kidx[o])
                    if not (with_path == want[o]).all():
                        errors.append(("lanes", it))
            except Exception as e:  # noqa: BLE001
                errors.append(("lanes", repr(e)))

        ts = [threading.Thread(target=certs, args=("a", a, 1)), threading.Thread(target=certs, args=("b", b, 2)),
              threading.Thread(target=lanes)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in ts), "a caller thread hung"
    assert not errors, errors[:5]
    assert armed["a"] >= 60 and armed["b"] >= 60, armed


def test_armed_exclusive_cu_option(oracle_lib, monkeypatch):
    """PBFTV_QC_EXCLUSIVE_CU=1: the armed workgroups take their CUs' whole LDS
    (no batch block shares their SIMDs).  Certificates narrow and wide are
    still served armed and right, also while a lane-path batch runs."""
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_EXCLUSIVE_CU", "1")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=5, per_key=80, seed=95)
    sigs[::6, 37] ^= 0x10
    n_all = len(kidx)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n_all,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)
    rng = np.random.default_rng(96)
    armed = 0
    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        for it, n in enumerate([3, 3, 4, 67, 67, 100, 3, 8, 1] * 4):
            o = rng.choice(n_all, n, replace=False)
            assert (v.verify_batch(hashes[o], sigs[o], kidx[o]) == want[o]).all(), (it, n)
            armed += v.qc_stamps(0)["armed"]
        o = rng.choice(n_all, 5000)
        assert (v.verify_batch(hashes[o], sigs[o], kidx[o]) == want[o]).all()  # a batch beside the armed CUs
        for it in range(10):
            o = rng.choice(n_all, 3, replace=False)
            assert (v.verify_batch(hashes[o], sigs[o], kidx[o]) == want[o]).all(), it
    assert armed >= 24, armed


def _corrupted_certs(oracle_lib, per_cert, n_certs, seed, rng):
    """n_certs certificates of per_cert votes by a 100-key committee (OpenSSL,
    tools/synth.py), every one with 1-3 votes corrupted (a flipped bit of r, s
    or the hash), so neither an all-accept nor an all-reject answer passes and
    consecutive certificates differ in which votes fail.  Expected bits: oracle."""
    import os
    import sys
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth
    pub, H, S, K = synth.certs(100, per_cert, n_certs, seed)
    H = H.copy()
    for c in range(n_certs):
        for j in rng.choice(per_cert, int(rng.integers(1, min(3, per_cert - 1) + 1)), replace=False):
            i = c * per_cert + int(j)
            col = int(rng.integers(0, 96))
            (S[i] if col < 64 else H[i])[col % 64 if col < 64 else col - 64] ^= np.uint8(1 << int(rng.integers(0, 8)))
    n = len(K)
    bm = np.zeros((n + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, n, pub.ctypes.data,
                                              len(pub), bm.ctypes.data, 8)
    want = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    assert 0 < want.reshape(n_certs, per_cert).sum(1).min() and want.reshape(n_certs, per_cert).all(1).sum() == 0
    return pub, [(H[c * per_cert:(c + 1) * per_cert], S[c * per_cert:(c + 1) * per_cert],
                  K[c * per_cert:(c + 1) * per_cert], want[c * per_cert:(c + 1) * per_cert]) for c in range(n_certs)]


@pytest.mark.parametrize("mode", ["keeper", "expiring"])
def test_rekey_then_wide_certificates(oracle_lib, mode, monkeypatch):
    """The sequence of round 4's on-hardware false reject (gpurun_out/r04a:
    0 of 67 accepted on the first 67-signature certificate after a new key
    set): register key set A (100 keys) -> 67-signature certificates, back to
    back and after 1-s idle gaps -> register key set B (100 keys, same
    geometry: the key-table slots are reused in place) -> 3-signature
    certificates served armed -> 67- and 129-signature certificates -> 3 again.
    Every certificate carries corrupted votes; every bitmap against the oracle,
    and each quorum count.  "expiring": no keeper and a 300-ms budget, so the
    1-s gaps find the armed kernel gone (the round-3 library's behaviour at
    the reference's tick)."""
    import time
    from simple_pbft_amd import Verifier
    if mode == "expiring":
        monkeypatch.setenv("PBFTV_QC_KEEP_MS", "0")
        monkeypatch.setenv("PBFTV_QC_ARM_MS", "300")
    rng = np.random.default_rng(505)
    pubA, a67 = _corrupted_certs(oracle_lib, 67, 24, 201, rng)
    pubB, b3 = _corrupted_certs(oracle_lib, 3, 70, 0x50424654, rng)
    pubB2, b67 = _corrupted_certs(oracle_lib, 67, 30, 0x50424654, rng)
    assert (pubB == pubB2).all() and not (pubA == pubB).all()
    # 129 signatures (past the armed kernel's 128 waves): two certificates' votes in one call
    b129 = [tuple(np.concatenate([x[j], y[j][:62]]) for j in range(4)) for x, y in zip(b67[24::2], b67[25::2])]
    b67 = b67[:24]
    bad = []
    armed = {"b3": 0}

    def serve(v, label, calls, gap=0.0):
        for i, (H, S, K, want) in enumerate(calls):
            if gap:
                time.sleep(gap)
            bm, acc, ok = v.qc_verify(H, S, K, quorum=len(K))
            if not ((bm == want).all() and acc == int(want.sum()) and not ok):
                bad.append((label, i, len(K), int(acc), int(want.sum())))
            if label.startswith("B3"):
                armed["b3"] += v.qc_stamps(0)["armed"]

    with Verifier(device_mask=1) as v:
        v.register_keys(pubA)
        serve(v, "A67", a67[:20])
        serve(v, "A67_tick", a67[20:22], gap=1.0)
        serve(v, "A67_after", a67[22:])
        time.sleep(0.5)
        v.register_keys(pubB)
        serve(v, "B3", b3[:20])
        serve(v, "B3_gap2ms", b3[20:60], gap=0.002)
        serve(v, "B67", b67)
        serve(v, "B129", b129)
        serve(v, "B3_after", b3[60:])
    assert not bad, bad[:10]
    assert armed["b3"] >= 50, armed  # the 3-signature certificates were served by the armed kernel


def test_external_device_sync_bounded_by_budget(oracle_lib, monkeypatch):
    """A hipDeviceSynchronize made OUTSIDE the library (the caller's own HIP
    code) while the keeper holds an armed kernel on the GPU waits for that
    kernel: the wait is bounded by its budget (PBFTV_QC_ARM_MS; the keeper
    rotates at half of it), documented as ~1.5 budgets.  With a 200-ms budget
    the sync must return within 2 budgets plus slack, and later certificates
    are still served right."""
    import ctypes
    import time
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_ARM_MS", "200")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=4, per_key=12, seed=83)
    sigs[::4, 33] ^= 0x02
    n_all = len(kidx)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n_all,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)
    hip = ctypes.CDLL("libamdhip64.so")  # the runtime libpbftv.so already loaded (same soname)
    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        waits = []
        for rep in range(3):
            for i in range(0, 12, 3):
                assert (v.verify_batch(hashes[i:i + 3], sigs[i:i + 3], kidx[i:i + 3]) == want[i:i + 3]).all()
            assert v.qc_stamps(0)["armed"]
            time.sleep(0.03 * rep)
            t0 = time.perf_counter()
            assert hip.hipDeviceSynchronize() == 0
            waits.append(time.perf_counter() - t0)
        assert max(waits) < 2 * 0.2 + 0.15, waits
        for i in range(12, n_all - 3, 3):
            assert (v.verify_batch(hashes[i:i + 3], sigs[i:i + 3], kidx[i:i + 3]) == want[i:i + 3]).all(), i


def test_quiesce_during_rotations(oracle_lib, monkeypatch):
    """a quiesce (another context's device free bumps the halt word
    of every mailbox on the GPU) can land while a rotation has two armed
    kernels resident; both leave at once.  Each armed stream slot has its own
    expired word, so the owner sees its CURRENT kernel's exit and serves the
    next certificate with a launch instead of ringing a kernel that is gone.
    A 40-ms budget makes the keeper rotate every 20 ms while a second context
    frees device memory in a loop: every certificate right, none slow."""
    import threading
    import time
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_ARM_MS", "40")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=5, per_key=40, seed=87)
    sigs[::6, 21] ^= 0x40
    n_all = len(kidx)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n_all,
                                              keys.ctypes.data, len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)
    stop = threading.Event()
    frees = [0]
    with Verifier(device_mask=1) as a, Verifier(device_mask=1) as b:
        a.register_keys(keys)

        def freer():
            while not stop.is_set():
                buf = b.alloc(0, 1 << 16)
                buf.free()
                frees[0] += 1
                time.sleep(0.003)
        th = threading.Thread(target=freer)
        th.start()
        rng = np.random.default_rng(88)
        slow, wrong = [], []
        try:
            t_end = time.perf_counter() + 3.0
            it = 0
            while time.perf_counter() < t_end:
                m = int(rng.choice([1, 3, 4, 8, 67]))
                o = rng.choice(n_all, m, replace=False)
                t0 = time.perf_counter()
                got = a.verify_batch(hashes[o], sigs[o], kidx[o])
                dt = time.perf_counter() - t0
                if dt > 0.5:
                    slow.append((it, m, dt))
                if not (got == want[o]).all():
                    wrong.append((it, m))
                it += 1
                time.sleep(float(rng.choice([0.0, 0.005, 0.02])))
        finally:
            stop.set()
            th.join()
    assert not wrong, wrong[:5]
    assert not slow, slow[:5]
    assert frees[0] > 100 and it > 100, (frees[0], it)


def test_caller_sync_memcpy_not_held_by_armed_kernel(oracle_lib, monkeypatch):
    """A caller's synchronous hipMemcpy (the null stream) on the GPU while the
    keeper holds an armed kernel: the armed kernels run on the highest-priority
    streams, which HIP keeps on hardware queues of their own, so the copy does
    not wait for the resident kernel (on a normal-priority stream it waited the
    whole budget: tools/queue_share.hip).  5-s budget, so a wait would show."""
    import ctypes
    import time
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_ARM_MS", "5000")
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=3, per_key=8, seed=85)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        for i in range(0, 9, 3):
            assert v.verify_batch(hashes[i:i + 3], sigs[i:i + 3], kidx[i:i + 3]).all()
        assert v.qc_stamps(0)["armed"]
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), 4096) == 0
        host = np.zeros(4096, np.uint8)
        try:
            for kind in (1, 2):  # hipMemcpyHostToDevice, hipMemcpyDeviceToHost
                t0 = time.perf_counter()
                assert hip.hipMemcpy(p if kind == 1 else host.ctypes.data, host.ctypes.data if kind == 1 else p,
                                     4096, kind) == 0
                assert time.perf_counter() - t0 < 0.2, kind
        finally:
            v.close()  # (the free quiesces the armed kernel first)
            hip.hipFree(p)


@pytest.mark.parametrize("mode", ["yield", "launched"])
def test_certificates_beside_a_batch(oracle_lib, mode, monkeypatch):
    """Certificates while a large batch runs on the context's own stream:
    "yield" (PBFTV_QC_YIELD=1): the batch enqueue halts the armed kernel, the
    certificate is launched meanwhile, and the keeper arms again once the batch
    is expected done; "launched" (PBFTV_QC_ARM=0): every certificate is a
    launch.  Either way the launch goes to the latency stream, never behind the
    batch queued on the context stream: it returns long before the batch
    (several ms of queued work) has finished.  Every bitmap against the oracle."""
    import time
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_YIELD" if mode == "yield" else "PBFTV_QC_ARM", "1" if mode == "yield" else "0")
    monkeypatch.setenv("PBFTV_GBITS", "24")
    monkeypatch.setenv("PBFTV_QBITS", "16")
    keys, H, S, K = oracle_sign_pool(oracle_lib, 4, 16, seed=93)
    S[::5, 9] ^= 0x08
    n_all = len(K)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, n_all, keys.ctypes.data,
                                              len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)
    n = 1 << 20
    reps = n // n_all
    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        dh, ds, dk = (v.to_device(0, np.tile(a, (reps, 1)) if a.ndim > 1 else np.tile(a, reps)) for a in (H, S, K))
        db = v.alloc(0, n // 8 + 1)
        try:
            for i in range(0, 9, 3):  # idle: armed (yield) or launched
                assert (v.verify_batch(H[i:i + 3], S[i:i + 3], K[i:i + 3]) == want[i:i + 3]).all()
            for _ in range(6):  # ~6 ms of queued work on the context stream
                v.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr)
            t0 = time.perf_counter()
            got = v.verify_batch(H[9:12], S[9:12], K[9:12])
            dt = time.perf_counter() - t0
            assert (got == want[9:12]).all()
            assert not v.qc_stamps(0)["armed"]  # halted (yield) or never armed
            assert dt < 3e-3, dt  # not behind the six queued batches
            v.sync(0)
            assert (np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool) == np.tile(want, reps)).all()
            if mode == "yield":
                time.sleep(0.05)  # past the batches' expected end: the keeper arms again
                for i in range(12, 30, 3):
                    assert (v.verify_batch(H[i:i + 3], S[i:i + 3], K[i:i + 3]) == want[i:i + 3]).all()
                assert v.qc_stamps(0)["armed"]
        finally:
            for b in (dh, ds, dk, db):
                b.free()


@pytest.mark.parametrize("cu_yield", ["1", "2"])
def test_cu_yield_certificates_during_batches(oracle_lib, cu_yield, monkeypatch):
    """The CU yield (PBFTV_QC_CU_YIELD; 2 also parks the instruction-cache
    partner CU): with the narrow server held resident (PBFTV_QC_YIELD=0),
    device-resident 1M batches on a library stream read their CU's certificate
    word every comb step and park while an armed workgroup there serves.
    Certificates served meanwhile by the armed server, and the batches' bitmap,
    all against the oracle; the batches finish (a raised word parks a comb wave
    at most 50 us)."""
    import threading
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_QC_YIELD", "0")
    monkeypatch.setenv("PBFTV_QC_CU_YIELD", cu_yield)
    monkeypatch.setenv("PBFTV_GBITS", "24")
    monkeypatch.setenv("PBFTV_QBITS", "16")
    keys, H, S, K = oracle_sign_pool(oracle_lib, 4, 16, seed=97)
    S[::5, 9] ^= 0x08
    n_all = len(K)
    want = np.zeros((n_all + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, n_all, keys.ctypes.data,
                                              len(keys), want.ctypes.data, 8)
    want = np.unpackbits(want, bitorder="little")[:n_all].astype(bool)
    n = 1 << 20
    reps = n // n_all
    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        dh, ds, dk = (v.to_device(0, np.tile(a, (reps, 1)) if a.ndim > 1 else np.tile(a, reps)) for a in (H, S, K))
        db = v.alloc(0, n // 8 + 1)
        st = v.stream_create(0)
        try:
            for i in range(0, 12, 3):  # arm the narrow server
                assert (v.verify_batch(H[i:i + 3], S[i:i + 3], K[i:i + 3]) == want[i:i + 3]).all()
            before = v.qc_counters(0)
            stop = threading.Event()
            done = [0]

            def stream():
                while not stop.is_set():
                    v.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr, stream=st)
                    v.stream_wait(0, st)
                    done[0] += 1
            th = threading.Thread(target=stream)
            th.start()
            try:
                calls = 0
                while done[0] < 4 or calls < 40:
                    i = 3 * (calls % (n_all // 3))
                    assert (v.verify_batch(H[i:i + 3], S[i:i + 3], K[i:i + 3]) == want[i:i + 3]).all()
                    calls += 1
            finally:
                stop.set()
                th.join()
            after = v.qc_counters(0)
            assert after["armed"] - before["armed"] >= calls // 2  # served by the resident server
            assert (np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool) == np.tile(want, reps)).all()
        finally:
            db.free()
            v.stream_destroy(0, st)
            for b in (dh, ds, dk):
                b.free()
