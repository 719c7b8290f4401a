"""GPU parity of the device-side Go-JSON message path and the
pool flush (pbftv_flush_votes: Go-JSON + SHA-256 + verifyMsg + ECDSA in one
round trip), through the C ABI, against the oracle: Go-JSON restated in
oracle/gojson.py (pinned by the reference's logged preimages, test_oracle.py),
FIPS SHA-256 (hashlib), the oracle's textbook ECDSA verify, and its verifyMsg.
Bit-exact for every digest and every bit."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import fixture_arrays
from oracle import gojson

pytestmark = pytest.mark.gpu

N_ORDER = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551

# byte strings that exercise every encodeState.string branch (escapes, HTML,
# valid multi-byte runes, U+2028/9, invalid / truncated / overlong / surrogate
# sequences)
ALPHABET = [b"x", b"Z", b"0", b"<", b">", b"&", b'"', b"\\", b"\t", b"\n", b"\r", b"\x00", b"\x01", b"\x1f",
            b"\x7f", b"\xe2\x80\xa8", b"\xe2\x80\xa9", b"\xff", b"\xc2\xa2", b"\xe0\x9f\xbf", b"\xe0\xa0\x80",
            b"\xf0\x90\x80\x80", b"\xf4\x8f\xbf\xbf", b"\xf4\x90\x80\x80", b"\xef\xbf\xbd", b"\xe2\x82",
            b"\xc0\x80", b"\xed\xa0\x80", b"\x80", b"\xf5"]
INT_EDGES = [0, 1, -1, 9, 10, 99, 100, -10, 2 ** 63 - 1, -2 ** 63, -2 ** 63 + 1, 10 ** 18, 10 ** 18 - 1, -10 ** 18,
             1668519247222762700]


@pytest.fixture(scope="module")
def ver():
    from simple_pbft_amd import Verifier
    v = Verifier()
    yield v
    v.close()


@pytest.fixture(params=["wave", "lane"])
def path(request, monkeypatch):
    monkeypatch.setenv("PBFTV_WAVE_MAX", "100000000" if request.param == "wave" else "0")
    return request.param


def rand_str(rng, maxlen=12):
    if rng.integers(0, 3) == 0:
        return rng.bytes(int(rng.integers(0, maxlen)))
    return b"".join(ALPHABET[i] for i in rng.integers(0, len(ALPHABET), rng.integers(0, maxlen)))


def rand_int(rng):
    if rng.integers(0, 3) == 0:
        return INT_EDGES[int(rng.integers(0, len(INT_EDGES)))]
    return int(rng.integers(-2 ** 63, 2 ** 63 - 1))


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def hexes(a) -> list[str]:
    return [x.tobytes().hex() for x in a]


@pytest.mark.parametrize("n", [1, 7, 64, 65, 1000, 5000])
def test_device_gojson_digests_vs_oracle(ver, n):
    rng = np.random.default_rng(n)
    reqs = [(rand_int(rng), rand_str(rng), rand_str(rng), rand_int(rng)) for _ in range(n)]
    assert hexes(ver.digest_request_batch(reqs)) == [sha(gojson.request(*r)) for r in reqs]
    votes = [(rand_int(rng), rand_int(rng), rand_str(rng, 70), rand_str(rng), int(rng.integers(0, 2)))
             for _ in range(n)]
    assert hexes(ver.digest_vote_batch(votes)) == [sha(gojson.vote(*v)) for v in votes]
    reps = [(rand_int(rng), rand_int(rng), rand_str(rng), rand_str(rng), rand_str(rng, 40)) for _ in range(n)]
    assert hexes(ver.digest_reply_batch(reps)) == [sha(gojson.reply(*r)) for r in reps]
    pps = [(rand_int(rng), rand_int(rng), rand_str(rng, 70), reqs[i] if rng.integers(0, 4) else None)
           for i in range(n)]
    assert hexes(ver.digest_preprepare_batch(pps)) == [sha(gojson.preprepare(*p)) for p in pps]


def test_device_gojson_fixtures_and_empty(ver, digest_kats):
    """The reference's logged requests and the committed vote/reply KATs through
    the device encoder; an empty batch is a no-op."""
    reqs = [(r["timestamp"], bytes.fromhex(r["clientID"]), bytes.fromhex(r["operation"]), r["sequenceID"])
            for r in digest_kats["requests"] + digest_kats["escapes"]]
    assert hexes(ver.digest_request_batch(reqs)) == [r["digest"] for r in digest_kats["requests"] +
                                                     digest_kats["escapes"]]
    pps = [(p["viewID"], p["sequenceID"], bytes.fromhex(p["digest"]),
            None if p["request"] is None else (p["request"][0], bytes.fromhex(p["request"][1]),
                                               bytes.fromhex(p["request"][2]), p["request"][3]))
           for p in digest_kats["preprepares"]]
    assert hexes(ver.digest_preprepare_batch(pps)) == [sha(bytes.fromhex(p["preimage"]))
                                                       for p in digest_kats["preprepares"]]
    assert ver.digest_vote_batch([]).shape[0] == 0
    assert ver.digest_preprepare_batch([]).shape[0] == 0


def _sign(oracle_lib, h: bytes, priv: bytes, rng) -> bytes:
    out = np.zeros(64, np.uint8)
    while True:
        if oracle_lib.oracle_ecdsa_p256_sign(h, priv, rng.bytes(32), out.ctypes.data):
            return out.tobytes()


@pytest.mark.parametrize("n", [3, 67, 700])
def test_flush_votes_vs_oracle(ver, oracle_lib, path, n):
    from simple_pbft_amd.pbftv import VoteColumns
    rng = np.random.default_rng(1000 + n)
    n_keys = 5
    privs, keys = [], np.zeros((n_keys, 64), np.uint8)
    for k in range(n_keys):
        d = int.from_bytes(rng.bytes(32), "big") % (N_ORDER - 1) + 1
        privs.append(d.to_bytes(32, "big"))
        assert oracle_lib.oracle_p256_pubkey(privs[-1], keys[k].ctypes.data) == 1
    assert ver.register_keys(keys).all()
    # states: several sequences in flight (sequence-keyed pools)
    k_states = 6
    s_view = np.array([10, 10, 11, 10, 12, 10], np.int64)
    s_last = np.array([-1, 5, -1, 100, 7, -1], np.int64)
    s_dig = np.frombuffer(rng.bytes(32 * k_states), np.uint8).reshape(k_states, 32).copy()
    votes, sidx, kidx, sigs = [], [], [], []
    for i in range(n):
        st = int(rng.integers(0, k_states + 1))  # k_states = out of range
        sd = s_dig[min(st, k_states - 1)].tobytes().hex().encode()
        kind = int(rng.integers(0, 8))
        view = int(s_view[min(st, k_states - 1)]) + (1 if kind == 1 else 0)
        seq = int(rng.integers(0, 200))
        dg = [sd, sd, sd.upper(), sd[:-1], sd + b"0", rand_str(rng, 64), sd, sd][kind]
        node = b"node%d" % int(rng.integers(0, n_keys))
        v = (view, seq, dg, node, int(rng.integers(0, 2)))
        key = int(rng.integers(0, n_keys))
        sig = _sign(oracle_lib, hashlib.sha256(gojson.vote(*v)).digest(), privs[key], rng)
        corrupt = int(rng.integers(0, 6))
        if corrupt == 0:
            sig = bytes([sig[0] ^ 1]) + sig[1:]
        elif corrupt == 1:
            key = (key + 1) % n_keys
        votes.append(v)
        sidx.append(st)
        kidx.append(key)
        sigs.append(sig)
    cols = VoteColumns(votes)
    S = np.frombuffer(b"".join(sigs), np.uint8).reshape(n, 64)
    K = np.array(kidx, np.uint32)
    dg, sig_ok, msg_ok = ver.flush_votes(cols, S, K, (s_view, s_last, s_dig), np.array(sidx, np.uint32))
    pre = [gojson.vote(*v) for v in votes]
    H = np.frombuffer(b"".join(hashlib.sha256(p).digest() for p in pre), np.uint8).reshape(n, 32)
    assert hexes(dg) == [sha(p) for p in pre]
    want_bm = np.zeros((n + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, n, keys.ctypes.data,
                                              n_keys, want_bm.ctypes.data, 8)
    assert sig_ok.tolist() == np.unpackbits(want_bm, bitorder="little")[:n].astype(bool).tolist()
    want_msg = []
    for (view, seq, d, _, _), st in zip(votes, sidx):
        if st >= k_states:
            want_msg.append(False)
            continue
        want_msg.append(oracle_lib.oracle_verify_msg(int(s_view[st]), int(s_last[st]), s_dig[st].tobytes(), view,
                                                     seq, d, len(d)) == 1)
    assert msg_ok.tolist() == want_msg
    if n >= 67:  # both outcomes present (3 votes may all pass)
        assert sig_ok.any() and not sig_ok.all() and any(want_msg) and not all(want_msg)
    # partial requests: digests only / signatures only
    d2, s2, m2 = ver.flush_votes(cols, S, K, digests=False)
    assert d2 is None and m2 is None and s2.tolist() == sig_ok.tolist()


def test_flush_votes_fixture_signatures(ver, ecdsa_fixtures, path):
    """The committed ECDSA vectors re-checked through the flush entry point's
    signature stage: their hashes are not vote digests, so every bit must be 0
    except where a vector's hash happens to equal its vote's digest (never)."""
    from simple_pbft_amd.pbftv import VoteColumns
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    ver.register_keys(keys)
    n = len(kidx)
    votes = [(0, i, b"%064x" % i, b"node", 0) for i in range(n)]
    _, ok, _ = ver.flush_votes(VoteColumns(votes), sigs, kidx, digests=False)
    assert not ok.any()


def _keys(oracle_lib, rng, n_keys):
    privs, keys = [], np.zeros((n_keys, 64), np.uint8)
    for k in range(n_keys):
        d = int.from_bytes(rng.bytes(32), "big") % (N_ORDER - 1) + 1
        privs.append(d.to_bytes(32, "big"))
        assert oracle_lib.oracle_p256_pubkey(privs[-1], keys[k].ctypes.data) == 1
    return privs, keys


def _signed(oracle_lib, rng, preimages, privs):
    """Sign each preimage with a random key; corrupt some (flipped r, wrong key).
    Returns (sigs n x 64, key_idx, hashes n x 32)."""
    n_keys = len(privs)
    sigs, kidx, hs = [], [], []
    for pre in preimages:
        h = hashlib.sha256(pre).digest()
        key = int(rng.integers(0, n_keys))
        sig = _sign(oracle_lib, h, privs[key], rng)
        c = int(rng.integers(0, 6))
        if c == 0:
            sig = bytes([sig[0] ^ 1]) + sig[1:]
        elif c == 1:
            key = (key + 1) % n_keys
        sigs.append(sig)
        kidx.append(key)
        hs.append(h)
    n = len(preimages)
    return (np.frombuffer(b"".join(sigs), np.uint8).reshape(n, 64).copy(), np.array(kidx, np.uint32),
            np.frombuffer(b"".join(hs), np.uint8).reshape(n, 32).copy())


def _oracle_bits(oracle_lib, H, S, K, keys):
    n = len(K)
    want = np.zeros((n + 7) // 8 + 1, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, n, keys.ctypes.data,
                                              len(keys), want.ctypes.data, 8)
    return np.unpackbits(want, bitorder="little")[:n].astype(bool).tolist()


@pytest.mark.parametrize("n", [3, 67, 700])
def test_flush_requests_vs_oracle(ver, oracle_lib, path, n):
    """Client-signed requests (sequenceID as sent) + StartConsensus digests with
    the assigned sequence IDs, one round trip (pbft_impl.go:67-73)."""
    from simple_pbft_amd.pbftv import RequestColumns
    rng = np.random.default_rng(2000 + n)
    privs, keys = _keys(oracle_lib, rng, 4)
    assert ver.register_keys(keys).all()
    reqs = [(rand_int(rng), rand_str(rng), rand_str(rng, 30), 0 if rng.integers(0, 4) else rand_int(rng))
            for _ in range(n)]
    pre = [gojson.request(*r) for r in reqs]
    S, K, H = _signed(oracle_lib, rng, pre, privs)
    assigned = np.array([rand_int(rng) for _ in range(n)], np.int64)
    dg, ok, cons = ver.flush_requests(RequestColumns(reqs), S, K, assigned)
    assert hexes(dg) == [sha(p) for p in pre]
    assert ok.tolist() == _oracle_bits(oracle_lib, H, S, K, keys)
    assert hexes(cons) == [sha(gojson.request(r[0], r[1], r[2], int(a))) for r, a in zip(reqs, assigned)]
    if n >= 67:
        assert ok.any() and not ok.all()
    d2, s2, c2 = ver.flush_requests(RequestColumns(reqs), S, K, digests=False)
    assert d2 is None and c2 is None and s2.tolist() == ok.tolist()


@pytest.mark.parametrize("n", [3, 67, 700])
def test_flush_replies_vs_oracle(ver, oracle_lib, path, n):
    from simple_pbft_amd.pbftv import ReplyColumns
    rng = np.random.default_rng(3000 + n)
    privs, keys = _keys(oracle_lib, rng, 4)
    assert ver.register_keys(keys).all()
    reps = [(rand_int(rng), rand_int(rng), rand_str(rng), b"node%d" % int(rng.integers(0, 4)),
             [b"Executed", rand_str(rng, 40)][int(rng.integers(0, 2))]) for _ in range(n)]
    pre = [gojson.reply(*r) for r in reps]
    S, K, H = _signed(oracle_lib, rng, pre, privs)
    dg, ok = ver.flush_replies(ReplyColumns(reps), S, K)
    assert hexes(dg) == [sha(p) for p in pre]
    assert ok.tolist() == _oracle_bits(oracle_lib, H, S, K, keys)
    if n >= 67:
        assert ok.any() and not ok.all()


@pytest.mark.parametrize("n", [3, 67, 700])
def test_flush_preprepares_vs_oracle(ver, oracle_lib, path, n):
    """Primary-signed pre-prepares: signature over Go-JSON(PrePrepareMsg), and
    State.PrePrepare's verifyMsg with the embedded request as the state's ReqMsg
    (nil request -> digest of "null"), against several states."""
    from simple_pbft_amd.pbftv import PrePrepareColumns
    rng = np.random.default_rng(4000 + n)
    privs, keys = _keys(oracle_lib, rng, 3)
    assert ver.register_keys(keys).all()
    k_states = 5
    s_view = np.array([0, 0, 3, 0, 7], np.int64)
    s_last = np.array([-1, 50, -1, 1000, 20], np.int64)
    pps, sidx = [], []
    for i in range(n):
        st = int(rng.integers(0, k_states + 1))
        req = None if rng.integers(0, 6) == 0 else (rand_int(rng), rand_str(rng), rand_str(rng, 20),
                                                    int(rng.integers(0, 300)))
        rd = hashlib.sha256(gojson.request_or_null(req)).hexdigest().encode()
        kind = int(rng.integers(0, 7))
        dg = [rd, rd, rd, rd.upper(), rd[:-1], rand_str(rng, 64), rd + b"1"][kind]
        view = int(s_view[min(st, k_states - 1)]) + (1 if rng.integers(0, 8) == 0 else 0)
        seq = req[3] if req is not None and rng.integers(0, 2) else int(rng.integers(0, 2000))
        pps.append((view, seq, dg, req))
        sidx.append(st)
    pre = [gojson.preprepare(*p) for p in pps]
    S, K, H = _signed(oracle_lib, rng, pre, privs)
    dg, rdg, ok, mok = ver.flush_preprepares(PrePrepareColumns(pps), S, K, (s_view, s_last), np.array(sidx, np.uint32),
                                             req_digests=True)
    assert hexes(dg) == [sha(p) for p in pre]
    assert hexes(rdg) == [sha(gojson.request_or_null(p[3])) for p in pps]
    assert ok.tolist() == _oracle_bits(oracle_lib, H, S, K, keys)
    want_msg = []
    for (view, seq, d, req), st in zip(pps, sidx):
        if st >= k_states:
            want_msg.append(False)
            continue
        qd = hashlib.sha256(gojson.request_or_null(req)).digest()
        want_msg.append(oracle_lib.oracle_verify_msg(int(s_view[st]), int(s_last[st]), qd, view, seq, d,
                                                     len(d)) == 1)
    assert mok.tolist() == want_msg
    if n >= 67:
        assert ok.any() and not ok.all() and any(want_msg) and not all(want_msg)
    # digests only (the pbftv_digest_preprepare_batch body) agree
    assert hexes(ver.digest_preprepare_batch(pps)) == hexes(dg)
