"""Wire format of signed votes and the host-side DER parse of
a10: the product (C ABI, csrc/der.cpp + gojson_enc.h) against the oracle
restatements (oracle/der.py: go1.19 ecdsa.VerifyASN1 over cryptobyte;
oracle/gojson.py: encodeByteSlice = base64.StdEncoding, nil -> null).
Parity pinned by restatement only (no Go here): "parity unpinned" against
Go itself, cross-checked on the DER side by the GPU test that feeds
re-encoded fixture signatures through the verify."""
from __future__ import annotations

import os
import random
import subprocess

import numpy as np
import pytest

from oracle import der as der_ref
from oracle import gojson

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551


@pytest.fixture(scope="module")
def pb():
    from simple_pbft_amd import pbftv
    if not os.path.exists(pbftv.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "simple_pbft_amd"), "-j8"], check=True)
    return pbftv


def test_vote_signed_matches_restatement(pb):
    rng = random.Random(0x50424654)
    for _ in range(300):
        dg = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 70)))
        nid = rng.choice([b"Apple", b"MS", b"Google", b"IBM", b"<n\x00d\xe2\x80\xa8>"])
        sig = None if rng.random() < 0.1 else bytes(rng.randrange(256) for _ in range(rng.randrange(0, 80)))
        v, s, mt = rng.randrange(-5, 1 << 40), rng.randrange(-(1 << 62), 1 << 62), rng.randrange(0, 3)
        want = gojson.vote_signed(v, s, dg, nid, mt, sig)
        assert pb.gojson_vote_signed(v, s, dg, nid, mt, sig) == want
        # the signing preimage is the unsigned VoteMsg, a strict prefix of the wire form
        assert want.startswith(pb.gojson_vote(v, s, dg, nid, mt)[:-1])


def test_vote_signed_known_answer(pb):
    # base64.StdEncoding KATs (RFC 4648 §10) inside the field; nil vs empty
    for raw, enc in [(b"", b'""'), (b"f", b'"Zg=="'), (b"fo", b'"Zm8="'), (b"foo", b'"Zm9v"'),
                     (b"foob", b'"Zm9vYg=="'), (b"fooba", b'"Zm9vYmE="'), (b"foobar", b'"Zm9vYmFy"'),
                     (None, b"null"), (b"\xfb\xff", b'"+/8="')]:
        got = pb.gojson_vote_signed(0, 1, b"d", b"MS", 1, raw)
        assert got == b'{"viewID":0,"sequenceID":1,"digest":"d","nodeID":"MS","msgType":1,"signature":' + enc + b"}"


def _rand_bytes(rng, lo=0, hi=40):
    return bytes(rng.randrange(256) for _ in range(rng.randrange(lo, hi)))


def _rand_sig(rng):
    return None if rng.random() < 0.15 else _rand_bytes(rng, 0, 80)


def test_other_signed_messages_match_restatement(pb):
    """Signed RequestMsg / ReplyMsg / PrePrepareMsg wire forms
    against oracle/gojson.py, and the signing preimage is the unsigned encoding
    (a strict prefix of the wire form)."""
    rng = random.Random(0x5349474E)
    for _ in range(200):
        ts, seq = rng.randrange(-(1 << 62), 1 << 62), rng.randrange(-(1 << 62), 1 << 62)
        cid, op, res = _rand_bytes(rng), _rand_bytes(rng), _rand_bytes(rng)
        nid = rng.choice([b"Apple", b"MS", b"<n\x00d\xe2\x80\xa8>"])
        sig, rsig = _rand_sig(rng), _rand_sig(rng)
        want = gojson.request_signed(ts, cid, op, seq, sig)
        assert pb.gojson_request_signed(ts, cid, op, seq, sig) == want
        assert want.startswith(pb.gojson_request(ts, cid, op, seq)[:-1])
        view = rng.randrange(-5, 1 << 40)
        want = gojson.reply_signed(view, ts, cid, nid, res, sig)
        assert pb.gojson_reply_signed(view, ts, cid, nid, res, sig) == want
        assert want.startswith(pb.gojson_reply(view, ts, cid, nid, res)[:-1])
        req = None if rng.random() < 0.2 else (ts, cid, op, seq)
        dg = _rand_bytes(rng, 0, 70)
        want = gojson.preprepare_signed(view, seq, dg, req, rsig, sig)
        assert pb.gojson_preprepare_signed(view, seq, dg, req, rsig, sig) == want
        # the primary's preimage embeds the unsigned request
        assert pb.gojson_preprepare(view, seq, dg, req) == gojson.preprepare(view, seq, dg, req)


def test_signed_messages_known_answer(pb):
    assert pb.gojson_request_signed(1668519246, b"client1", b"printf", 0, b"foo") == (
        b'{"timestamp":1668519246,"clientID":"client1","operation":"printf","sequenceID":0,"signature":"Zm9v"}')
    assert pb.gojson_reply_signed(0, 5, b"c", b"MS", b"Executed", None) == (
        b'{"viewID":0,"timestamp":5,"clientID":"c","nodeID":"MS","result":"Executed","signature":null}')
    assert pb.gojson_preprepare_signed(0, 7, b"ab", (1, b"c", b"o", 7), b"f", b"fo") == (
        b'{"viewID":0,"sequenceID":7,"digest":"ab","requestMsg":{"timestamp":1,"clientID":"c","operation":"o",'
        b'"sequenceID":7,"signature":"Zg=="},"signature":"Zm8="}')
    assert pb.gojson_preprepare_signed(0, 7, b"ab", None, b"f", b"") == (
        b'{"viewID":0,"sequenceID":7,"digest":"ab","requestMsg":null,"signature":""}')


def _malformed():
    good = der_ref.encode(0x1234, N - 1)
    body = good[2:]
    return [
        b"", b"\x30", b"\x30\x00", b"\x30\x02\x02\x00",
        good + b"\x00",                                   # trailing data after the SEQUENCE
        b"\x30" + bytes([len(body) + 3]) + body + b"\x02\x01\x01",  # a third INTEGER
        b"\x31" + good[1:],                               # SET, not SEQUENCE
        b"\x3f" + good[1:],                               # high-tag-number form
        b"\x30\x80" + body + b"\x00\x00",                 # indefinite length
        b"\x30\x81" + bytes([len(body)]) + body,          # long form for a length < 128
        b"\x30\x82\x00" + bytes([len(body)]) + body,      # leading zero length byte
        b"\x30\x85\x00\x00\x00\x00" + bytes([len(body)]) + body,  # 5 length bytes
        b"\x30\x06\x02\x00\x02\x02\x00\x01",              # empty INTEGER
        b"\x30\x07\x02\x02\x00\x01\x02\x01\x01",          # non-minimal 00 lead
        b"\x30\x07\x02\x02\xff\x80\x02\x01\x01",          # non-minimal ff lead
        b"\x30\x06\x02\x01\x80\x02\x01\x01",              # negative r
        b"\x30\x06\x02\x01\x00\x02\x01\x01",              # r = 0: parses (Verify rejects later)
        b"\x30\x06\x02\x01\x01\x02\x01\x7f",              # smallest valid shape
        der_ref.encode(1 << 256, 5),                      # r needs 33 value bytes
        der_ref.encode((1 << 256) - 1, (1 << 255)),       # max 32-byte values with 00 lead
        good[:-1],                                        # truncated
    ]


def test_der_edge_cases(pb):
    for d in _malformed():
        assert pb.der_to_rs(d) == der_ref.to_rs(d), d.hex()
    assert pb.der_to_rs(b"\x30\x06\x02\x01\x00\x02\x01\x01") == bytes(32) + (1).to_bytes(32, "big")


def test_der_random_and_mutated(pb):
    rng = random.Random(7)
    for _ in range(2000):
        r = rng.choice([rng.randrange(1, N), rng.randrange(1, 1 << rng.randrange(1, 257)), N - 1, 1, 0x80])
        s = rng.choice([rng.randrange(1, N), rng.randrange(1, 1 << 64), 1 << 255])
        d = der_ref.encode(r, s)
        assert pb.der_to_rs(d) == r.to_bytes(32, "big") + s.to_bytes(32, "big")
        m = bytearray(d)
        for _ in range(rng.randrange(1, 3)):
            op = rng.randrange(3)
            if op == 0 and m:
                m[rng.randrange(len(m))] ^= 1 << rng.randrange(8)
            elif op == 1 and m:
                del m[rng.randrange(len(m))]
            else:
                m.insert(rng.randrange(len(m) + 1), rng.randrange(256))
        assert pb.der_to_rs(bytes(m)) == der_ref.to_rs(bytes(m)), bytes(m).hex()


def test_der_batch(pb):
    ders = _malformed() + [der_ref.encode(i + 1, N - 1 - i) for i in range(50)]
    rs, parsed = pb.der_to_rs_batch(ders)
    want = [der_ref.to_rs(d) for d in ders]
    assert parsed == sum(w is not None for w in want)
    for row, w in zip(rs, want):
        assert row.tobytes() == (w if w is not None else bytes(64))
    rs0, p0 = pb.der_to_rs_batch([])
    assert p0 == 0 and rs0.shape == (0, 64)


@pytest.mark.gpu
def test_der_fixtures_through_verify(ecdsa_fixtures):
    """Golden signatures re-encoded as DER -> host parse -> GPU verify: same bits
    as the fixtures' r||s (the parse is exact for every in-range r, s)."""
    from conftest import fixture_arrays
    from simple_pbft_amd import Verifier, pbftv
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    ders = []
    for row in sigs:
        r, s = int.from_bytes(row[:32].tobytes(), "big"), int.from_bytes(row[32:].tobytes(), "big")
        ders.append(der_ref.encode(r, s))
    rs, _ = pbftv.der_to_rs_batch(ders)
    v = Verifier()
    try:
        v.register_keys(keys)
        got = v.verify_batch(hashes, np.ascontiguousarray(rs), kidx)
    finally:
        v.close()
    assert (got == expect).all()
