"""The oracle pinned against the golden vectors (CPU only).

Pins: FIPS 180-4 examples (SHA-256), the digest preimages rebuilt from the
reference's own logs (log/node1.log), RFC 6979 §A.2.5 published P-256
signatures, and OpenSSL 3.0 libcrypto (an independent ECDSA implementation) on
every committed ECDSA vector."""
from __future__ import annotations

import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, fixture_arrays
from oracle import gojson, openssl_xcheck, p256


def test_sha256_oracle_fips_and_boundaries(oracle_lib, sha_fixtures):
    out = np.zeros(32, np.uint8)
    for v in sha_fixtures:
        m = bytes.fromhex(v["msg"]) if "msg" in v else bytes.fromhex(v["msg_repeat"]["byte"]) * v["msg_repeat"]["count"]
        arr = np.frombuffer(m, np.uint8) if m else np.zeros(1, np.uint8)
        oracle_lib.oracle_sha256(arr.ctypes.data, len(m), out.ctypes.data)
        assert out.tobytes().hex() == v["digest"] == hashlib.sha256(m).hexdigest()
    assert sha_fixtures[0]["digest"] == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"


def test_sha256_oracle_random(oracle_lib):
    rng = np.random.default_rng(1)
    out = np.zeros(32, np.uint8)
    for n in list(range(0, 200)) + [511, 512, 513, 4096]:
        m = rng.bytes(n)
        arr = np.frombuffer(m, np.uint8) if m else np.zeros(1, np.uint8)
        oracle_lib.oracle_sha256(arr.ctypes.data, n, out.ctypes.data)
        assert out.tobytes() == hashlib.sha256(m).digest()


def test_hash_hex_is_utils_hash(oracle_lib):
    buf = __import__("ctypes").create_string_buffer(65)
    oracle_lib.oracle_hash_hex(b"abc", 3, buf)
    assert buf.value.decode() == hashlib.sha256(b"abc").hexdigest()  # lowercase hex, utils.go:16


def test_digest_kats_from_reference_logs(digest_kats):
    want = {"client1": "a63fc9e814525ac811f0ee3adcbe17bc46a58b828b8e1e07aa214f839f7365a9",
            "client2": "e5485d99d877dc5b37daf4a69c51f3b8c6501b5ffcce86ca77d5a80f365c13e4",
            "client3": "982077e48ed4e9a84ee74d5d35f4666e7fb5196169c8f75df1ca031d0563179a"}
    for r in digest_kats["requests"]:
        pre = gojson.request(r["timestamp"], bytes.fromhex(r["clientID"]), bytes.fromhex(r["operation"]),
                             r["sequenceID"])
        assert pre.hex() == r["preimage"]
        assert len(pre) == 99
        assert hashlib.sha256(pre).hexdigest() == want[bytes.fromhex(r["clientID"]).decode()]
    assert bytes.fromhex(digest_kats["requests"][0]["preimage"]) == (
        b'{"timestamp":1668519246,"clientID":"client1","operation":"printf","sequenceID":1668519247222762700}')


def _c_request(L, ts, cid, op, seq):
    n = L.oracle_gojson_request(ts, cid, len(cid), op, len(op), seq, None, 0)
    buf = np.zeros(max(n, 1), np.uint8)
    L.oracle_gojson_request(ts, cid, len(cid), op, len(op), seq, buf.ctypes.data, n)
    return buf[:n].tobytes()


def test_gojson_c_and_python_restatements_agree(oracle_lib, digest_kats):
    for r in digest_kats["requests"] + digest_kats["escapes"]:
        cid, op = bytes.fromhex(r["clientID"]), bytes.fromhex(r["operation"])
        c = _c_request(oracle_lib, r["timestamp"], cid, op, r["sequenceID"])
        assert c.hex() == r["preimage"] == gojson.request(r["timestamp"], cid, op, r["sequenceID"]).hex()
    rng = np.random.default_rng(2)
    alphabet = [b"a", b"<", b">", b"&", b'"', b"\\", b"\n", b"\x00", b"\x7f", b"\xe2\x80\xa8", b"\xe2\x80\xa9",
                b"\xff", b"\xc3\xa9", b"\xed\xa0\x80", b"\xf0\x9f\x98\x80", b"\xe2\x82", b"\xf4\x90\x80\x80"]
    for _ in range(500):
        s = b"".join(alphabet[i] for i in rng.integers(0, len(alphabet), rng.integers(0, 12)))
        s2 = rng.bytes(int(rng.integers(0, 10)))
        assert _c_request(oracle_lib, -5, s, s2, 7) == gojson.request(-5, s, s2, 7)


def test_gojson_escape_rules():
    assert gojson.string(b"<a&b>") == b'"\\u003ca\\u0026b\\u003e"'
    assert gojson.string(b'"\\\n\r\t') == b'"\\"\\\\\\n\\r\\t"'
    assert gojson.string(b"\x01\x1f") == b'"\\u0001\\u001f"'
    assert gojson.string(b"\x08\x0c") == b'"\\u0008\\u000c"'          # go1.19: no \b \f short forms
    assert gojson.string("  ".encode()) == b'"\\u2028\\u2029"'
    assert gojson.string(b"\xff") == b'"\\ufffd"'
    assert gojson.string(b"\xed\xa0\x80") == b'"\\ufffd\\ufffd\\ufffd"'  # surrogates are invalid UTF-8
    assert gojson.string("é✓😀".encode()) == '"é✓😀"'.encode()
    assert gojson.vote(1, 2, b"d", b"n", 1) == b'{"viewID":1,"sequenceID":2,"digest":"d","nodeID":"n","msgType":1}'
    assert gojson.preprepare(1, 2, b"d", None) == b'{"viewID":1,"sequenceID":2,"digest":"d","requestMsg":null}'


def test_verify_msg_oracle(oracle_lib):
    d = hashlib.sha256(b"req").digest()
    hx = d.hex().encode()
    V = oracle_lib.oracle_verify_msg
    assert V(10, -1, d, 10, 5, hx, 64) == 1
    assert V(10, -1, d, 11, 5, hx, 64) == 0          # wrong view (pbft_impl.go:178)
    assert V(10, 5, d, 10, 5, hx, 64) == 0           # last >= seq (pbft_impl.go:184-188)
    assert V(10, 4, d, 10, 5, hx, 64) == 1
    assert V(10, -1, d, 10, 5, hx.upper(), 64) == 0  # Go string compare is exact
    assert V(10, -1, d, 10, 5, hx + b"0", 65) == 0


def test_rfc6979_published_vectors():
    x = 0xC9AFA9D845BA75166B5C215767B1D6934E50C3DB36E89B127B8A622B120F6721
    q = p256.pubkey(x)
    assert q == (0x60FED4BA255A9D31C961EB74C6356D68C049B8923B61FA6CE669622E60F29FB6,
                 0x7903FE1008B8BC99A41AE9E95628BC64F2F1B20C2D7E9F5177A3C294D4462299)
    assert p256.verify(p256.sha256(b"sample"), 0xEFD48B2AACB6A8FD1140DD9CD45E81D69D2C877B56AAF991C34D0EA84EAF3716,
                       0xF7CB1C942D657C41D436C7A1B6E29F65F3E900DBB9AFF4064DC4AB2F843ACDA8, *q)


def test_ecdsa_c_oracle_on_fixtures(oracle_lib, ecdsa_fixtures):
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    n = len(kidx)
    bm = np.zeros((n + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n,
                                              keys.ctypes.data, len(keys), bm.ctypes.data, 4)
    got = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    assert (got == expect).all()
    for j, k in enumerate(ecdsa_fixtures["keys"]):
        assert bool(oracle_lib.oracle_p256_key_valid(keys[j].ctypes.data)) == k["valid"]


@pytest.mark.skipif(not openssl_xcheck.available(), reason="libcrypto missing")
def test_ecdsa_fixtures_pinned_by_openssl(ecdsa_fixtures):
    keys = ecdsa_fixtures["keys"]
    for v in ecdsa_fixtures["vectors"]:
        k = v["key"]
        if k >= len(keys):
            assert not v["expect"]
            continue
        qx, qy = int(keys[k]["x"], 16), int(keys[k]["y"], 16)
        r, s = int(v["r"], 16), int(v["s"], 16)
        h = bytes.fromhex(v["hash"])
        assert openssl_xcheck.ecdsa_verify(h, r, s, qx, qy) == v["expect"], v["kind"]


def test_python_restatement_on_fixture_subset(ecdsa_fixtures):
    keys = ecdsa_fixtures["keys"]
    for v in ecdsa_fixtures["vectors"][::7]:
        k = v["key"]
        if k >= len(keys):
            continue
        got = p256.verify(bytes.fromhex(v["hash"]), int(v["r"], 16), int(v["s"], 16), int(keys[k]["x"], 16),
                          int(keys[k]["y"], 16))
        assert got == v["expect"], v["kind"]


def test_oracle_sign_roundtrip(oracle_lib):
    d = (123456789).to_bytes(32, "big")
    pub = np.zeros(64, np.uint8)
    assert oracle_lib.oracle_p256_pubkey(d, pub.ctypes.data)
    h = hashlib.sha256(b"x").digest()
    sig = np.zeros(64, np.uint8)
    assert oracle_lib.oracle_ecdsa_p256_sign(h, d, (987654321).to_bytes(32, "big"), sig.ctypes.data)
    assert oracle_lib.oracle_ecdsa_p256_verify(h, sig.ctypes.data, pub.ctypes.data) == 1
    assert openssl_xcheck.ecdsa_verify(h, int.from_bytes(sig[:32].tobytes(), "big"),
                                       int.from_bytes(sig[32:].tobytes(), "big"),
                                       int.from_bytes(pub[:32].tobytes(), "big"),
                                       int.from_bytes(pub[32:].tobytes(), "big"))


def test_openssl_standin_threads_match_fixtures(ecdsa_fixtures):
    """The multi-threaded OpenSSL stand-in CPU baseline (oracle/openssl_standin.c,
    bench.py's cpu_openssl_standin) gives the golden accept bits at 1 and 4 threads."""
    import ctypes
    so = os.path.join(ROOT, "oracle", "libopenssl_standin.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    L = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    L.standin_ecdsa_p256_verify_batch.restype = ctypes.c_int64
    L.standin_ecdsa_p256_verify_batch.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint32, vp, ctypes.c_int]
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    n = len(kidx)
    for threads in (1, 4):
        bm = np.zeros((n + 7) // 8, np.uint8)
        acc = L.standin_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n,
                                                keys.ctypes.data, len(keys), bm.ctypes.data, threads)
        got = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
        assert (got == expect).all() and acc == expect.sum()
