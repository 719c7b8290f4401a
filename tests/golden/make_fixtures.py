#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root:  python tests/golden/make_fixtures.py

Every vector is produced by the pure-Python restatement (oracle/p256.py,
hashlib) and cross-checked against OpenSSL 3.0 libcrypto -- an independent
implementation -- before it is written; generation aborts on any
disagreement.  The reference itself (Go) cannot be built or run here
(SURVEY.md §8(c)), so these are the pins:

* sha256.json       -- FIPS 180-4 examples + padding-boundary lengths.
* digest_kats.json  -- the digest preimages of the reference's own logged
                       run (log/node1.log:3,20,30,49,59,80 and log/node2.log
                       sequence IDs), rebuilt with Go-JSON rules, plus
                       Go-JSON escaping cases for the four message structs.
* ecdsa.json        -- RFC 6979 §A.2.5 published P-256/SHA-256 signatures,
                       seeded valid signatures, high-S, the eight corruption
                       classes of SURVEY.md §8(c), e >= n, R.x >= n, u1 = 0,
                       the u1*G == u2*Q doubling case, the cancellation case,
                       and invalid keys.
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import gojson, openssl_xcheck, p256  # noqa: E402

SEED = 0x50424654  # "PBFT", SURVEY.md §8(d)


def hx(b: bytes) -> str:
    return b.hex()


def i2h(v: int) -> str:
    return v.to_bytes(32, "big").hex()


# ----------------------------------------------------------------------------- sha256
def make_sha256():
    vecs = []
    fips = [b"abc", b"", b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
            b"abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu"]
    for m in fips:
        vecs.append({"msg": hx(m), "digest": hashlib.sha256(m).hexdigest(), "src": "FIPS 180-4 example"})
    rng = random.Random(SEED)
    for n in [1, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 255, 256, 1000, 4095, 4096]:
        m = bytes(rng.getrandbits(8) for _ in range(n))
        vecs.append({"msg": hx(m), "digest": hashlib.sha256(m).hexdigest(), "src": f"padding boundary len={n}"})
    m = b"a" * 1000000
    vecs.append({"msg_repeat": {"byte": "61", "count": 1000000},
                 "digest": hashlib.sha256(m).hexdigest(), "src": "FIPS 180-4 one million 'a'"})
    assert vecs[0]["digest"].startswith("ba7816bf") and vecs[0]["digest"].endswith("15ad")
    return vecs


# ----------------------------------------------------------------------------- digests
def make_digest_kats():
    # (timestamp, clientID, operation, sequenceID): log/node1.log:3,20 / 30,49 / 59,80
    logged = [(1668519246, "client1", "printf", 1668519247222762700),
              (1668519366, "client2", "printf", 1668519366935576000),
              (1668519455, "client3", "printf", 1668519456530528400)]
    out = {"requests": [], "votes": [], "preprepares": [], "replies": [], "escapes": []}
    for ts, cid, op, seq in logged:
        pre = gojson.request(ts, cid.encode(), op.encode(), seq)
        out["requests"].append({"timestamp": ts, "clientID": hx(cid.encode()), "operation": hx(op.encode()),
                                "sequenceID": seq, "preimage": hx(pre), "digest": hashlib.sha256(pre).hexdigest(),
                                "src": "log/node1.log request tuple"})
    expect = {"client1": "a63fc9e814525ac811f0ee3adcbe17bc46a58b828b8e1e07aa214f839f7365a9",
              "client2": "e5485d99d877dc5b37daf4a69c51f3b8c6501b5ffcce86ca77d5a80f365c13e4",
              "client3": "982077e48ed4e9a84ee74d5d35f4666e7fb5196169c8f75df1ca031d0563179a"}
    for r in out["requests"]:
        assert r["digest"] == expect[bytes.fromhex(r["clientID"]).decode()], "SURVEY §8(c) KAT mismatch"
    d1 = out["requests"][0]["digest"]
    view = 10000000000  # node.go:55
    for nid, mt in [("ReplicaNode1", 0), ("ReplicaNode3", 0), ("ReplicaNode3", 1), ("MainNode", 1)]:
        pre = gojson.vote(view, 1668519247222762700, d1.encode(), nid.encode(), mt)
        out["votes"].append({"viewID": view, "sequenceID": 1668519247222762700, "digest": hx(d1.encode()),
                             "nodeID": hx(nid.encode()), "msgType": mt, "preimage": hx(pre),
                             "digest_of_preimage": hashlib.sha256(pre).hexdigest()})
    ts, cid, op, seq = logged[0]
    for has in (True, False):
        pre = gojson.preprepare(view, seq, d1.encode(), (ts, cid.encode(), op.encode(), seq) if has else None)
        out["preprepares"].append({"viewID": view, "sequenceID": seq, "digest": hx(d1.encode()),
                                   "request": [ts, hx(cid.encode()), hx(op.encode()), seq] if has else None,
                                   "preimage": hx(pre), "digest_of_preimage": hashlib.sha256(pre).hexdigest()})
    for nid in ("MainNode", "ReplicaNode2"):
        pre = gojson.reply(view, ts, cid.encode(), nid.encode(), b"Executed")
        out["replies"].append({"viewID": view, "timestamp": ts, "clientID": hx(cid.encode()), "nodeID": hx(nid.encode()),
                               "result": hx(b"Executed"), "preimage": hx(pre),
                               "digest_of_preimage": hashlib.sha256(pre).hexdigest()})
    # Go-JSON string escaping cases (encoding/json encodeState.string, go1.19)
    cases = [b'quote"back\\slash', b"<script>&amp;</script>", b"tab\tnl\nret\r", b"\x00\x01\x1f\x7f",
             b"\x08\x0c form/backspace (go1.19: \\u0008 \\u000c)", "héllo wörld ✓ 𝄞".encode(),
             "line para ".encode(), b"bad \xff utf8 \xc0\xaf overlong", b"\xed\xa0\x80 surrogate",
             b"trunc \xe2\x82", b"\xf4\x90\x80\x80 >U+10FFFF", "U+FFFD itself: �".encode(), b"",
             b"-neg and big ints"]
    for i, s in enumerate(cases):
        ts_i = -1 if i % 3 == 0 else (2 ** 63 - 1 if i % 3 == 1 else -(2 ** 63))
        pre = gojson.request(ts_i, s, s[::-1], -i)
        out["escapes"].append({"timestamp": ts_i, "clientID": hx(s), "operation": hx(s[::-1]), "sequenceID": -i,
                               "preimage": hx(pre), "digest": hashlib.sha256(pre).hexdigest()})
    return out


# ----------------------------------------------------------------------------- ecdsa
def make_ecdsa():
    rng = random.Random(SEED)
    keys = []
    privs = []
    # key 0: RFC 6979 A.2.5 key
    d0 = 0xC9AFA9D845BA75166B5C215767B1D6934E50C3DB36E89B127B8A622B120F6721
    for i in range(8):
        d = d0 if i == 0 else rng.randrange(1, p256.N)
        privs.append(d)
        keys.append(p256.pubkey(d))
    # key 8: Q = G (d = 1), used for the doubling / cancellation cases
    privs.append(1)
    keys.append(p256.G)
    # key 9: crafted point with x in [n, p) (for R.x >= n), private key unknown
    t = 1
    while True:
        x = p256.N + t
        rhs = (x * x * x + p256.A * x + p256.B) % p256.P
        y = pow(rhs, (p256.P + 1) // 4, p256.P)
        if y * y % p256.P == rhs:
            break
        t += 1
    privs.append(None)
    keys.append((x, y))
    assert p256.on_curve(keys[-1]) and x >= p256.N
    n_valid_keys = len(keys)
    # invalid keys (must never verify): off-curve, x >= p, infinity encoding (0,0)
    gx, gy = p256.G
    keys.append((gx, (gy + 1) % p256.P))
    # non-canonical encoding: (t, y) is on the curve for a small t, (t + p, y) is not canonical
    t = 1
    while True:
        rhs = (t * t * t + p256.A * t + p256.B) % p256.P
        y = pow(rhs, (p256.P + 1) // 4, p256.P)
        if y * y % p256.P == rhs:
            break
        t += 1
    keys.append((t + p256.P, y))
    keys.append((0, 0))
    inval = list(range(n_valid_keys, len(keys)))

    vecs = []

    def add(h, r, s, k, kind):
        vecs.append({"hash": hx(h), "r": r, "s": s, "key": k, "kind": kind})

    # RFC 6979 A.2.5, SHA-256
    add(p256.sha256(b"sample"), 0xEFD48B2AACB6A8FD1140DD9CD45E81D69D2C877B56AAF991C34D0EA84EAF3716,
        0xF7CB1C942D657C41D436C7A1B6E29F65F3E900DBB9AFF4064DC4AB2F843ACDA8, 0, "rfc6979 sample")
    add(p256.sha256(b"test"), 0xF1ABB023518351CD71D881567B1EA663ED3EFCF6C5132B354F28D3B0B7D38367,
        0x019F4113742A2B14BD25926B49C649155F267E60D3814B4C0CC84250E46F0083, 0, "rfc6979 test")
    valid = []
    for i in range(96):
        k = i % 8
        h = p256.sha256(b"pbft vote %d" % i)
        r, s = p256.sign(h, privs[k], rng.randrange(1, p256.N))
        add(h, r, s, k, "valid")
        valid.append((h, r, s, k))
    for (h, r, s, k) in valid[:8]:
        add(h, r, p256.N - s, k, "high-S valid")
    # corruption classes, 4 each
    for j, (h, r, s, k) in enumerate(valid[8:40]):
        c = j % 8
        if c == 0:
            add(h, r ^ (1 << rng.randrange(256)), s, k, "flip r")
        elif c == 1:
            add(h, r, s ^ (1 << rng.randrange(256)), k, "flip s")
        elif c == 2:
            hb = bytearray(h); hb[rng.randrange(32)] ^= 1 << rng.randrange(8)
            add(bytes(hb), r, s, k, "flip hash")
        elif c == 3:
            add(h, r, s, (k + 1) % 8, "wrong key")
        elif c == 4:
            add(h, 0, s, k, "r=0")
        elif c == 5:
            add(h, r, 0, k, "s=0")
        elif c == 6:
            add(h, p256.N, s, k, "r=n")
        else:
            add(h, r, p256.N + rng.randrange(0, 2 ** 128) if j % 2 else 2 ** 256 - 1, k, "s>=n")
    # range edges
    add(valid[0][0], p256.N - 1, valid[0][2], valid[0][3], "r=n-1 (in range, wrong)")
    add(valid[0][0], valid[0][1], 1, valid[0][3], "s=1 (in range, wrong)")
    add(valid[0][0], 2 ** 256 - 1, valid[0][2], valid[0][3], "r=2^256-1")
    # e >= n: hashes whose integer value exceeds n, with real signatures
    for j in range(6):
        e = p256.N + rng.randrange(0, 2 ** 256 - p256.N)
        h = e.to_bytes(32, "big")
        k = j % 8
        r, s = p256.sign(h, privs[k], rng.randrange(1, p256.N))
        add(h, r, s, k, "e>=n valid")
    add(b"\xff" * 32, *p256.sign(b"\xff" * 32, privs[1], 12345), 1, "e=2^256-1 valid")
    add(p256.N.to_bytes(32, "big"), *p256.sign(p256.N.to_bytes(32, "big"), privs[2], 777), 2, "e=n (u1=0) valid")
    add(b"\x00" * 32, *p256.sign(b"\x00" * 32, privs[3], 999), 3, "e=0 (u1=0) valid")
    # R.x >= n: key 9 = R with x in [n,p); hash=0 -> u1=0; r = x-n, s = r -> u2 = 1 -> R = Q
    rx = keys[9][0] - p256.N
    add(b"\x00" * 32, rx, rx, 9, "R.x>=n valid (u1=0,u2=1)")
    add(b"\x00" * 32, rx + 1, rx + 1, 9, "R.x>=n wrong r")
    add(b"\x00" * 32, keys[9][0], keys[9][0], 9, "R.x>=n unreduced r=x")
    # doubling: Q = G, e == r -> u1 == u2 -> u1*G + u2*Q = 2u*G
    for j in range(3):
        kk = rng.randrange(1, p256.N)
        R = p256.scalar_mult(kk, p256.G)
        r = R[0] % p256.N
        s = 2 * r * pow(kk, -1, p256.N) % p256.N
        add(r.to_bytes(32, "big"), r, s, 8, "u1G==u2Q doubling valid")
    # cancellation: Q = G, e == -r mod n -> u1 = -u2 -> infinity -> reject
    for j in range(3):
        r = rng.randrange(1, p256.N)
        e = (-r) % p256.N
        add(e.to_bytes(32, "big"), r, rng.randrange(1, p256.N), 8, "u1G==-u2Q infinity")
    # invalid keys with otherwise well-formed signatures
    for kidx in inval:
        h, r, s, k = valid[0]
        add(h, r, s, kidx, "invalid key")
    # key index beyond the table
    add(valid[1][0], valid[1][1], valid[1][2], len(keys) + 5, "key index out of range")

    # cross-check: python restatement vs OpenSSL
    for v in vecs:
        h = bytes.fromhex(v["hash"])
        k = v["key"]
        if k < len(keys):
            qx, qy = keys[k]
            mine = p256.verify(h, v["r"], v["s"], qx, qy)
            ossl = openssl_xcheck.ecdsa_verify(h, v["r"], v["s"], qx, qy) if (v["r"] < 2 ** 256 and v["s"] < 2 ** 256) else False
        else:
            mine = ossl = False
        if mine != ossl:
            raise SystemExit(f"oracle/OpenSSL disagree on {v['kind']}: mine={mine} openssl={ossl}")
        v["expect"] = bool(mine)
        v["r"] = i2h(v["r"]) if v["r"] < 2 ** 256 else None
        v["s"] = i2h(v["s"]) if v["s"] < 2 ** 256 else None
    vecs = [v for v in vecs if v["r"] is not None and v["s"] is not None]
    kinds_expected = {"valid": True, "high-S valid": True, "rfc6979 sample": True, "rfc6979 test": True,
                      "e>=n valid": True, "e=2^256-1 valid": True, "e=n (u1=0) valid": True,
                      "e=0 (u1=0) valid": True, "R.x>=n valid (u1=0,u2=1)": True, "u1G==u2Q doubling valid": True}
    for v in vecs:
        want = kinds_expected.get(v["kind"], False)
        if v["expect"] != want:
            raise SystemExit(f"unexpected outcome for {v['kind']}: {v['expect']}")
    key_list = [{"x": i2h(x), "y": i2h(y), "valid": p256.key_valid(x, y)} for (x, y) in keys]
    return {"seed": SEED, "keys": key_list, "vectors": vecs,
            "note": "expect = go1.19 crypto/ecdsa.Verify outcome (restated), cross-checked with OpenSSL 3.0 ECDSA_do_verify"}


def main():
    if not openssl_xcheck.available():
        raise SystemExit("libcrypto not found: fixtures must be cross-checked with OpenSSL")
    with open(os.path.join(HERE, "sha256.json"), "w") as f:
        json.dump(make_sha256(), f, indent=0)
    with open(os.path.join(HERE, "digest_kats.json"), "w") as f:
        json.dump(make_digest_kats(), f, indent=0)
    with open(os.path.join(HERE, "ecdsa.json"), "w") as f:
        json.dump(make_ecdsa(), f, indent=0)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
