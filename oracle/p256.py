"""ECDSA-P256 restatement -- TEST INFRASTRUCTURE ONLY (the checker, never the product).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  The product path (``simple_pbft_amd``) never does.

What it restates
----------------
The reference (1556174776/simple_pbft @ 2025-02-19) has no signature code: its
author lists "consensus messages between nodes need digital signatures and
verification" as future work (``需要改进的地方.md:17``).  The parity target fixed
by SURVEY.md §0.1 / §8(a10) is therefore the Go standard library
``crypto/ecdsa.Verify`` on ``elliptic.P256()`` at the Go version pinned by
``go.mod:3`` (go 1.19).  Go is absent from this image, so the published
algorithm is restated here (SEC 1 v2 §4.1.4 / FIPS 186-4 §6.4, as implemented
by go1.19 ``crypto/ecdsa/ecdsa.go: Verify / verifyGeneric``):

    accept  iff  1 <= r < n  and  1 <= s < n            (Verify's range checks)
            and  e = int(hash[:32])  (hashToInt, big-endian, no reduction)
            and  w = s^-1 mod n, u1 = e*w mod n, u2 = r*w mod n
            and  R = u1*G + u2*Q is not the point at infinity
            and  R.x mod n == r.
High-S signatures are accepted (Go does not enforce low-S).

Key validity: go1.19 panics in ``ScalarMult`` for a point that is not on the
curve ("crypto/elliptic: ScalarMult was called on an invalid point").  The
batch verifier validates keys at registration instead (SURVEY.md §7 "Hard
parts"); an invalid key never verifies.  ``key_valid`` restates that check.

Pinning: ``tests/test_oracle.py`` checks this module against the RFC 6979
§A.2.5 P-256/SHA-256 published vectors and against OpenSSL 3.0.2 libcrypto
(an independent implementation) on every committed fixture.
"""
from __future__ import annotations

import hashlib
import random

# Curve parameters, FIPS 186-4 D.1.2.3 (== go1.19 crypto/elliptic/params p256Params)
P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
A = P - 3
B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
GX = 0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296
GY = 0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5
G = (GX, GY)
INF = None


def on_curve(pt) -> bool:
    if pt is None:
        return False
    x, y = pt
    if not (0 <= x < P and 0 <= y < P):
        return False
    return (y * y - (x * x * x + A * x + B)) % P == 0


def key_valid(x: int, y: int) -> bool:
    """Registration-time key check (see module docstring)."""
    return on_curve((x, y))


def point_add(p1, p2):
    """Affine group law with the point at infinity as ``None`` (complete)."""
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1 + A) * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    y3 = (lam * (x1 - x3) - y1) % P
    return (x3, y3)


def scalar_mult(k: int, pt):
    acc = None
    add = pt
    while k:
        if k & 1:
            acc = point_add(acc, add)
        add = point_add(add, add)
        k >>= 1
    return acc


def hash_to_int(h: bytes) -> int:
    """go1.19 crypto/ecdsa hashToInt for P-256: leftmost 256 bits, big-endian."""
    h = h[:32]
    e = int.from_bytes(h, "big")
    excess = len(h) * 8 - 256
    if excess > 0:
        e >>= excess
    return e


def verify(h: bytes, r: int, s: int, qx: int, qy: int) -> bool:
    """Restates go1.19 crypto/ecdsa.Verify (+ registration-time key check)."""
    if not key_valid(qx, qy):
        return False
    if r <= 0 or s <= 0 or r >= N or s >= N:
        return False
    e = hash_to_int(h)
    w = pow(s, -1, N)
    u1 = e * w % N
    u2 = r * w % N
    R = point_add(scalar_mult(u1, G), scalar_mult(u2, (qx, qy)))
    if R is None:
        return False
    return R[0] % N == r


def pubkey(d: int):
    return scalar_mult(d, G)


def sign(h: bytes, d: int, k: int):
    """Textbook ECDSA signing with an explicit nonce (fixture generation only)."""
    e = hash_to_int(h)
    R = scalar_mult(k, G)
    r = R[0] % N
    s = pow(k, -1, N) * (e + r * d) % N
    if r == 0 or s == 0:
        raise ValueError("degenerate nonce")
    return r, s


def keygen(rng: random.Random):
    d = rng.randrange(1, N)
    q = pubkey(d)
    return d, q


def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()
