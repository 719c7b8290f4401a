"""go1.19 ``crypto/ecdsa.VerifyASN1`` DER parse -- TEST INFRASTRUCTURE ONLY.

Restates the parse step of VerifyASN1 (Go stdlib, not under /root/reference;
SURVEY.md §8 a10 puts DER parsing on the host with Go's strictness) over
golang.org/x/crypto/cryptobyte as vendored in go1.19:

    input.ReadASN1(&inner, SEQUENCE) && input.Empty() &&
    inner.ReadASN1Integer(r) && inner.ReadASN1Integer(s) && inner.Empty()

Returns (r, s) as Python ints (possibly negative), or None where the parse
fails.  The checker for simple_pbft_amd/csrc/der.cpp; never the product.
"""
from __future__ import annotations


def _read_asn1(buf: bytes, tag: int):
    """cryptobyte.String.ReadASN1: (contents, rest) or None."""
    if len(buf) < 2:
        return None
    t, lb = buf[0], buf[1]
    if t & 0x1F == 0x1F:  # high-tag-number form unsupported
        return None
    if lb & 0x80 == 0:
        hdr, ln = 2, lb
    else:
        ll = lb & 0x7F
        if ll == 0 or ll > 4 or len(buf) < 2 + ll:
            return None
        ln = int.from_bytes(buf[2:2 + ll], "big")
        if ln < 128:  # should have used the short form
            return None
        if ln >> ((ll - 1) * 8) == 0:  # leading zero length byte
            return None
        hdr = 2 + ll
    if len(buf) < hdr + ln or t != tag:
        return None
    return buf[hdr:hdr + ln], buf[hdr + ln:]


def _read_int(buf: bytes):
    """ReadASN1Integer into a big.Int (checkASN1Integer minimality)."""
    got = _read_asn1(buf, 0x02)
    if got is None:
        return None
    v, rest = got
    if len(v) == 0:
        return None
    if len(v) > 1 and ((v[0] == 0 and v[1] & 0x80 == 0) or (v[0] == 0xFF and v[1] & 0x80 == 0x80)):
        return None
    return int.from_bytes(v, "big", signed=True), rest


def parse(der: bytes):
    got = _read_asn1(der, 0x30)
    if got is None or got[1]:
        return None
    inner = got[0]
    a = _read_int(inner)
    if a is None:
        return None
    b = _read_int(a[1])
    if b is None or b[1]:
        return None
    return a[0], b[0]


def to_rs(der: bytes):
    """The product's contract: 64-B r||s when parsed with 0 <= r, s < 2^256, else None."""
    p = parse(der)
    if p is None or not all(0 <= v < 1 << 256 for v in p):
        return None
    return p[0].to_bytes(32, "big") + p[1].to_bytes(32, "big")


def encode(r: int, s: int) -> bytes:
    """Minimal DER of a signature (what crypto/ecdsa.SignASN1 emits for r, s > 0)."""
    def integer(v: int) -> bytes:
        b = v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big", signed=True)
        return b"\x02" + _len(len(b)) + b
    body = integer(r) + integer(s)
    return b"\x30" + _len(len(body)) + body


def _len(n: int) -> bytes:
    if n < 128:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b
