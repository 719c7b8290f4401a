"""Go 1.19 encoding/json restatement -- TEST INFRASTRUCTURE ONLY.

Builds the digest preimages of the reference's messages exactly as
``json.Marshal`` does (pbft/consensus/pbft_impl.go:235-243 over the structs of
pbft/consensus/pbft_msg_types.go:3-38).  Rules are listed in
oracle/gojson_ref.c (the C twin this module is checked against).  Strings
are bytes (Go strings are byte strings and may hold invalid UTF-8).
"""
from __future__ import annotations

_HEX = b"0123456789abcdef"


def _utf8_len(s: bytes, i: int):
    """(size, rune) of a valid UTF-8 sequence at s[i:] per Go's utf8 tables, or (0, None)."""
    c = s[i]
    rem = len(s) - i
    if 0xC2 <= c <= 0xDF:
        if rem < 2 or (s[i + 1] & 0xC0) != 0x80:
            return 0, None
        return 2, ((c & 0x1F) << 6) | (s[i + 1] & 0x3F)
    if 0xE0 <= c <= 0xEF:
        lo, hi = (0xA0 if c == 0xE0 else 0x80), (0x9F if c == 0xED else 0xBF)
        if rem < 2 or not (lo <= s[i + 1] <= hi):
            return 0, None
        if rem < 3 or (s[i + 2] & 0xC0) != 0x80:
            return 0, None
        return 3, ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F)
    if 0xF0 <= c <= 0xF4:
        lo, hi = (0x90 if c == 0xF0 else 0x80), (0x8F if c == 0xF4 else 0xBF)
        if rem < 2 or not (lo <= s[i + 1] <= hi):
            return 0, None
        if rem < 3 or (s[i + 2] & 0xC0) != 0x80:
            return 0, None
        if rem < 4 or (s[i + 3] & 0xC0) != 0x80:
            return 0, None
        return 4, ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F)
    return 0, None


def string(s: bytes) -> bytes:
    """go1.19 encodeState.string(s, escapeHTML=true)."""
    out = bytearray(b'"')
    i = 0
    while i < len(s):
        c = s[i]
        if c < 0x80:
            if c >= 0x20 and c not in b'"\\<>&':
                out.append(c)
            elif c in b'\\"':
                out += b"\\" + bytes([c])
            elif c == 0x0A:
                out += b"\\n"
            elif c == 0x0D:
                out += b"\\r"
            elif c == 0x09:
                out += b"\\t"
            else:
                out += b"\\u00" + bytes([_HEX[c >> 4], _HEX[c & 15]])
            i += 1
            continue
        size, rune = _utf8_len(s, i)
        if size == 0:
            out += b"\\ufffd"
            i += 1
            continue
        if rune in (0x2028, 0x2029):
            out += b"\\u202" + bytes([_HEX[rune & 15]])
        else:
            out += s[i:i + size]
        i += size
    out += b'"'
    return bytes(out)


def _int(v: int) -> bytes:
    return str(int(v)).encode()


def request(timestamp: int, client_id: bytes, operation: bytes, sequence_id: int) -> bytes:
    """RequestMsg, pbft_msg_types.go:3-8."""
    return (b'{"timestamp":' + _int(timestamp) + b',"clientID":' + string(client_id) + b',"operation":' +
            string(operation) + b',"sequenceID":' + _int(sequence_id) + b"}")


def vote(view_id: int, sequence_id: int, digest: bytes, node_id: bytes, msg_type: int) -> bytes:
    """VoteMsg, pbft_msg_types.go:25-31 (embedded MsgType tagged "msgType")."""
    return (b'{"viewID":' + _int(view_id) + b',"sequenceID":' + _int(sequence_id) + b',"digest":' + string(digest) +
            b',"nodeID":' + string(node_id) + b',"msgType":' + _int(msg_type) + b"}")


def _bytes_field(b: bytes | None) -> bytes:
    """encodeByteSlice (go1.19): base64.StdEncoding in quotes; a nil slice is null."""
    import base64
    return b"null" if b is None else b'"' + base64.b64encode(b) + b'"'


def _with_signature(body: bytes, signature: bytes | None) -> bytes:
    """A struct's encoding with the build-added last field Signature []byte `json:"signature"`."""
    return body[:-1] + b',"signature":' + _bytes_field(signature) + b"}"


def vote_signed(view_id: int, sequence_id: int, digest: bytes, node_id: bytes, msg_type: int,
                signature: bytes | None) -> bytes:
    """Signed VoteMsg wire JSON (build-added field after the embedded MsgType):
    Go encodes a []byte as a base64.StdEncoding string and a nil slice as null."""
    return _with_signature(vote(view_id, sequence_id, digest, node_id, msg_type), signature)


def request_signed(timestamp: int, client_id: bytes, operation: bytes, sequence_id: int,
                   signature: bytes | None) -> bytes:
    """Signed RequestMsg wire JSON."""
    return _with_signature(request(timestamp, client_id, operation, sequence_id), signature)


def reply_signed(view_id: int, timestamp: int, client_id: bytes, node_id: bytes, result: bytes,
                 signature: bytes | None) -> bytes:
    """Signed ReplyMsg wire JSON."""
    return _with_signature(reply(view_id, timestamp, client_id, node_id, result), signature)


def preprepare_signed(view_id: int, sequence_id: int, digest: bytes, req, req_signature: bytes | None,
                      signature: bytes | None) -> bytes:
    """Signed PrePrepareMsg wire JSON: the embedded request is the client's
    signed RequestMsg (null if nil); the primary's signature is over preprepare() (unsigned)."""
    body = request_signed(*req, req_signature) if req is not None else b"null"
    return _with_signature(b'{"viewID":' + _int(view_id) + b',"sequenceID":' + _int(sequence_id) + b',"digest":' +
                           string(digest) + b',"requestMsg":' + body + b"}", signature)


def request_or_null(req) -> bytes:
    """digest(*RequestMsg) preimage: json.Marshal of a nil pointer is null (pbft_impl.go:190)."""
    return request(*req) if req is not None else b"null"


def reply(view_id: int, timestamp: int, client_id: bytes, node_id: bytes, result: bytes) -> bytes:
    """ReplyMsg, pbft_msg_types.go:10-16."""
    return (b'{"viewID":' + _int(view_id) + b',"timestamp":' + _int(timestamp) + b',"clientID":' + string(client_id) +
            b',"nodeID":' + string(node_id) + b',"result":' + string(result) + b"}")


def preprepare(view_id: int, sequence_id: int, digest: bytes, req) -> bytes:
    """PrePrepareMsg, pbft_msg_types.go:18-23; req = (ts, clientID, op, seq) or None (-> null)."""
    body = request(*req) if req is not None else b"null"
    return (b'{"viewID":' + _int(view_id) + b',"sequenceID":' + _int(sequence_id) + b',"digest":' + string(digest) +
            b',"requestMsg":' + body + b"}")
