"""ctypes binding of the C ABI in include/pbftv.h (libpbftv.so, built in-tree).

This is plumbing for tests and bench.py: the product is the shared library.
Loading fails loudly if libpbftv.so is missing, and ``Verifier()`` fails with
``PbftvError(PBFTV_ENODEV)`` when no gfx950 GPU is visible -- there is no
CPU fallback anywhere in this package.
"""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PBFTV_LIB") or os.path.join(HERE, "libpbftv.so")  # PBFTV_LIB: experiment builds only
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "pbftv.h")

PBFTV_OK = 0
PBFTV_EINVAL = -1
PBFTV_ENODEV = -2
PBFTV_EDEVICE = -3
PBFTV_ENOMEM = -4
PBFTV_ENOKEYS = -5

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i64p = ctypes.POINTER(ctypes.c_int64)
_vp = ctypes.c_void_p

_lib = None


class PbftvError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"pbftv error {code}: {msg}")
        self.code = code


def lib() -> ctypes.CDLL:
    """Load libpbftv.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                      "or `make -C simple_pbft_amd`")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "pbftv_open": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_uint32]),
        "pbftv_close": (None, [_vp]),
        "pbftv_device_count": (ctypes.c_int, [_vp]),
        "pbftv_device_id": (ctypes.c_int, [_vp, ctypes.c_int]),
        "pbftv_strerror": (ctypes.c_char_p, [ctypes.c_int]),
        "pbftv_last_error": (ctypes.c_char_p, []),
        "pbftv_reserve": (ctypes.c_int, [_vp, ctypes.c_uint64]),
        "pbftv_dev_alloc": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(_vp)]),
        "pbftv_dev_free": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
        "pbftv_host_alloc": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.POINTER(_vp)]),
        "pbftv_host_free": (ctypes.c_int, [_vp, _vp]),
        "pbftv_memcpy_h2d": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, ctypes.c_uint64]),
        "pbftv_memcpy_d2h": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, ctypes.c_uint64]),
        "pbftv_memset_dev": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_uint64]),
        "pbftv_stream": (_vp, [_vp, ctypes.c_int]),
        "pbftv_stream_sync": (ctypes.c_int, [_vp, ctypes.c_int]),
        "pbftv_stream_create": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(_vp)]),
        "pbftv_stream_destroy": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
        "pbftv_stream_wait": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
        "pbftv_set_kernel_timing": (ctypes.c_int, [_vp, ctypes.c_int]),
        "pbftv_kernel_time_ms": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                ctypes.POINTER(ctypes.c_uint64)]),
        "pbftv_reset_kernel_times": (ctypes.c_int, [_vp]),
        "pbftv_qc_stamps": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
        "pbftv_set_latency_path_max": (ctypes.c_int, [_vp, ctypes.c_uint64]),
        "pbftv_qc_stamps_all": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_uint32]),
        "pbftv_qc_counters": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
        "pbftv_hash_hex": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_char_p]),
        "pbftv_sha256_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint64, _vp]),
        "pbftv_digest_check_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp]),
        "pbftv_sha256_batch_dev": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp,
                                                  _vp, _vp]),
        "pbftv_sha256_order_dev": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_uint64, _vp, _vp]),
        "pbftv_gojson_request": (ctypes.c_uint64, [ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                                   ctypes.c_uint64, ctypes.c_int64, _vp, ctypes.c_uint64]),
        "pbftv_gojson_vote": (ctypes.c_uint64, [ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint64,
                                                ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int64, _vp,
                                                ctypes.c_uint64]),
        "pbftv_gojson_vote_signed": (ctypes.c_uint64, [ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p,
                                                       ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64,
                                                       ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int,
                                                       _vp, ctypes.c_uint64]),
        "pbftv_gojson_request_signed": (ctypes.c_uint64, [ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint64,
                                                          ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int64,
                                                          ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, _vp,
                                                          ctypes.c_uint64]),
        "pbftv_gojson_reply_signed": (ctypes.c_uint64, [ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p,
                                                        ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64,
                                                        ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                                        ctypes.c_uint64, ctypes.c_int, _vp, ctypes.c_uint64]),
        "pbftv_gojson_preprepare_signed": (ctypes.c_uint64, [ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p,
                                                             ctypes.c_uint64, ctypes.c_int, ctypes.c_int64,
                                                             ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                                             ctypes.c_uint64, ctypes.c_int64, ctypes.c_char_p,
                                                             ctypes.c_uint64, ctypes.c_int, ctypes.c_char_p,
                                                             ctypes.c_uint64, ctypes.c_int, _vp, ctypes.c_uint64]),
        "pbftv_flush_requests": (ctypes.c_int, [_vp, ctypes.c_uint64] + [_vp] * 14),
        "pbftv_flush_replies": (ctypes.c_int, [_vp, ctypes.c_uint64] + [_vp] * 15),
        "pbftv_flush_preprepares": (ctypes.c_int, [_vp, ctypes.c_uint64] + [_vp] * 16 + [ctypes.c_uint32] +
                                    [_vp] * 7),
        "pbftv_ecdsa_der_to_rs": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint64, _vp]),
        "pbftv_ecdsa_der_to_rs_batch": (ctypes.c_int64, [_vp, _vp, _vp, ctypes.c_uint64, _vp]),
        "pbftv_gojson_reply": (ctypes.c_uint64, [ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint64,
                                                 ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64,
                                                 _vp, ctypes.c_uint64]),
        "pbftv_gojson_preprepare": (ctypes.c_uint64, [ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p,
                                                      ctypes.c_uint64, ctypes.c_int, ctypes.c_int64, ctypes.c_char_p,
                                                      ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64,
                                                      ctypes.c_int64, _vp, ctypes.c_uint64]),
        "pbftv_digest_request_batch": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                      _vp]),
        "pbftv_digest_vote_batch": (ctypes.c_int, [_vp, ctypes.c_uint64] + [_vp] * 10),
        "pbftv_digest_reply_batch": (ctypes.c_int, [_vp, ctypes.c_uint64] + [_vp] * 12),
        "pbftv_digest_preprepare_batch": (ctypes.c_int, [_vp, ctypes.c_uint64] + [_vp] * 15),
        "pbftv_flush_votes": (ctypes.c_int, [_vp, ctypes.c_uint64] + [_vp] * 11 + [ctypes.c_uint32] + [_vp] * 7),
        "pbftv_verify_msg_batch": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64, _vp, ctypes.c_uint64, _vp, _vp,
                                                  _vp, _vp, _vp, _vp]),
        "pbftv_register_keys": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp]),
        "pbftv_add_keys": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp]),
        "pbftv_set_key": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _vp]),
        "pbftv_table_config": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                              ctypes.POINTER(ctypes.c_uint64)]),
        "pbftv_ecdsa_p256_verify_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint64, _vp]),
        "pbftv_ecdsa_p256_verify_batch_dev": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, ctypes.c_uint64, _vp,
                                                             _vp]),
        "pbftv_qc_verify": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, _vp,
                                           ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def header_symbols() -> list[str]:
    """Every function declared in include/pbftv.h."""
    with open(HEADER_PATH) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pbftv_[a-z0-9_]+)\s*\(", text)))


def _ptr(a) -> int | None:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"]
        return a.ctypes.data
    if isinstance(a, (bytes, bytearray)):
        return ctypes.cast(ctypes.c_char_p(bytes(a)), ctypes.c_void_p).value
    return int(a)


def _check(rc: int):
    if rc != PBFTV_OK:
        L = lib()
        raise PbftvError(rc, (L.pbftv_last_error() or b"").decode() or L.pbftv_strerror(rc).decode())


def bitmap_to_bool(bm: np.ndarray, n: int) -> np.ndarray:
    return np.unpackbits(np.asarray(bm, dtype=np.uint8), bitorder="little")[:n].astype(bool)


# ---------------------------------------------------------------- host-only helpers (no GPU)
def gojson_request(ts: int, client_id: bytes, operation: bytes, seq: int) -> bytes:
    L = lib()
    n = L.pbftv_gojson_request(ts, client_id, len(client_id), operation, len(operation), seq, None, 0)
    buf = np.zeros(max(n, 1), np.uint8)
    L.pbftv_gojson_request(ts, client_id, len(client_id), operation, len(operation), seq, buf.ctypes.data, n)
    return buf[:n].tobytes()


def gojson_vote(view: int, seq: int, digest: bytes, node_id: bytes, msg_type: int) -> bytes:
    L = lib()
    n = L.pbftv_gojson_vote(view, seq, digest, len(digest), node_id, len(node_id), msg_type, None, 0)
    buf = np.zeros(max(n, 1), np.uint8)
    L.pbftv_gojson_vote(view, seq, digest, len(digest), node_id, len(node_id), msg_type, buf.ctypes.data, n)
    return buf[:n].tobytes()


def gojson_vote_signed(view: int, seq: int, digest: bytes, node_id: bytes, msg_type: int,
                       signature: bytes | None) -> bytes:
    """Signed VoteMsg wire JSON: VoteMsg + "signature" as base64, None -> null."""
    L = lib()
    sig = signature if signature is not None else b""
    args = (view, seq, digest, len(digest), node_id, len(node_id), msg_type, sig, len(sig),
            1 if signature is None else 0)
    n = L.pbftv_gojson_vote_signed(*args, None, 0)
    buf = np.zeros(max(n, 1), np.uint8)
    L.pbftv_gojson_vote_signed(*args, buf.ctypes.data, n)
    return buf[:n].tobytes()


def _sig_args(signature: bytes | None):
    sig = signature if signature is not None else b""
    return sig, len(sig), 1 if signature is None else 0


def _encode(fn, *args) -> bytes:
    n = fn(*args, None, 0)
    buf = np.zeros(max(n, 1), np.uint8)
    fn(*args, buf.ctypes.data, n)
    return buf[:n].tobytes()


def gojson_request_signed(ts: int, client_id: bytes, operation: bytes, seq: int, signature: bytes | None) -> bytes:
    """Signed RequestMsg wire JSON: RequestMsg + "signature" (base64, None -> null)."""
    return _encode(lib().pbftv_gojson_request_signed, ts, client_id, len(client_id), operation, len(operation), seq,
                   *_sig_args(signature))


def gojson_reply_signed(view: int, ts: int, client_id: bytes, node_id: bytes, result: bytes,
                        signature: bytes | None) -> bytes:
    """Signed ReplyMsg wire JSON."""
    return _encode(lib().pbftv_gojson_reply_signed, view, ts, client_id, len(client_id), node_id, len(node_id),
                   result, len(result), *_sig_args(signature))


def gojson_preprepare_signed(view: int, seq: int, digest: bytes, req, req_signature: bytes | None,
                             signature: bytes | None) -> bytes:
    """Signed PrePrepareMsg wire JSON; req = (ts, clientID, op, seq) or None, the
    embedded request carrying the client's signature req_signature."""
    if req is None:
        r = (0, 0, b"", 0, b"", 0, 0)
    else:
        ts, cid, op, rseq = req
        r = (1, ts, cid, len(cid), op, len(op), rseq)
    return _encode(lib().pbftv_gojson_preprepare_signed, view, seq, digest, len(digest), *r,
                   *_sig_args(req_signature), *_sig_args(signature))


def der_to_rs(der: bytes) -> bytes | None:
    """go1.19 ecdsa.VerifyASN1's DER parse: r||s (64 B BE), or None where Go rejects."""
    out = np.zeros(64, np.uint8)
    r = lib().pbftv_ecdsa_der_to_rs(der, len(der), out.ctypes.data)
    if r < 0:
        raise ValueError(f"pbftv_ecdsa_der_to_rs: {r}")
    return out.tobytes() if r == 1 else None


def der_to_rs_batch(ders: list[bytes]) -> tuple[np.ndarray, int]:
    """Batch form: (n x 64 uint8 r||s, rejected rows zeroed; number parsed)."""
    n = len(ders)
    lens = np.array([len(d) for d in ders], np.uint32)
    offs = np.zeros(n, np.uint64)
    if n > 1:
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    data = np.frombuffer(b"".join(ders) + b"\0", np.uint8)
    out = np.zeros((max(n, 1), 64), np.uint8)
    got = lib().pbftv_ecdsa_der_to_rs_batch(data.ctypes.data, offs.ctypes.data, lens.ctypes.data, n,
                                            out.ctypes.data)
    if got < 0:
        raise ValueError(f"pbftv_ecdsa_der_to_rs_batch: {got}")
    return out[:n], int(got)


def gojson_reply(view: int, ts: int, client_id: bytes, node_id: bytes, result: bytes) -> bytes:
    L = lib()
    args = (view, ts, client_id, len(client_id), node_id, len(node_id), result, len(result))
    n = L.pbftv_gojson_reply(*args, None, 0)
    buf = np.zeros(max(n, 1), np.uint8)
    L.pbftv_gojson_reply(*args, buf.ctypes.data, n)
    return buf[:n].tobytes()


def gojson_preprepare(view: int, seq: int, digest: bytes, req) -> bytes:
    L = lib()
    if req is None:
        args = (view, seq, digest, len(digest), 0, 0, b"", 0, b"", 0, 0)
    else:
        ts, cid, op, rseq = req
        args = (view, seq, digest, len(digest), 1, ts, cid, len(cid), op, len(op), rseq)
    n = L.pbftv_gojson_preprepare(*args, None, 0)
    buf = np.zeros(max(n, 1), np.uint8)
    L.pbftv_gojson_preprepare(*args, buf.ctypes.data, n)
    return buf[:n].tobytes()


def verify_msg_batch(state_view: int, state_last_seq: int, req_digest: bytes, view_ids, seq_ids,
                     digests_got: list[bytes]) -> np.ndarray:
    n = len(digests_got)
    blob = b"".join(digests_got)
    off = np.zeros(n, np.uint64)
    ln = np.array([len(d) for d in digests_got], np.uint32)
    if n:
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    v = np.ascontiguousarray(view_ids, np.int64)
    s = np.ascontiguousarray(seq_ids, np.int64)
    bm = np.zeros((n + 7) // 8 + 1, np.uint8)
    blob_arr = np.frombuffer(blob, np.uint8) if blob else np.zeros(1, np.uint8)
    rd = np.frombuffer(req_digest, np.uint8).copy()
    _check(lib().pbftv_verify_msg_batch(state_view, state_last_seq, rd.ctypes.data, n, v.ctypes.data, s.ctypes.data,
                                        blob_arr.ctypes.data, off.ctypes.data, ln.ctypes.data, bm.ctypes.data))
    return bitmap_to_bool(bm, n)


# ---------------------------------------------------------------- GPU context
K_ECDSA_SCALARS = 0
K_ECDSA_COMB = 1
K_SHA256 = 2
K_ECDSA_WAVE = 3
K_GOJSON = 4


class RequestColumns:
    """RequestMsgs (pbft_msg_types.go:3-8) column-wise for pbftv_digest_request_batch."""

    def __init__(self, requests):
        """requests: list of (timestamp, clientID bytes, operation bytes, sequenceID)."""
        self.n = len(requests)
        self.ts = np.array([r[0] for r in requests], np.int64)
        self.seq = np.array([r[3] for r in requests], np.int64)
        self.cid = Verifier.pack([r[1] for r in requests])
        self.op = Verifier.pack([r[2] for r in requests])

    def args(self):
        (cb, co, cl), (ob, oo, ol) = self.cid, self.op
        return [self.ts.ctypes.data, cb.ctypes.data, co.ctypes.data, cl.ctypes.data, ob.ctypes.data, oo.ctypes.data,
                ol.ctypes.data, self.seq.ctypes.data]


class ReplyColumns:
    """ReplyMsgs (pbft_msg_types.go:10-16) column-wise for pbftv_digest_reply_batch."""

    def __init__(self, replies):
        """replies: list of (viewID, timestamp, clientID bytes, nodeID bytes, result bytes)."""
        self.n = len(replies)
        self.view = np.array([x[0] for x in replies], np.int64)
        self.ts = np.array([x[1] for x in replies], np.int64)
        self.cid = Verifier.pack([x[2] for x in replies])
        self.node = Verifier.pack([x[3] for x in replies])
        self.result = Verifier.pack([x[4] for x in replies])

    def args(self):
        out = [self.view.ctypes.data, self.ts.ctypes.data]
        for b, o, ln in (self.cid, self.node, self.result):
            out += [b.ctypes.data, o.ctypes.data, ln.ctypes.data]
        return out


class VoteColumns:
    """A snapshot of VoteMsgs (pbft_msg_types.go:25-31) laid out column-wise, as
    the cgo shim would hand a pool snapshot to pbftv_flush_votes: int64 columns
    plus byte-string blobs with per-vote offsets/lengths."""

    def __init__(self, votes):
        """votes: list of (viewID, sequenceID, digest bytes, nodeID bytes, msgType)."""
        self.n = len(votes)
        self.view = np.array([x[0] for x in votes], np.int64)
        self.seq = np.array([x[1] for x in votes], np.int64)
        self.type = np.array([x[4] for x in votes], np.int64)
        self.digest = Verifier.pack([x[2] for x in votes])
        self.node = Verifier.pack([x[3] for x in votes])

    def args(self):
        (db, do, dl), (nb, no, nl) = self.digest, self.node
        return [self.view.ctypes.data, self.seq.ctypes.data, db.ctypes.data, do.ctypes.data, dl.ctypes.data,
                nb.ctypes.data, no.ctypes.data, nl.ctypes.data, self.type.ctypes.data]


class PrePrepareColumns:
    """PrePrepareMsgs (pbft_msg_types.go:18-23) column-wise: request None -> requestMsg null
    (its request columns still hold a placeholder row)."""

    def __init__(self, pps):
        """pps: list of (viewID, sequenceID, digest bytes, request) with request None or
        (timestamp, clientID bytes, operation bytes, sequenceID)."""
        self.n = len(pps)
        self.view = np.array([x[0] for x in pps], np.int64)
        self.seq = np.array([x[1] for x in pps], np.int64)
        self.has = np.array([x[3] is not None for x in pps], np.uint8)
        reqs = [x[3] if x[3] is not None else (0, b"", b"", 0) for x in pps]
        self.rts = np.array([r[0] for r in reqs], np.int64)
        self.rseq = np.array([r[3] for r in reqs], np.int64)
        self.digest = Verifier.pack([x[2] for x in pps])
        self.cid = Verifier.pack([r[1] for r in reqs])
        self.op = Verifier.pack([r[2] for r in reqs])

    def args(self):
        (db, do, dl), (cb, co, cl), (ob, oo, ol) = self.digest, self.cid, self.op
        return [self.view.ctypes.data, self.seq.ctypes.data, db.ctypes.data, do.ctypes.data, dl.ctypes.data,
                self.has.ctypes.data, self.rts.ctypes.data, cb.ctypes.data, co.ctypes.data, cl.ctypes.data,
                ob.ctypes.data, oo.ctypes.data, ol.ctypes.data, self.rseq.ctypes.data]


def _sig_inputs(n: int, sigs, key_idx, what: str):
    if sigs is None:
        return None, None, None
    sigs = np.ascontiguousarray(sigs, np.uint8)
    key_idx = np.ascontiguousarray(key_idx, np.uint32)
    if sigs.shape != (n, 64) or key_idx.shape != (n,):
        raise ValueError(f"{what}: sigs must be (n, 64) uint8 and key_idx (n,)")
    return sigs, key_idx, np.zeros((n + 7) // 8 + 1, np.uint8)


def _states(n: int, states, state_idx, what: str, with_digests: bool):
    sv = np.ascontiguousarray(states[0], np.int64)
    sl = np.ascontiguousarray(states[1], np.int64)
    si = np.ascontiguousarray(state_idx, np.uint32)
    k = len(sv)
    sd = np.ascontiguousarray(states[2], np.uint8) if with_digests else None
    if sl.shape != (k,) or si.shape != (n,) or (with_digests and sd.shape != (k, 32)):
        raise ValueError(f"{what}: states must be (k,), (k,){', (k, 32)' if with_digests else ''} "
                         "and state_idx (n,)")
    return k, sv, sl, sd, si


class DeviceBuffer:
    """A pbftv_dev_alloc allocation on one of the context's devices."""

    def __init__(self, ver: "Verifier", dev: int, ptr: int, nbytes: int):
        self.ver, self.dev, self.ptr, self.nbytes = ver, dev, ptr, nbytes

    def to_host(self, nbytes: int | None = None, dtype=np.uint8) -> np.ndarray:
        nb = self.nbytes if nbytes is None else nbytes
        out = np.zeros(max(nb, 1), np.uint8)
        if nb:
            _check(self.ver._L.pbftv_memcpy_d2h(self.ver._h, self.dev, out.ctypes.data, self.ptr, nb))
        return out[:nb].view(dtype)

    def zero(self):
        _check(self.ver._L.pbftv_memset_dev(self.ver._h, self.dev, self.ptr, 0, self.nbytes))

    def free(self):
        if self.ptr and self.ver._h is not None:
            _check(self.ver._L.pbftv_dev_free(self.ver._h, self.dev, self.ptr))
        self.ptr = 0


class PinnedArray:
    """A numpy view of pbftv_host_alloc memory (pinned: host-buffer verifies
    from it skip the staging copy).  Free with .free() before the Verifier closes."""

    def __init__(self, ver: "Verifier", shape, dtype):
        self.ver = ver
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        p = ctypes.c_void_p()
        _check(ver._L.pbftv_host_alloc(ver._h, max(nbytes, 1), ctypes.byref(p)))
        self.ptr = p.value
        buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(self.ptr)
        self.a = np.frombuffer(buf, np.uint8)[:nbytes].view(dtype).reshape(shape)

    def free(self):
        if self.ptr and self.ver._h is not None:
            self.a = None
            _check(self.ver._L.pbftv_host_free(self.ver._h, self.ptr))
        self.ptr = 0


class Verifier:
    """A pbftv_ctx: the GPUs in device_mask (0 = all visible gfx950 devices)."""

    def __init__(self, device_mask: int = 0):
        self._L = lib()
        h = ctypes.c_void_p()
        _check(self._L.pbftv_open(ctypes.byref(h), device_mask))
        self._h = h
        self._wave_env = os.environ.get("PBFTV_WAVE_MAX")  # what pbftv_open read

    def set_latency_path_max(self, n: int):
        """pbftv_set_latency_path_max: batches up to n take the latency path."""
        _check(self._L.pbftv_set_latency_path_max(self._h, n))

    def _sync_env(self):
        # the library reads PBFTV_WAVE_MAX once, at pbftv_open (no getenv on its
        # call path); tests flip the variable under one context, so the binding
        # forwards a change before the calls that depend on it
        e = os.environ.get("PBFTV_WAVE_MAX")
        if e != self._wave_env:
            self._wave_env = e
            self.set_latency_path_max(int(e) if e is not None else 2048)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.pbftv_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    def device_count(self) -> int:
        return self._L.pbftv_device_count(self._h)

    def device_id(self, i: int) -> int:
        return self._L.pbftv_device_id(self._h, i)

    def reserve(self, n: int):
        _check(self._L.pbftv_reserve(self._h, n))

    # ---- device memory plumbing (no torch: torch bundles its own HIP runtime)
    def alloc(self, dev: int, nbytes: int) -> "DeviceBuffer":
        p = ctypes.c_void_p()
        _check(self._L.pbftv_dev_alloc(self._h, dev, nbytes, ctypes.byref(p)))
        return DeviceBuffer(self, dev, p.value, nbytes)

    def to_device(self, dev: int, arr: np.ndarray, pad: int = 0) -> "DeviceBuffer":
        arr = np.ascontiguousarray(arr)
        buf = self.alloc(dev, arr.nbytes + pad)
        if arr.nbytes:
            _check(self._L.pbftv_memcpy_h2d(self._h, dev, buf.ptr, arr.ctypes.data, arr.nbytes))
        if pad:
            _check(self._L.pbftv_memset_dev(self._h, dev, buf.ptr + arr.nbytes, 0, pad))
        return buf

    def pinned(self, arr: np.ndarray) -> PinnedArray:
        """A pinned copy of arr (pbftv_host_alloc)."""
        arr = np.ascontiguousarray(arr)
        p = PinnedArray(self, arr.shape, arr.dtype)
        p.a[...] = arr
        return p

    def stream(self, dev: int) -> int:
        return self._L.pbftv_stream(self._h, dev)

    def stream_create(self, dev: int) -> int:
        st = ctypes.c_void_p()
        _check(self._L.pbftv_stream_create(self._h, dev, ctypes.byref(st)))
        return st.value

    def stream_destroy(self, dev: int, stream: int):
        _check(self._L.pbftv_stream_destroy(self._h, dev, stream))

    def stream_wait(self, dev: int, stream: int):
        _check(self._L.pbftv_stream_wait(self._h, dev, stream))

    def sync(self, dev: int):
        _check(self._L.pbftv_stream_sync(self._h, dev))

    def set_kernel_timing(self, on: bool):
        _check(self._L.pbftv_set_kernel_timing(self._h, 1 if on else 0))

    def kernel_time_ms(self, dev: int, kernel: int):
        ms = ctypes.c_double()
        cnt = ctypes.c_uint64()
        _check(self._L.pbftv_kernel_time_ms(self._h, dev, kernel, ctypes.byref(ms), ctypes.byref(cnt)))
        return ms.value, cnt.value

    def reset_kernel_times(self):
        _check(self._L.pbftv_reset_kernel_times(self._h))

    def qc_stamps_all(self, n: int, dev: int = 0) -> np.ndarray:
        """pbftv_qc_stamps_all: (n, 4) uint64 {seen wall, seen clk, done wall, done clk}
        per armed wave of the last call (zeros after a launch)."""
        o = np.zeros((n, 4), np.uint64)
        self._L.pbftv_qc_stamps_all(self._h, dev, o.ctypes.data, n)
        return o

    def qc_counters(self, dev: int = 0) -> dict:
        """pbftv_qc_counters: the latency path's counters since the context
        opened -- calls, served armed, armed calls rerun by a launch (an
        exceptional signature), signatures through a launched kernel's exact
        path, launches, armings, keeper rotations -- and the armed kernel now
        (armed_waves 0: none; armed_wide)."""
        o = np.zeros(8, np.uint64)
        _check(self._L.pbftv_qc_counters(self._h, dev, o.ctypes.data))
        names = ("calls", "armed", "reruns", "exact_sigs", "launches", "armings", "rotations")
        r = {k: int(v) for k, v in zip(names, o[:7])}
        r["armed_waves"] = int(o[7]) & 0xFFFFFFFF
        r["armed_wide"] = bool(int(o[7]) >> 32)
        return r

    def qc_stamps(self, dev: int = 0) -> dict:
        """pbftv_qc_stamps: where the last latency-path call's time went (host
        hand-over / total in us; for an armed serve, the GPU's own serve time
        and the mean shader clock over it)."""
        o = np.zeros(8, np.uint64)
        _check(self._L.pbftv_qc_stamps(self._h, dev, o.ctypes.data))
        armed = bool(int(o[2]) & 1)
        r = {"handover_us": float(o[0]) * 1e-3, "total_us": float(o[1]) * 1e-3, "armed": armed,
             "entry_us": float(int(o[2]) >> 32) * 1e-3, "slots_in_us": float((int(o[2]) >> 1) & 0x7FFFFFFF) * 1e-3}
        w0, c0, w1, c1, khz = (int(x) for x in (o[3], o[4], o[5], o[6], o[7]))
        if armed and w1 > w0 and khz:  # (stamps are written only with PBFTV_QC_STAMPS=1)
            wall_s = (w1 - w0) / (khz * 1e3)
            r["gpu_serve_us"] = wall_s * 1e6
            if c1 > c0:
                r["sclk_mhz"] = (c1 - c0) / wall_s * 1e-6
        return r

    # ---- sha256 / digests
    def hash_hex(self, content: bytes) -> str:
        out = ctypes.create_string_buffer(65)
        arr = np.frombuffer(content, np.uint8) if content else np.zeros(1, np.uint8)
        _check(self._L.pbftv_hash_hex(self._h, arr.ctypes.data, len(content), out))
        return out.value.decode()

    @staticmethod
    def pack(messages: list[bytes]):
        lengths = np.array([len(m) for m in messages], np.uint32)
        offsets = np.zeros(len(messages), np.uint64)
        if len(messages):
            offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
        blob = np.frombuffer(b"".join(messages), np.uint8) if sum(map(len, messages)) else np.zeros(1, np.uint8)
        return np.ascontiguousarray(blob), offsets, lengths

    def sha256_batch(self, data: np.ndarray, offsets: np.ndarray, lengths: np.ndarray) -> np.ndarray:
        n = len(lengths)
        out = np.zeros((max(n, 1), 32), np.uint8)
        data = np.ascontiguousarray(data, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        lengths = np.ascontiguousarray(lengths, np.uint32)
        _check(self._L.pbftv_sha256_batch(self._h, data.ctypes.data, offsets.ctypes.data, lengths.ctypes.data, n,
                                          out.ctypes.data))
        return out[:n]

    def digest_check_batch(self, data, offsets, lengths, expected: np.ndarray) -> np.ndarray:
        n = len(lengths)
        bm = np.zeros((n + 7) // 8 + 1, np.uint8)
        data = np.ascontiguousarray(data, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        lengths = np.ascontiguousarray(lengths, np.uint32)
        expected = np.ascontiguousarray(expected, np.uint8)
        _check(self._L.pbftv_digest_check_batch(self._h, data.ctypes.data, offsets.ctypes.data, lengths.ctypes.data,
                                                expected.ctypes.data, n, bm.ctypes.data))
        return bitmap_to_bool(bm, n)

    def digest_request_batch(self, requests) -> np.ndarray:
        """requests: RequestColumns, or a list of (timestamp, clientID bytes, operation bytes, sequenceID)."""
        cols = requests if isinstance(requests, RequestColumns) else RequestColumns(requests)
        out = np.zeros((max(cols.n, 1), 32), np.uint8)
        _check(self._L.pbftv_digest_request_batch(self._h, cols.n, *cols.args(), out.ctypes.data))
        return out[:cols.n]

    def digest_vote_batch(self, votes) -> np.ndarray:
        """votes: VoteColumns, or a list of (viewID, sequenceID, digest bytes, nodeID bytes, msgType)."""
        cols = votes if isinstance(votes, VoteColumns) else VoteColumns(votes)
        out = np.zeros((max(cols.n, 1), 32), np.uint8)
        _check(self._L.pbftv_digest_vote_batch(self._h, cols.n, *cols.args(), out.ctypes.data))
        return out[:cols.n]

    def digest_reply_batch(self, replies) -> np.ndarray:
        """replies: ReplyColumns, or a list of (viewID, timestamp, clientID bytes, nodeID bytes, result bytes)."""
        cols = replies if isinstance(replies, ReplyColumns) else ReplyColumns(replies)
        out = np.zeros((max(cols.n, 1), 32), np.uint8)
        _check(self._L.pbftv_digest_reply_batch(self._h, cols.n, *cols.args(), out.ctypes.data))
        return out[:cols.n]

    def digest_preprepare_batch(self, pps) -> np.ndarray:
        """pps: list of (viewID, sequenceID, digest bytes, request) with request
        None (requestMsg nil) or (timestamp, clientID bytes, operation bytes, sequenceID)."""
        n = len(pps)
        v = np.array([x[0] for x in pps], np.int64)
        q = np.array([x[1] for x in pps], np.int64)
        has = np.array([x[3] is not None for x in pps], np.uint8)
        reqs = [x[3] if x[3] is not None else (0, b"", b"", 0) for x in pps]
        rts = np.array([r[0] for r in reqs], np.int64)
        rsq = np.array([r[3] for r in reqs], np.int64)
        db, do, dl = self.pack([x[2] for x in pps])
        cb, co, cl = self.pack([r[1] for r in reqs])
        ob, oo, ol = self.pack([r[2] for r in reqs])
        out = np.zeros((max(n, 1), 32), np.uint8)
        _check(self._L.pbftv_digest_preprepare_batch(self._h, n, v.ctypes.data, q.ctypes.data, db.ctypes.data,
                                                     do.ctypes.data, dl.ctypes.data, has.ctypes.data, rts.ctypes.data,
                                                     cb.ctypes.data, co.ctypes.data, cl.ctypes.data, ob.ctypes.data,
                                                     oo.ctypes.data, ol.ctypes.data, rsq.ctypes.data,
                                                     out.ctypes.data))
        return out[:n]

    def flush_votes(self, cols: "VoteColumns", sigs=None, key_idx=None, states=None, state_idx=None,
                    digests: bool = True):
        """pbftv_flush_votes: (digests | None, sig_ok | None, msg_ok | None).
        states: (view_ids int64[k], last_seqs int64[k], req_digests uint8[k, 32])."""
        self._sync_env()
        n = cols.n
        nb = (n + 7) // 8 + 1
        out_d = np.zeros((max(n, 1), 32), np.uint8) if digests else None
        sbm = np.zeros(nb, np.uint8) if sigs is not None else None
        mbm = np.zeros(nb, np.uint8) if states is not None else None
        sp = kp = svp = slp = sdp = sip = None
        k = 0
        if sigs is not None:
            sigs = np.ascontiguousarray(sigs, np.uint8)
            key_idx = np.ascontiguousarray(key_idx, np.uint32)
            if sigs.shape != (n, 64) or key_idx.shape != (n,):
                raise ValueError("flush_votes: sigs must be (n, 64) uint8 and key_idx (n,)")
            sp, kp = sigs.ctypes.data, key_idx.ctypes.data
        if states is not None:
            sv = np.ascontiguousarray(states[0], np.int64)
            sl = np.ascontiguousarray(states[1], np.int64)
            sd = np.ascontiguousarray(states[2], np.uint8)
            si = np.ascontiguousarray(state_idx, np.uint32)
            k = len(sv)
            if sl.shape != (k,) or sd.shape != (k, 32) or si.shape != (n,):
                raise ValueError("flush_votes: states must be (k,), (k,), (k, 32) and state_idx (n,)")
            svp, slp, sdp, sip = sv.ctypes.data, sl.ctypes.data, sd.ctypes.data, si.ctypes.data
        _check(self._L.pbftv_flush_votes(self._h, n, *cols.args(), sp, kp, k, svp, slp, sdp, sip,
                                         _ptr(out_d), _ptr(sbm), _ptr(mbm)))
        return (out_d[:n] if digests else None, bitmap_to_bool(sbm, n) if sbm is not None else None,
                bitmap_to_bool(mbm, n) if mbm is not None else None)

    def flush_requests(self, cols: "RequestColumns", sigs=None, key_idx=None, assigned_seqs=None,
                       digests: bool = True):
        """pbftv_flush_requests: (digests | None, sig_ok | None, consensus digests | None)."""
        self._sync_env()
        n = cols.n
        S, K, sbm = _sig_inputs(n, sigs, key_idx, "flush_requests")
        out_d = np.zeros((max(n, 1), 32), np.uint8) if digests else None
        aseq = out_c = None
        if assigned_seqs is not None:
            aseq = np.ascontiguousarray(assigned_seqs, np.int64)
            if aseq.shape != (n,):
                raise ValueError("flush_requests: assigned_seqs must be (n,)")
            out_c = np.zeros((max(n, 1), 32), np.uint8)
        _check(self._L.pbftv_flush_requests(self._h, n, *cols.args(), _ptr(S), _ptr(K), _ptr(aseq), _ptr(out_d),
                                            _ptr(sbm), _ptr(out_c)))
        return (out_d[:n] if out_d is not None else None, bitmap_to_bool(sbm, n) if sbm is not None else None,
                out_c[:n] if out_c is not None else None)

    def flush_replies(self, cols: "ReplyColumns", sigs=None, key_idx=None, digests: bool = True):
        """pbftv_flush_replies: (digests | None, sig_ok | None)."""
        self._sync_env()
        n = cols.n
        S, K, sbm = _sig_inputs(n, sigs, key_idx, "flush_replies")
        out_d = np.zeros((max(n, 1), 32), np.uint8) if digests else None
        _check(self._L.pbftv_flush_replies(self._h, n, *cols.args(), _ptr(S), _ptr(K), _ptr(out_d), _ptr(sbm)))
        return (out_d[:n] if out_d is not None else None, bitmap_to_bool(sbm, n) if sbm is not None else None)

    def flush_preprepares(self, cols: "PrePrepareColumns", sigs=None, key_idx=None, states=None, state_idx=None,
                          digests: bool = True, req_digests: bool = False):
        """pbftv_flush_preprepares: (digests | None, request digests | None, sig_ok | None, msg_ok | None).
        states: (view_ids int64[k], last_seqs int64[k])."""
        self._sync_env()
        n = cols.n
        S, K, sbm = _sig_inputs(n, sigs, key_idx, "flush_preprepares")
        out_d = np.zeros((max(n, 1), 32), np.uint8) if digests else None
        out_r = np.zeros((max(n, 1), 32), np.uint8) if req_digests else None
        k, sv, sl, si, mbm = 0, None, None, None, None
        if states is not None:
            k, sv, sl, _, si = _states(n, states, state_idx, "flush_preprepares", False)
            mbm = np.zeros((n + 7) // 8 + 1, np.uint8)
        _check(self._L.pbftv_flush_preprepares(self._h, n, *cols.args(), _ptr(S), _ptr(K), k, _ptr(sv), _ptr(sl),
                                               _ptr(si), _ptr(out_d), _ptr(out_r), _ptr(sbm), _ptr(mbm)))
        return (out_d[:n] if out_d is not None else None, out_r[:n] if out_r is not None else None,
                bitmap_to_bool(sbm, n) if sbm is not None else None,
                bitmap_to_bool(mbm, n) if mbm is not None else None)

    # ---- ecdsa
    def register_keys(self, pub_xy: np.ndarray) -> np.ndarray:
        pub_xy = np.ascontiguousarray(pub_xy, np.uint8).reshape(-1, 64)
        k = pub_xy.shape[0]
        valid = np.zeros(max(k, 1), np.uint8)
        _check(self._L.pbftv_register_keys(self._h, pub_xy.ctypes.data, k, valid.ctypes.data))
        return valid[:k].astype(bool)

    def add_keys(self, pub_xy: np.ndarray) -> np.ndarray:
        """pbftv_add_keys: append keys (indices after the registered ones); their validity."""
        pub_xy = np.ascontiguousarray(pub_xy, np.uint8).reshape(-1, 64)
        k = pub_xy.shape[0]
        valid = np.zeros(max(k, 1), np.uint8)
        _check(self._L.pbftv_add_keys(self._h, pub_xy.ctypes.data, k, valid.ctypes.data))
        return valid[:k].astype(bool)

    def set_key(self, index: int, pub_xy) -> bool:
        """pbftv_set_key: replace key `index` in place; its validity."""
        pub = np.ascontiguousarray(pub_xy, np.uint8).reshape(64)
        valid = np.zeros(1, np.uint8)
        _check(self._L.pbftv_set_key(self._h, index, pub.ctypes.data, valid.ctypes.data))
        return bool(valid[0])

    def table_config(self):
        """(G window bits, key window bits, table bytes per device)."""
        g, q, b = ctypes.c_int(), ctypes.c_int(), ctypes.c_uint64()
        _check(self._L.pbftv_table_config(self._h, ctypes.byref(g), ctypes.byref(q), ctypes.byref(b)))
        return g.value, q.value, b.value

    def verify_batch(self, hashes: np.ndarray, sig_rs: np.ndarray, key_idx: np.ndarray) -> np.ndarray:
        self._sync_env()
        hashes = np.ascontiguousarray(hashes, np.uint8).reshape(-1, 32)
        sig_rs = np.ascontiguousarray(sig_rs, np.uint8).reshape(-1, 64)
        key_idx = np.ascontiguousarray(key_idx, np.uint32)
        n = hashes.shape[0]
        assert sig_rs.shape[0] == n and key_idx.shape[0] == n
        bm = np.zeros((n + 7) // 8 + 1, np.uint8)
        _check(self._L.pbftv_ecdsa_p256_verify_batch(self._h, hashes.ctypes.data, sig_rs.ctypes.data,
                                                     key_idx.ctypes.data, n, bm.ctypes.data))
        return bitmap_to_bool(bm, n)

    def verify_batch_dev(self, dev: int, d_hashes: int, d_sigs: int, d_key_idx: int, n: int, d_bitmap: int,
                         stream: int | None = None):
        self._sync_env()
        _check(self._L.pbftv_ecdsa_p256_verify_batch_dev(self._h, dev, d_hashes, d_sigs, d_key_idx, n, d_bitmap,
                                                         stream))

    def sha256_order_dev(self, dev: int, d_lengths: int, n: int, d_order: int, stream: int | None = None):
        _check(self._L.pbftv_sha256_order_dev(self._h, dev, d_lengths, n, d_order, stream))

    def sha256_batch_dev(self, dev: int, d_data: int, d_offsets: int, d_lengths: int, d_order: int | None, n: int,
                         d_digests: int, d_expected: int | None = None, d_bitmap: int | None = None,
                         stream: int | None = None):
        _check(self._L.pbftv_sha256_batch_dev(self._h, dev, d_data, d_offsets, d_lengths, d_order, n, d_digests,
                                              d_expected, d_bitmap, stream))

    def qc_verify_prepared(self, hashes, sig_rs, key_idx, quorum: int):
        """A zero-argument callable running pbftv_qc_verify on fixed inputs with every
        argument marshalled once (the per-call cost is then the library's plus one
        ctypes call, as for a cgo caller); returns (accepted, quorum reached)."""
        self._sync_env()
        hashes = np.ascontiguousarray(hashes, np.uint8).reshape(-1, 32)
        sig_rs = np.ascontiguousarray(sig_rs, np.uint8).reshape(-1, 64)
        key_idx = np.ascontiguousarray(key_idx, np.uint32)
        n = hashes.shape[0]
        bm = np.zeros((n + 7) // 8 + 1, np.uint8)
        acc, ok = ctypes.c_uint64(), ctypes.c_int()
        fn = self._L.pbftv_qc_verify
        args = (self._h, _vp(hashes.ctypes.data), _vp(sig_rs.ctypes.data), _vp(key_idx.ctypes.data),
                ctypes.c_uint64(n), ctypes.c_uint32(quorum), _vp(bm.ctypes.data), ctypes.byref(acc),
                ctypes.byref(ok))

        def call():
            _check(fn(*args))
            return acc.value, bool(ok.value)
        call.keep = (hashes, sig_rs, key_idx, bm)  # the buffers live as long as the callable
        return call

    def qc_verify(self, hashes, sig_rs, key_idx, quorum: int):
        self._sync_env()
        hashes = np.ascontiguousarray(hashes, np.uint8).reshape(-1, 32)
        sig_rs = np.ascontiguousarray(sig_rs, np.uint8).reshape(-1, 64)
        key_idx = np.ascontiguousarray(key_idx, np.uint32)
        n = hashes.shape[0]
        bm = np.zeros((n + 7) // 8 + 1, np.uint8)
        acc = ctypes.c_uint64()
        ok = ctypes.c_int()
        _check(self._L.pbftv_qc_verify(self._h, hashes.ctypes.data, sig_rs.ctypes.data, key_idx.ctypes.data, n,
                                       quorum, bm.ctypes.data, ctypes.byref(acc), ctypes.byref(ok)))
        return bitmap_to_bool(bm, n), int(acc.value), bool(ok.value)
