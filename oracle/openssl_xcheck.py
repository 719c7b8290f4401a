"""OpenSSL 3.0 libcrypto cross-check -- TEST INFRASTRUCTURE ONLY.

An implementation of ECDSA-P256 and SHA-256 independent of both the oracle
restatement and the GPU kernels, used to pin the oracle:
every committed ECDSA fixture must get the same accept/reject from
OpenSSL's ``ECDSA_do_verify`` as from ``oracle/p256.py`` and
``oracle/liboracle.so``.  Keys OpenSSL refuses to load (off-curve, coordinate
>= p, the point at infinity) count as reject, matching the batch verifier's
registration-time key check.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import hashlib

NID_X9_62_prime256v1 = 415

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        L = ctypes.CDLL(path)
        L.EC_KEY_new_by_curve_name.restype = ctypes.c_void_p
        L.EC_KEY_new_by_curve_name.argtypes = [ctypes.c_int]
        L.EC_KEY_free.argtypes = [ctypes.c_void_p]
        L.BN_bin2bn.restype = ctypes.c_void_p
        L.BN_bin2bn.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p]
        L.BN_free.argtypes = [ctypes.c_void_p]
        L.EC_KEY_set_public_key_affine_coordinates.restype = ctypes.c_int
        L.EC_KEY_set_public_key_affine_coordinates.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.ECDSA_SIG_new.restype = ctypes.c_void_p
        L.ECDSA_SIG_free.argtypes = [ctypes.c_void_p]
        L.ECDSA_SIG_set0.restype = ctypes.c_int
        L.ECDSA_SIG_set0.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.ECDSA_do_verify.restype = ctypes.c_int
        L.ECDSA_do_verify.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.ERR_clear_error.argtypes = []
        _lib = L
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except OSError:
        return False


def ecdsa_verify(h: bytes, r: int, s: int, qx: int, qy: int) -> bool:
    L = lib()
    key = L.EC_KEY_new_by_curve_name(NID_X9_62_prime256v1)
    try:
        # coordinates >= p are refused by the affine setter; encode with enough bytes
        xb = qx.to_bytes(max(32, (qx.bit_length() + 7) // 8), "big")
        yb = qy.to_bytes(max(32, (qy.bit_length() + 7) // 8), "big")
        bx = L.BN_bin2bn(xb, len(xb), None)
        by = L.BN_bin2bn(yb, len(yb), None)
        ok = L.EC_KEY_set_public_key_affine_coordinates(key, bx, by)
        L.BN_free(bx)
        L.BN_free(by)
        if ok != 1:
            L.ERR_clear_error()
            return False
        sig = L.ECDSA_SIG_new()
        rb = r.to_bytes(max(32, (r.bit_length() + 7) // 8), "big")
        sb = s.to_bytes(max(32, (s.bit_length() + 7) // 8), "big")
        br = L.BN_bin2bn(rb, len(rb), None)
        bs = L.BN_bin2bn(sb, len(sb), None)
        L.ECDSA_SIG_set0(sig, br, bs)
        res = L.ECDSA_do_verify(h, len(h), sig, key)
        L.ECDSA_SIG_free(sig)
        L.ERR_clear_error()
        return res == 1
    finally:
        L.EC_KEY_free(key)


def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()
