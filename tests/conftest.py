"""Shared fixtures.  GPU tests are marked ``@pytest.mark.gpu`` (run on the MI355X
box with ``-m gpu``); everything else runs on the CPU of this container."""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


def _load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ecdsa_fixtures():
    return _load_json("ecdsa.json")


@pytest.fixture(scope="session")
def sha_fixtures():
    return _load_json("sha256.json")


@pytest.fixture(scope="session")
def digest_kats():
    return _load_json("digest_kats.json")


def _build(path_so, make_dir):
    if not os.path.exists(path_so):
        subprocess.run(["make", "-C", make_dir, "-s"], check=True)
    return path_so


@pytest.fixture(scope="session")
def oracle_lib():
    """The CPU oracle (test infrastructure) -- checker only."""
    so = _build(os.path.join(ROOT, "oracle", "liboracle.so"), os.path.join(ROOT, "oracle"))
    L = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    L.oracle_sha256.argtypes = [vp, ctypes.c_uint64, vp]
    L.oracle_hash_hex.argtypes = [vp, ctypes.c_uint64, ctypes.c_char_p]
    L.oracle_sha256_batch.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_int]
    L.oracle_p256_key_valid.argtypes = [vp]
    L.oracle_ecdsa_p256_verify.argtypes = [vp, vp, vp]
    L.oracle_ecdsa_p256_verify_batch.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint32, vp, ctypes.c_int]
    L.oracle_p256_pubkey.argtypes = [vp, vp]
    L.oracle_ecdsa_p256_sign.argtypes = [vp, vp, vp, vp]
    L.oracle_gojson_request.restype = ctypes.c_uint64
    L.oracle_gojson_request.argtypes = [ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                        ctypes.c_uint64, ctypes.c_int64, vp, ctypes.c_uint64]
    L.oracle_gojson_vote.restype = ctypes.c_uint64
    L.oracle_gojson_vote.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                     ctypes.c_uint64, ctypes.c_int64, vp, ctypes.c_uint64]
    L.oracle_gojson_reply.restype = ctypes.c_uint64
    L.oracle_gojson_reply.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint64,
                                      ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64, vp,
                                      ctypes.c_uint64]
    L.oracle_gojson_preprepare.restype = ctypes.c_uint64
    L.oracle_gojson_preprepare.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint64,
                                           ctypes.c_int, ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint64,
                                           ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int64, vp, ctypes.c_uint64]
    L.oracle_verify_msg.argtypes = [ctypes.c_int64, ctypes.c_int64, vp, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_char_p, ctypes.c_uint64]
    return L


def fixture_arrays(fx):
    """ECDSA fixtures -> (keys[k,64], hashes[n,32], sigs[n,64], key_idx[n], expect[n])."""
    keys = np.array([list(bytes.fromhex(k["x"]) + bytes.fromhex(k["y"])) for k in fx["keys"]], np.uint8)
    vs = fx["vectors"]
    hashes = np.array([list(bytes.fromhex(v["hash"])) for v in vs], np.uint8)
    sigs = np.array([list(bytes.fromhex(v["r"]) + bytes.fromhex(v["s"])) for v in vs], np.uint8)
    kidx = np.array([v["key"] for v in vs], np.uint32)
    expect = np.array([v["expect"] for v in vs], bool)
    return keys, hashes, sigs, kidx, expect


def oracle_sign_pool(oracle_lib, n_keys: int, per_key: int, seed: int):
    """Deterministic valid signatures made with the oracle's textbook signer."""
    rng = np.random.default_rng(seed)
    N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
    keys = np.zeros((n_keys, 64), np.uint8)
    privs = []
    for k in range(n_keys):
        d = int.from_bytes(rng.bytes(32), "big") % (N - 1) + 1
        privs.append(d.to_bytes(32, "big"))
        out = np.zeros(64, np.uint8)
        assert oracle_lib.oracle_p256_pubkey(privs[-1], out.ctypes.data) == 1
        keys[k] = out
    n = n_keys * per_key
    hashes = np.frombuffer(rng.bytes(32 * n), np.uint8).reshape(n, 32).copy()
    sigs = np.zeros((n, 64), np.uint8)
    kidx = np.repeat(np.arange(n_keys, dtype=np.uint32), per_key)
    for i in range(n):
        while True:
            kb = rng.bytes(32)
            if oracle_lib.oracle_ecdsa_p256_sign(hashes[i].ctypes.data, privs[kidx[i]], kb, sigs[i].ctypes.data):
                break
    return keys, hashes, sigs, kidx


def signed_digits(u: int, widths) -> list:
    """Signed recoding of u over windows of the given widths (p256_algo.h
    signed_digit_w): [(digit, start bit)]."""
    out, c, bit = [], 0, 0
    for wd in widths:
        d = ((u >> bit) & ((1 << wd) - 1)) + c
        c = 1 if d > (1 << (wd - 1)) else 0
        out.append((d - (c << wd), bit))
        bit += wd
    return out


def chosen_scalar_sig(u1: int, u2: int, flip_r: bool = False):
    """A signature under the key Q = G whose verify recomputes exactly (u1, u2):
    R = (u1 + u2) G, r = x(R) mod n (r = 1 when R is infinity: rejected),
    s = r / u2, e = u1 s.  Returns (hash, r||s, expected accept bit)."""
    from oracle import p256
    N = p256.N
    R = p256.scalar_mult((u1 + u2) % N, p256.G)
    r = 1 if R is None else R[0] % N
    s = r * pow(u2, -1, N) % N
    e = u1 * s % N
    h = e.to_bytes(32, "big")
    if flip_r:
        r ^= 2
    rs = r.to_bytes(32, "big") + s.to_bytes(32, "big")
    return (np.frombuffer(h, np.uint8), np.frombuffer(rs, np.uint8),
            p256.verify(h, r, s, p256.GX, p256.GY))


def crafted_exceptional():
    """Valid signatures with chosen (u1, u2) under the key Q = G: pick u1, u2,
    R = (u1 + u2) G, r = x(R) mod n, s = r / u2, e = u1 s (the verifier then
    recomputes exactly u1, u2).  The (u1, u2) pairs make table points meet
    inside the sum -- at the first (G entry + Q entry) level and at the
    butterfly / comb levels -- for every window geometry, so every doubling
    and cancellation path (and the exact reruns behind them) is exercised.
    Expected bits come from the oracle restatement (parity pinned by the
    golden fixtures)."""
    from oracle import p256
    N = p256.N
    pairs = [(5, 5), (77 << 24, 77 << 24), (3 << 20, 3 << 20), (1 << 16, 1 << 16), (9 << 8, 9 << 8),
             ((1 << 23) + 1, (1 << 23) + 1), (12345, 2 * 12345), (1 << 20, (1 << 24) - (1 << 20)),
             ((5 << 40) + 7, (5 << 40) + 7), ((3 << 20) + (1 << 24), 3 << 20), (2, N - 2),
             (0xABCDEF << 48, 0xABCDEF << 48), (N - 1, N - 1), (N - 5, 5 + (1 << 30))]
    H, S, K, E = [], [], [], []
    for u1, u2 in pairs:
        R = p256.scalar_mult((u1 + u2) % N, p256.G)
        if R is None:  # u1 + u2 == 0: any well-formed signature with these scalars is rejected
            r = 1
        else:
            r = R[0] % N
        s = r * pow(u2, -1, N) % N
        e = u1 * s % N
        h = e.to_bytes(32, "big")
        for rr, ss, hh in ((r, s, h), (r ^ 2, s, h)):
            H.append(np.frombuffer(hh, np.uint8))
            S.append(np.frombuffer(rr.to_bytes(32, "big") + ss.to_bytes(32, "big"), np.uint8))
            K.append(0)
            E.append(p256.verify(hh, rr, ss, p256.GX, p256.GY))
    key = np.frombuffer(p256.GX.to_bytes(32, "big") + p256.GY.to_bytes(32, "big"), np.uint8)[None, :]
    return key, np.stack(H), np.stack(S), np.array(K, np.uint32), np.array(E, bool)
