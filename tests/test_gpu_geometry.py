"""GPU parity for every comb table geometry (uniform W-bit windows and the
mixed 21 / 29 codes, p256_algo.h CombGeom): the golden vectors, oracle-signed
random batches and the crafted doubling/cancellation sums, through the lane
and the wave path.  A module of its own so that no other context holds tables
while these force the large ones (G at 29 alone is 120 GB of HBM)."""
from __future__ import annotations


import numpy as np
import pytest

from conftest import chosen_scalar_sig, crafted_exceptional, fixture_arrays, oracle_sign_pool, signed_digits

pytestmark = pytest.mark.gpu

# every (G, key) pair with instantiated kernels (kernels.h PBFTV_COMBOS)
GEOMETRIES = [(29, 24), (29, 22), (29, 21), (29, 20), (29, 16), (26, 24), (26, 22), (26, 21), (26, 20), (26, 16),
              (24, 24), (24, 22), (24, 20), (20, 20), (24, 16), (16, 16), (16, 12), (16, 8), (8, 8)]
GEOMETRIES_CRAFTED = [(29, 24), (29, 21), (26, 24), (26, 22), (26, 21), (24, 24), (24, 22), (24, 20), (20, 20),
                      (24, 16), (16, 16), (16, 8), (8, 8)]


@pytest.fixture(params=["wave", "lane"])
def path(request, monkeypatch):
    monkeypatch.setenv("PBFTV_WAVE_MAX", "100000000" if request.param == "wave" else "0")
    return request.param


@pytest.mark.parametrize("gq", GEOMETRIES)
def test_ecdsa_every_table_width(oracle_lib, ecdsa_fixtures, gq, path, monkeypatch):
    """Golden vectors + random corruptions vs the oracle for every comb geometry."""
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_GBITS", str(gq[0]))
    monkeypatch.setenv("PBFTV_QBITS", str(gq[1]))
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    with Verifier() as v:
        assert v.register_keys(keys).tolist() == [k["valid"] for k in ecdsa_fixtures["keys"]]
        assert v.table_config()[:2] == gq
        assert (v.verify_batch(hashes, sigs, kidx) == expect).all()
        pk, h, sg, ki = oracle_sign_pool(oracle_lib, n_keys=5, per_key=50, seed=gq[0] * 100 + gq[1])
        sg[::3, 7] ^= 0x20
        v.register_keys(pk)
        got = v.verify_batch(h, sg, ki)
        n = len(ki)
        bm = np.zeros((n + 7) // 8, np.uint8)
        oracle_lib.oracle_ecdsa_p256_verify_batch(h.ctypes.data, sg.ctypes.data, ki.ctypes.data, n, pk.ctypes.data,
                                                  len(pk), bm.ctypes.data, 8)
        assert (got == np.unpackbits(bm, bitorder="little")[:n].astype(bool)).all()



@pytest.mark.parametrize("gq", GEOMETRIES_CRAFTED)
def test_ecdsa_crafted_exceptional_sums(gq, path, monkeypatch):
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_GBITS", str(gq[0]))
    monkeypatch.setenv("PBFTV_QBITS", str(gq[1]))
    key, H, S, K, E = crafted_exceptional()
    assert E.sum() >= 10  # the crafted ones verify, the r-flipped ones do not
    with Verifier() as v:
        v.register_keys(key)
        assert v.table_config()[:2] == gq
        assert (v.verify_batch(H, S, K) == E).all()


@pytest.mark.parametrize("gq", [(29, 21), (29, 24), (26, 22), (16, 16), (8, 8)])
def test_comb_schedule_edge_digits(oracle_lib, gq, monkeypatch):
    """k_ecdsa_comb's per-wave schedule (verify_kernels.h; p256_algo.h
    comb2_verify): waves whose lanes all have non-zero first digits add the
    first two points affine + affine and fuse the last addition with the x
    check; a lane with a zero first digit (of u1 or u2) or a zero last digit
    sends its whole wave through the generic steps.  Chosen-scalar signatures
    under Q = G put such lanes into some waves of an oracle-signed batch, plus
    last-step doublings and cancellations (the fused check reports them, the
    complete-addition rerun decides), each also with r corrupted; every bit
    against the oracle."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import window_widths
    from oracle import p256
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_GBITS", str(gq[0]))
    monkeypatch.setenv("PBFTV_QBITS", str(gq[1]))
    monkeypatch.setenv("PBFTV_WAVE_MAX", "0")
    N = p256.N
    rng = np.random.default_rng(gq[0] * 64 + gq[1])
    qw = window_widths(gq[1])
    last_bit = sum(qw[:-1])

    def rnd(bits):
        return int.from_bytes(rng.bytes(32), "big") % (1 << bits) % N or 1

    crafted = []  # (u1, u2): one per kind
    crafted.append((rnd(224) << 32, rnd(256)))          # zero first G digit
    crafted.append((rnd(256), rnd(224) << 32))          # zero first Q digit
    crafted.append((rnd(256), rnd(last_bit - 2)))       # zero last (Q) digit
    for _ in range(3):                                  # last-step doubling and cancellation
        while True:
            u2 = rnd(256)
            d, b = signed_digits(u2, qw)[-1]
            if d != 0:
                break
        crafted.append(((2 * d * (1 << b) - u2) % N, u2))
        crafted.append(((-u2) % N, u2))
    crafted.append((rnd(256), rnd(256)))                # plain
    assert signed_digits(crafted[2][1], qw)[-1][0] == 0
    pk, h, sg, ki = oracle_sign_pool(oracle_lib, n_keys=4, per_key=400, seed=gq[0] + gq[1])
    keys = np.concatenate([np.frombuffer(p256.GX.to_bytes(32, "big") + p256.GY.to_bytes(32, "big"),
                                         np.uint8)[None, :], pk])
    ki = ki + 1
    sg[::5, 9] ^= 0x40
    H, S, K = list(h), list(sg), list(ki)
    # crafted lane j of kind c at wave 2 c + j (two waves per kind), lane 7 + 13 j
    for c, (u1, u2) in enumerate(crafted):
        for j, flip in enumerate((False, True)):
            hh, rs, _ = chosen_scalar_sig(u1, u2, flip)
            at = 64 * (2 * c + j) + 7 + 13 * j
            H.insert(at, hh)
            S.insert(at, rs)
            K.insert(at, 0)
    H, S, K = np.stack(H), np.stack(S), np.array(K, np.uint32)
    n = len(K)
    with Verifier() as v:
        v.register_keys(keys)
        assert v.table_config()[:2] == gq
        got = v.verify_batch(H, S, K)
    bm = np.zeros((n + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, n, keys.ctypes.data,
                                              len(keys), bm.ctypes.data, 8)
    want = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    assert (got == want).all(), np.nonzero(got != want)[0][:20]
    ck = [64 * (2 * c + j) + 7 + 13 * j for c in range(len(crafted)) for j in range(2)]
    assert want[ck[0::2]].sum() >= len(crafted) - 3   # the unflipped ones verify (cancellations do not)
    assert not want[ck[1::2]].any()
