"""GPU parity for every comb table geometry (uniform W-bit windows and the
mixed 21 / 29 codes, p256_algo.h CombGeom): the golden vectors, oracle-signed
random batches and the crafted doubling/cancellation sums, through the lane
and the wave path.  A module of its own so that no other context holds tables
while these force the large ones (G at 29 alone is 120 GB of HBM)."""
from __future__ import annotations


import numpy as np
import pytest

from conftest import crafted_exceptional, fixture_arrays, oracle_sign_pool

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
