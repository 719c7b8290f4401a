"""The synthetic config-4 / certificate generator the bench and the GPU tests
rely on (tools/synth.py, tools/synth_sign.c): every signature distinct, valid
under the oracle unless corrupted, and the corruption mask exact.  CPU only."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture(scope="module")
def synth():
    so = os.path.join(ROOT, "tools", "libsynth_sign.so")
    if not os.path.exists(so):  # build() makes it; build it here if the suite runs first
        subprocess.run(["cc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tools", "synth_sign.c"),
                        "-lcrypto", "-lpthread"], check=True)
    import synth as s
    return s


def _oracle_bits(oracle_lib, pub, H, S, K):
    n = len(K)
    bm = np.zeros((n + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, n, pub.ctypes.data,
                                              len(pub), bm.ctypes.data, 8)
    return np.unpackbits(bm, bitorder="little")[:n].astype(bool)


def test_config4_distinct_and_oracle_valid(synth, oracle_lib):
    n = 20_000  # the batch signer's path (>= 4096)
    pub, H, S, K, ok = synth.config4(n, n_keys=100, seed=0x50424654)
    assert S.shape == (n, 64) and H.shape == (n, 32) and K.shape == (n,)
    assert len(np.unique(np.concatenate([H, S], 1), axis=0)) == n  # no repeated (hash, signature)
    assert ok.sum() == n - round(0.01 * n)
    sample = np.random.default_rng(5).choice(n, 1500, replace=False)
    sample = np.union1d(sample, np.nonzero(~ok)[0])  # every corrupted one, plus a sample
    got = _oracle_bits(oracle_lib, pub, H[sample].copy(), S[sample].copy(), K[sample].copy())
    assert (got == ok[sample]).all()


def test_certs_distinct_quorums(synth, oracle_lib):
    per, n_certs = 3, 2000  # 6,000 signatures through the batch signer
    pub, H, S, K = synth.certs(4, per, n_certs, seed=11)
    assert len(np.unique(S, axis=0)) == per * n_certs
    Kc = K.reshape(n_certs, per)
    assert all(len(set(r)) == per for r in Kc.tolist())  # distinct replicas per certificate
    assert (H.reshape(n_certs, per, 32) == H.reshape(n_certs, per, 32)[:, :1]).all()  # one digest per certificate
    idx = np.arange(0, per * n_certs, 7)
    assert _oracle_bits(oracle_lib, pub, H[idx].copy(), S[idx].copy(), K[idx].copy()).all()
