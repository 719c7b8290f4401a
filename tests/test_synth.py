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


def _config1_oracle(oracle_lib, c):
    """Per message kind: the oracle's signature verdicts and verifyMsg verdicts
    for a config-1 cluster (oracle/gojson.py preimages, the oracle verify,
    oracle_verify_msg against each message's State)."""
    import hashlib
    from oracle import gojson
    pub = c["pub"]
    out = {}

    def sig_bits(pre, S, K):
        H = np.frombuffer(b"".join(hashlib.sha256(p).digest() for p in pre), np.uint8).reshape(-1, 32).copy()
        return _oracle_bits(oracle_lib, pub, H, np.ascontiguousarray(S), np.ascontiguousarray(K, np.uint32))
    out["request_sig"] = sig_bits([gojson.request(*r) for r in c["requests"]], c["request_sigs"],
                                  np.full(len(c["requests"]), 4, np.uint32))
    out["preprepare_sig"] = sig_bits([gojson.preprepare(*p) for p in c["preprepares"]], c["preprepare_sigs"],
                                     np.zeros(len(c["preprepares"]), np.uint32))
    nodes = {b"MainNode": 0, b"ReplicaNode1": 1, b"ReplicaNode2": 2, b"ReplicaNode3": 3}
    out["vote_sig"] = sig_bits([gojson.vote(*v) for v in c["votes"]], c["vote_sigs"],
                               np.array([nodes[v[3]] for v in c["votes"]], np.uint32))
    out["reply_sig"] = sig_bits([gojson.reply(*r) for r in c["replies"]], c["reply_sigs"],
                                np.array([nodes[r[3]] for r in c["replies"]], np.uint32))
    req_d = [hashlib.sha256(gojson.request(r[0], r[1], r[2], int(a))).digest()
             for r, a in zip(c["requests"], c["assigned_seqs"])]
    sv, sl = c["state_view"], c["state_last"]

    def msg_bits(msgs, states, own_digest):
        res = []
        for m, st in zip(msgs, states):
            d = own_digest(m, st)
            res.append(oracle_lib.oracle_verify_msg(int(sv[st]), int(sl[st]), d, m[0], m[1], m[2], len(m[2])) == 1)
        return np.array(res)
    # State.PrePrepare: ReqMsg = the embedded request (pbft_impl.go:91-99)
    out["preprepare_msg"] = msg_bits(c["preprepares"], c["preprepare_state"],
                                     lambda m, st: hashlib.sha256(gojson.request(*m[3])).digest())
    out["vote_msg"] = msg_bits(c["votes"], c["vote_state"], lambda m, st: req_d[st])
    return out


def test_config1_corruptions_match_oracle(synth, oracle_lib):
    """The config-1 construction's expected bits (synth.config1_cluster) equal
    the oracle's on every message, every corruption class occurs, and the bench
    check rejects an all-accept verifier."""
    sys.path.insert(0, ROOT)
    import bench
    c = synth.config1_cluster(200)
    want = _config1_oracle(oracle_lib, c)
    for k in ("request_sig", "preprepare_sig", "preprepare_msg", "vote_sig", "vote_msg", "reply_sig"):
        key = k.rsplit("_", 1)[0] + "_" + k.rsplit("_", 1)[1] + "_ok"
        assert (want[k] == c[key]).all(), k
        assert not want[k].all(), k
    assert sorted(set(c["vote_class"].values())) == [0, 1, 2, 3]
    assert sorted(set(c["preprepare_class"].values())) == [0, 1, 2, 3]
    expect = {k: c[k + "_ok"] for k in want}
    assert bench.check_config1({k: v.copy() for k, v in expect.items()}, expect)[0]
    assert not bench.check_config1({k: np.ones_like(v) for k, v in expect.items()}, expect)[0]


def test_cert_corruptions_and_check(synth, oracle_lib):
    """synth.corrupt_certs: the mask equals the oracle on every corrupted vote and
    a sample; bench.check_certs accepts the true bits and rejects all-ones and a
    bitmap with one extra rejection."""
    sys.path.insert(0, ROOT)
    import bench
    per, n_certs = 3, 2000
    pub, H, S, K = synth.certs(4, per, n_certs, seed=11)
    want, bad_any, bad_two = synth.corrupt_certs(H, S, K, per, 4)
    assert len(bad_any) == 30 and len(bad_two) == 10 and (~want).sum() == 20 + 20
    idx = np.union1d(np.nonzero(~want)[0], np.arange(0, per * n_certs, 11))
    assert (_oracle_bits(oracle_lib, pub, H[idx].copy(), S[idx].copy(), K[idx].copy()) == want[idx]).all()
    assert bench.check_certs(want, want, per, bad_any, bad_two, 2)
    assert not bench.check_certs(np.ones_like(want), want, per, bad_any, bad_two, 2)
    w2 = want.copy()
    w2[np.nonzero(want)[0][0]] = False
    assert not bench.check_certs(w2, want, per, bad_any, bad_two, 2)
