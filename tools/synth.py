"""Synthetic signed-vote workloads for bench.py.

Signatures are produced with OpenSSL 3 libcrypto (ECDSA_do_sign) -- neither the
product library nor the oracle -- so the benchmark verifies signatures made by
an independent implementation.  Keys are derived deterministically from the
seed; nonces are OpenSSL's own (random), so signatures differ run to run while
the accept/reject pattern is fixed by construction:

    corrupt(i) for i in a seeded 1 % subset, split evenly over the 8 classes of
    SURVEY.md §8(c): flip r, flip s, flip hash, wrong key, r=0, s=0, r=n, s>=n.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import hashlib
import os

import numpy as np

NID_P256 = 415
N_ORDER = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
CLASSES = ["flip r", "flip s", "flip hash", "wrong key", "r=0", "s=0", "r=n", "s>=n"]

_L = None


def _lib():
    global _L
    if _L is None:
        L = ctypes.CDLL(ctypes.util.find_library("crypto") or "libcrypto.so.3")
        vp = ctypes.c_void_p
        L.EC_KEY_new_by_curve_name.restype = vp
        L.EC_KEY_new_by_curve_name.argtypes = [ctypes.c_int]
        L.EC_KEY_get0_group.restype = vp
        L.EC_KEY_get0_group.argtypes = [vp]
        L.EC_KEY_set_private_key.argtypes = [vp, vp]
        L.EC_KEY_set_public_key.argtypes = [vp, vp]
        L.EC_POINT_new.restype = vp
        L.EC_POINT_new.argtypes = [vp]
        L.EC_POINT_free.argtypes = [vp]
        L.EC_POINT_mul.argtypes = [vp, vp, vp, vp, vp, vp]
        L.EC_POINT_get_affine_coordinates.argtypes = [vp, vp, vp, vp, vp]
        L.BN_new.restype = vp
        L.BN_free.argtypes = [vp]
        L.BN_bin2bn.restype = vp
        L.BN_bin2bn.argtypes = [ctypes.c_char_p, ctypes.c_int, vp]
        L.BN_bn2binpad.argtypes = [vp, ctypes.c_char_p, ctypes.c_int]
        L.ECDSA_do_sign.restype = vp
        L.ECDSA_do_sign.argtypes = [ctypes.c_char_p, ctypes.c_int, vp]
        L.ECDSA_SIG_get0_r.restype = vp
        L.ECDSA_SIG_get0_r.argtypes = [vp]
        L.ECDSA_SIG_get0_s.restype = vp
        L.ECDSA_SIG_get0_s.argtypes = [vp]
        L.ECDSA_SIG_free.argtypes = [vp]
        L.EC_KEY_free.argtypes = [vp]
        _L = L
    return _L


class Signer:
    """n_keys deterministic P-256 keys (OpenSSL EC_KEY objects)."""

    def __init__(self, n_keys: int, seed: int):
        L = _lib()
        self.keys = []
        self.pub = np.zeros((n_keys, 64), np.uint8)
        self.priv = np.zeros((n_keys, 32), np.uint8)  # big-endian scalars (the batch signer's input)
        for j in range(n_keys):
            d = int.from_bytes(hashlib.sha256(b"pbft-key:%d:%d" % (seed, j)).digest(), "big") % (N_ORDER - 1) + 1
            self.priv[j] = np.frombuffer(d.to_bytes(32, "big"), np.uint8)
            k = L.EC_KEY_new_by_curve_name(NID_P256)
            grp = L.EC_KEY_get0_group(k)
            db = d.to_bytes(32, "big")
            bn = L.BN_bin2bn(db, 32, None)
            L.EC_KEY_set_private_key(k, bn)
            pt = L.EC_POINT_new(grp)
            L.EC_POINT_mul(grp, pt, bn, None, None, None)
            L.EC_KEY_set_public_key(k, pt)
            bx, by = L.BN_new(), L.BN_new()
            L.EC_POINT_get_affine_coordinates(grp, pt, bx, by, None)
            xb, yb = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
            L.BN_bn2binpad(bx, xb, 32)
            L.BN_bn2binpad(by, yb, 32)
            self.pub[j] = np.frombuffer(xb.raw + yb.raw, np.uint8)
            for b in (bx, by, bn):
                L.BN_free(b)
            L.EC_POINT_free(pt)
            self.keys.append(k)

    def sign(self, h: bytes, j: int) -> bytes:
        L = _lib()
        sig = L.ECDSA_do_sign(h, 32, self.keys[j])
        rb, sb = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
        L.BN_bn2binpad(L.ECDSA_SIG_get0_r(sig), rb, 32)
        L.BN_bn2binpad(L.ECDSA_SIG_get0_s(sig), sb, 32)
        L.ECDSA_SIG_free(sig)
        return rb.raw + sb.raw

    def close(self):
        L = _lib()
        for k in self.keys:
            L.EC_KEY_free(k)
        self.keys = []


_SIGN_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsynth_sign.so")


def _batch_signer():
    """tools/synth_sign.c (built by __graft_entry__.build()): OpenSSL signing on
    host threads; None when it is not built (then the per-signature loop)."""
    if not os.path.exists(_SIGN_SO):
        return None
    L = ctypes.CDLL(_SIGN_SO)
    vp = ctypes.c_void_p
    L.synth_sign_batch.argtypes = [vp, ctypes.c_uint32, vp, vp, ctypes.c_uint64, vp, ctypes.c_int]
    return L


def signed_pool(n_keys: int, pool: int, seed: int):
    """pool distinct (hash, sig, key) triples, keys round-robin."""
    s = Signer(n_keys, seed)
    rng = np.random.default_rng(seed)
    hashes = np.frombuffer(rng.bytes(32 * pool), np.uint8).reshape(pool, 32).copy()
    kidx = (np.arange(pool) % n_keys).astype(np.uint32)
    sigs = np.zeros((pool, 64), np.uint8)
    B = _batch_signer() if pool >= 4096 else None
    if B is not None:
        threads = max(1, min(16, os.cpu_count() or 1))
        rc = B.synth_sign_batch(s.priv.ctypes.data, n_keys, hashes.ctypes.data, kidx.ctypes.data, pool,
                                sigs.ctypes.data, threads)
        if rc != 0:
            raise RuntimeError(f"synth_sign_batch failed: {rc}")
    else:
        for i in range(pool):
            sigs[i] = np.frombuffer(s.sign(hashes[i].tobytes(), int(kidx[i])), np.uint8)
    pub = s.pub.copy()
    s.close()
    return pub, hashes, sigs, kidx


def corrupt_one(hashes, sigs, kidx, i: int, c: int, n_keys: int, rng):
    """Apply corruption class c (CLASSES[c]) to signature i in place."""
    nb = N_ORDER.to_bytes(32, "big")
    if c == 0:
        sigs[i, rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))
    elif c == 1:
        sigs[i, 32 + rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))
    elif c == 2:
        hashes[i, rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))
    elif c == 3:
        kidx[i] = (kidx[i] + 1 + rng.integers(0, n_keys - 1)) % n_keys
    elif c == 4:
        sigs[i, :32] = 0
    elif c == 5:
        sigs[i, 32:] = 0
    elif c == 6:
        sigs[i, :32] = np.frombuffer(nb, np.uint8)
    else:
        sigs[i, 32:] = 0xFF


def corrupt(hashes, sigs, kidx, n_keys: int, frac: float, seed: int):
    """Corrupt a seeded `frac` subset in place, evenly over CLASSES; returns the expected accept mask."""
    n = len(kidx)
    rng = np.random.default_rng(seed ^ 0x5A5A)
    m = int(round(n * frac))
    idx = rng.choice(n, m, replace=False)
    for t, i in enumerate(idx):
        corrupt_one(hashes, sigs, kidx, int(i), t % 8, n_keys, rng)
    ok = np.ones(n, bool)
    ok[idx] = False
    return ok


def config4(n: int, n_keys: int = 100, pool: int = 1 << 20, seed: int = 0x50424654, frac: float = 0.01):
    """n sigs over an n_keys table, `frac` corrupted.
    A pool of min(pool, n) distinct signatures, tiled to n when smaller.  The
    default makes every signature of the 1M batch distinct: with a tiled
    65,536 pool the key order put a lane's repeated copies in neighbouring
    lanes, whose table reads then hit in cache (round-2 PMC: 0.62 GB of HBM per
    comb launch instead of 1.58 GB) -- not a real workload."""
    pub, h, s, k = signed_pool(n_keys, min(pool, n), seed)
    reps = -(-n // len(k))
    H = np.tile(h, (reps, 1))[:n].copy()
    S = np.tile(s, (reps, 1))[:n].copy()
    K = np.tile(k, reps)[:n].copy()
    ok = corrupt(H, S, K, n_keys, frac, seed)
    return pub, H, S, K, ok


def qc(n_keys: int, sigs_per_qc: int, seed: int):
    """One quorum certificate: sigs_per_qc votes over one digest from distinct replicas."""
    s = Signer(n_keys, seed)
    h = hashlib.sha256(b"qc-digest:%d" % seed).digest()
    H = np.tile(np.frombuffer(h, np.uint8), (sigs_per_qc, 1))
    K = (np.arange(sigs_per_qc) % n_keys).astype(np.uint32)
    S = np.stack([np.frombuffer(s.sign(h, int(j)), np.uint8) for j in K])
    pub = s.pub.copy()
    s.close()
    return pub, H, S, K


def sha_config5(n: int, lo: int = 256, hi: int = 4096, seed: int = 0x50424654):
    """n messages of uniform random length in [lo, hi] B, random bytes."""
    rng = np.random.default_rng(seed)
    lengths = rng.integers(lo, hi + 1, n).astype(np.uint32)
    offsets = np.zeros(n, np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    total = int(lengths.sum())
    data = rng.integers(0, 256, total + 64, dtype=np.uint8)
    return data, offsets, lengths


NODES = [b"MainNode", b"ReplicaNode1", b"ReplicaNode2", b"ReplicaNode3"]  # pbft/network/node.go:60-65
VIEW = 10000000000                                                         # node.go:55


CLIENT_KEY = 4  # key index of the (one) client process in config 1

# corruption classes of the config-1 flushes (a Byzantine sender's messages):
# a bad signature, or a validly signed message that State.verifyMsg rejects
# (pbft_impl.go:176-202) -- wrong digest, wrong view, stale sequence ID
MSG_CLASSES = ["bad signature", "wrong digest", "wrong view", "stale sequence"]


def config1_cluster(n_req: int = 1000, seed: int = 0x50424654, bad_frac: float = 0.02) -> dict:
    """the reference's 4-node message pattern for n_req
    requests, every message signed.  Per request: the client's
    request verified by the primary (1), the primary's pre-prepare verified by
    3 replicas (3), 3 replica prepares each verified by 3 peers (9), 4 commits
    each verified by 3 peers (12), 4 replies verified by the client (4) = 29
    signature checks over 13 distinct signed messages.  Keys: the 4 nodes
    (NODES order) and the client (CLIENT_KEY).  The client signs its request
    with sequenceID 0 (as sent); StartConsensus assigns the sequence ID
    (pbft_impl.go:57-67) before the request digest is taken.

    Request i's consensus State has ViewID = VIEW and LastSequenceID = the
    previous request's sequence ID (-1 for the first): the state created after
    request i-1 committed.  A seeded `bad_frac` of each message kind (requests
    and replies: bad signature; pre-prepares and votes: MSG_CLASSES in turn,
    from request 1 on so that a stale sequence exists) is corrupted; the
    expected outcome of every message is returned with it ("*_sig_ok",
    "*_msg_ok"), so an all-accept verifier fails the check."""
    sys_path_fix()
    from simple_pbft_amd import pbftv as gj  # host-only Go-JSON encoder of the product (no GPU)
    s = Signer(5, seed)
    rng = np.random.default_rng(seed ^ 0xC0FF)
    n_votes_per = 7
    bad_req = set(rng.choice(n_req, int(round(n_req * bad_frac)), replace=False).tolist())
    elig = n_req - 1
    bad_pp = rng.choice(elig, max(4, int(round(n_req * bad_frac))), replace=False) + 1
    bad_pp = {int(i): t % 4 for t, i in enumerate(bad_pp)}
    nv = n_req * n_votes_per
    bad_v = rng.choice(nv - n_votes_per, max(4, int(round(nv * bad_frac))), replace=False) + n_votes_per
    bad_v = {int(i): t % 4 for t, i in enumerate(bad_v)}
    bad_rep = set(rng.choice(4 * n_req, int(round(4 * n_req * bad_frac)), replace=False).tolist())
    sent, assigned, req_sig, req_ok = [], [], [], []
    pps, pp_sig, pp_state, pp_sig_ok, pp_msg_ok = [], [], [], [], []
    votes, vote_sig, vote_state, vote_sig_ok, vote_msg_ok = [], [], [], [], []
    replies, reply_sig, reply_ok = [], [], []
    checks = []  # (kind, index, receiver)

    def flip(sig):
        b = bytearray(sig)
        b[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
        return bytes(b)

    def tamper(view, seq, d, cls, i):
        """(view, seq, digest) of a corrupted message of class cls for request i."""
        if cls == 1:
            d = hashlib.sha256(b"other request %d" % i).hexdigest().encode()
        elif cls == 2:
            view += 1
        elif cls == 3:
            seq = assigned[i - 1]  # == the state's LastSequenceID: already committed
        return view, seq, d

    for i in range(n_req):
        req0 = (1668519246 + i, b"client%d" % i, b"printf", 0)
        sent.append(req0)
        sg = s.sign(hashlib.sha256(gj.gojson_request(*req0)).digest(), CLIENT_KEY)
        req_sig.append(flip(sg) if i in bad_req else sg)
        req_ok.append(i not in bad_req)
        seq = 1668519247222762700 + 1000 * i
        assigned.append(seq)
        req = req0[:3] + (seq,)
        checks.append(("request", i, 0))
        d = hashlib.sha256(gj.gojson_request(*req)).hexdigest().encode()
        cls = bad_pp.get(i, -1)
        view_p, seq_p, d_p = tamper(VIEW, seq, d, cls, i) if cls > 0 else (VIEW, seq, d)
        pp = (view_p, seq_p, d_p, req)
        pps.append(pp)
        sg = s.sign(hashlib.sha256(gj.gojson_preprepare(*pp)).digest(), 0)
        pp_sig.append(flip(sg) if cls == 0 else sg)
        pp_state.append(i)
        pp_sig_ok.append(cls != 0)
        pp_msg_ok.append(cls <= 0)
        checks += [("preprepare", len(pps) - 1, r) for r in (1, 2, 3)]
        senders = [(x, 0) for x in (1, 2, 3)] + [(x, 1) for x in range(4)]  # prepares, then commits
        for sender, mtype in senders:
            j = len(votes)
            cls = bad_v.get(j, -1)
            view_v, seq_v, d_v = tamper(VIEW, seq, d, cls, i) if cls > 0 else (VIEW, seq, d)
            v = (view_v, seq_v, d_v, NODES[sender], mtype)
            votes.append(v)
            sg = s.sign(hashlib.sha256(gj.gojson_vote(*v)).digest(), sender)
            vote_sig.append(flip(sg) if cls == 0 else sg)
            vote_state.append(i)
            vote_sig_ok.append(cls != 0)
            vote_msg_ok.append(cls <= 0)
            checks += [("vote", j, r) for r in range(4) if r != sender]
        for sender in range(4):                        # replies to the client
            j = len(replies)
            rp = (VIEW, req[0], req[1], NODES[sender], b"Executed")
            replies.append(rp)
            sg = s.sign(hashlib.sha256(gj.gojson_reply(*rp)).digest(), sender)
            reply_sig.append(flip(sg) if j in bad_rep else sg)
            reply_ok.append(j not in bad_rep)
            checks.append(("reply", j, 4))
    pub = s.pub.copy()
    s.close()

    def rows(sigs):
        return np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 64)
    s_last = np.array([-1] + assigned[:-1], np.int64)
    return {"pub": pub, "requests": sent, "request_sigs": rows(req_sig), "assigned_seqs": np.array(assigned, np.int64),
            "preprepares": pps, "preprepare_sigs": rows(pp_sig), "votes": votes, "vote_sigs": rows(vote_sig),
            "replies": replies, "reply_sigs": rows(reply_sig), "checks": checks,
            "state_view": np.full(n_req, VIEW, np.int64), "state_last": s_last,
            "preprepare_state": np.array(pp_state, np.uint32), "vote_state": np.array(vote_state, np.uint32),
            "request_sig_ok": np.array(req_ok), "preprepare_sig_ok": np.array(pp_sig_ok),
            "preprepare_msg_ok": np.array(pp_msg_ok), "vote_sig_ok": np.array(vote_sig_ok),
            "vote_msg_ok": np.array(vote_msg_ok), "reply_sig_ok": np.array(reply_ok),
            "preprepare_class": bad_pp, "vote_class": bad_v}


def corrupt_certs(H, S, K, per_cert: int, n_keys: int, frac_one: float = 0.01, frac_two: float = 0.005,
                  seed: int = 0x50424654):
    """Configs 2/3 with Byzantine votes: a seeded `frac_one` of the certificates
    carry one bad vote and `frac_two` carry two, the votes corrupted over
    CLASSES in turn (in place).  Returns (expected accept mask, certificates
    with >= 1 bad vote, certificates with >= 2).  With n = 3f + 1 a QC of 2f + 1
    votes fails at one bad vote; the reference's 2f count
    (pbft_impl.go:212,227) fails only at two."""
    n_certs = len(K) // per_cert
    rng = np.random.default_rng(seed ^ 0xCE27)
    m1, m2 = int(round(n_certs * frac_one)), int(round(n_certs * frac_two))
    chosen = rng.choice(n_certs, m1 + m2, replace=False)
    one, two = np.sort(chosen[:m1]), np.sort(chosen[m1:])
    ok = np.ones(len(K), bool)
    t = 0
    for c, nbad in [(c, 1) for c in one] + [(c, 2) for c in two]:
        for v in rng.choice(per_cert, nbad, replace=False):
            i = int(c) * per_cert + int(v)
            corrupt_one(H, S, K, i, t % 8, n_keys, rng)
            ok[i] = False
            t += 1
    return ok, np.sort(chosen), two


def certs(n_keys: int, per_cert: int, n_certs: int, seed: int):
    """n_certs quorum certificates of per_cert votes over one digest each, from
    distinct replicas of an n_keys committee (configs 2 and 3, and the QC
    latency's one-certificate calls): every signature distinct."""
    s = Signer(n_keys, seed)
    rng = np.random.default_rng(seed)
    m = n_certs * per_cert
    H = np.repeat(np.frombuffer(rng.bytes(32 * n_certs), np.uint8).reshape(n_certs, 32), per_cert, axis=0)
    K = np.concatenate([rng.choice(n_keys, per_cert, replace=False) for _ in range(n_certs)]).astype(np.uint32)
    S = np.zeros((m, 64), np.uint8)
    B = _batch_signer() if m >= 4096 else None
    if B is not None:
        rc = B.synth_sign_batch(s.priv.ctypes.data, n_keys, H.ctypes.data, K.ctypes.data, m, S.ctypes.data,
                                max(1, min(16, os.cpu_count() or 1)))
        if rc != 0:
            raise RuntimeError(f"synth_sign_batch failed: {rc}")
    else:
        for i in range(m):
            S[i] = np.frombuffer(s.sign(H[i].tobytes(), int(K[i])), np.uint8)
    pub = s.pub.copy()
    s.close()
    return pub, H, S, K


def sys_path_fix():
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
