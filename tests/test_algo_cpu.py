"""The GPU kernels' arithmetic, compiled for the CPU (tests/cpp/algo_harness.cpp),
checked against Python big integers and the oracle: limb bounds of every
field operation (the invariants fe29.h documents), and the full verify
pipeline (scalars -> comb tables -> final complete addition) on every golden
vector.  This is test infrastructure: the product runs this code only on the GPU."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import crafted_exceptional, ROOT, fixture_arrays, oracle_sign_pool

P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
R = 1 << 261
M29 = (1 << 29) - 1
TABLE_WORDS = 33 * 128 * 16
M_BOUND = int(1.172 * 2 ** 256)
L_BOUND = int(2.344 * 2 ** 256)


@pytest.fixture(scope="module")
def H():
    d = os.path.join(ROOT, "tests", "cpp")
    so = os.path.join(d, "libalgo_harness.so")
    src = os.path.join(d, "algo_harness.cpp")
    hdrs = [os.path.join(ROOT, "simple_pbft_amd", "csrc", f) for f in ("fe29.h", "fes.h", "p256_algo.h", "p256_consts.h")]
    if not os.path.exists(so) or any(os.path.getmtime(h) > os.path.getmtime(so) for h in hdrs + [src]):
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", so, src], check=True)
    return ctypes.CDLL(so)


def limbs(v):
    return (ctypes.c_uint32 * 9)(*[(v >> (29 * i)) & M29 for i in range(9)])


def val(l):
    return sum(int(x) << (29 * i) for i, x in enumerate(l))


def rand_l_type(rng):
    """A lazily-added (L-type) input: limbs < 2^30, value < 2.344 * 2^256."""
    while True:
        l = [int(rng.choice([rng.integers(0, 1 << 30), (1 << 30) - 1, 0, 1 << 29])) for _ in range(9)]
        l[8] = int(rng.integers(0, 1 << 26))
        if val(l) < L_BOUND:
            return (ctypes.c_uint32 * 9)(*l), val(l)


def test_fe_mul_sqr_sub_bounds(H):
    rng = np.random.default_rng(1)
    out = (ctypes.c_uint32 * 9)()
    edge = [0, 1, P - 1, P, P + 1, 2 ** 256 - 1, M_BOUND - 1]
    for it in range(4000):
        if it < len(edge) ** 2:
            a, b = edge[it // len(edge)], edge[it % len(edge)]
            la, lb = limbs(a), limbs(b)
        elif it % 2:
            a, b = int(rng.integers(0, 2 ** 62)) ** 4 % P, int(rng.integers(0, 2 ** 62)) ** 4 % P
            la, lb = limbs(a), limbs(b)
        else:
            (la, a), (lb, b) = rand_l_type(rng), rand_l_type(rng)
        H.h_fe_mul(la, lb, out)
        v = val(out)
        assert v % P == a * b * pow(R, -1, P) % P
        assert all(x < (1 << 29) for x in out) and v < M_BOUND
        H.h_fe_sqr(la, out)
        v = val(out)
        assert v % P == a * a * pow(R, -1, P) % P and all(x < (1 << 29) for x in out) and v < M_BOUND
        H.h_fe_sub(la, lb, out)
        v = val(out)
        assert v % P == (a - b) % P and all(x < (1 << 29) for x in out) and v < 2 ** 256 + 2 ** 237
        H.h_fe_canon(limbs(a % M_BOUND), out)
        assert val(out) == (a % M_BOUND) % P


def test_fe_mul_small_and_words(H):
    rng = np.random.default_rng(2)
    out = (ctypes.c_uint32 * 9)()
    w = (ctypes.c_uint32 * 8)()
    for _ in range(500):
        a = int.from_bytes(rng.bytes(32), "big") % M_BOUND
        for k in (1, 2, 3):
            H.h_fe_mul_small(limbs(a), k, out)
            assert val(out) % P == k * a % P and val(out) < 2 ** 256 + 2 ** 237
            assert all(x < (1 << 29) for x in out)
        b = a % (2 ** 256)
        H.h_fe_to_words(limbs(b), w)
        assert sum(int(x) << (32 * i) for i, x in enumerate(w)) == b
        H.h_fe_from_words(w, out)
        assert val(out) == b


def test_fn_mul_and_scalars(H):
    rng = np.random.default_rng(3)
    out = (ctypes.c_uint32 * 9)()
    for _ in range(2000):
        a = int.from_bytes(rng.bytes(32), "big")
        b = int.from_bytes(rng.bytes(32), "big")
        H.h_fn_mul(limbs(a), limbs(b), out)
        assert val(out) % N == a * b * pow(R, -1, N) % N and val(out) < 2 * N
    W = ctypes.c_uint32 * 8
    for _ in range(50):
        e, r, s = (int.from_bytes(rng.bytes(32), "big") for _ in range(3))
        r, s = r % N or 1, s % N or 1
        u1, u2 = W(), W()
        ok = H.h_scalars(W(*[(e >> 32 * i) & 0xFFFFFFFF for i in range(8)]),
                         W(*[(r >> 32 * i) & 0xFFFFFFFF for i in range(8)]),
                         W(*[(s >> 32 * i) & 0xFFFFFFFF for i in range(8)]), u1, u2)
        assert ok
        w = pow(s, -1, N)
        assert sum(int(x) << 32 * i for i, x in enumerate(u1)) == e * w % N
        assert sum(int(x) << 32 * i for i, x in enumerate(u2)) == r * w % N


def _tables(H, keys):
    g = (ctypes.c_uint32 * TABLE_WORDS)()
    H.h_build_g_table(g)
    tabs, valid = [], []
    for k in keys:
        t = (ctypes.c_uint32 * TABLE_WORDS)()
        valid.append(H.h_build_table(k.tobytes(), t))
        tabs.append(t)
    return g, tabs, valid


def test_pipeline_on_golden_vectors(H, ecdsa_fixtures):
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    g, tabs, valid = _tables(H, keys)
    assert [bool(v) for v in valid] == [k["valid"] for k in ecdsa_fixtures["keys"]]
    for i in range(len(kidx)):
        k = int(kidx[i])
        got = H.h_verify(hashes[i].tobytes(), sigs[i].tobytes(), g, tabs[k], valid[k]) if k < len(tabs) else 0
        assert bool(got) == expect[i], ecdsa_fixtures["vectors"][i]["kind"]


def test_pipeline_random_vs_oracle(H, oracle_lib):
    keys, hashes, sigs, kidx = oracle_sign_pool(oracle_lib, n_keys=4, per_key=40, seed=5)
    rng = np.random.default_rng(6)
    n = len(kidx)
    flip = rng.random(n) < 0.4
    sigs[flip, 50] ^= 0x10
    g, tabs, valid = _tables(H, keys)
    bm = np.zeros((n + 7) // 8, np.uint8)
    oracle_lib.oracle_ecdsa_p256_verify_batch(hashes.ctypes.data, sigs.ctypes.data, kidx.ctypes.data, n,
                                              keys.ctypes.data, len(keys), bm.ctypes.data, 4)
    want = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    for i in range(n):
        got = H.h_verify(hashes[i].tobytes(), sigs[i].tobytes(), g, tabs[kidx[i]], valid[kidx[i]])
        assert bool(got) == want[i]
    assert (want == ~flip).all()


def test_comb_fast_and_checked_paths_agree(H):
    """The unchecked comb (deferred Z == 0 test) and the complete-addition comb
    give the same point; and scalars whose comb would need a doubling are
    handled (u = 0, tiny u, u = n - 1)."""
    g = (ctypes.c_uint32 * TABLE_WORDS)()
    H.h_build_g_table(g)
    W = ctypes.c_uint32 * 8
    out_a, out_b = (ctypes.c_uint32 * 16)(), (ctypes.c_uint32 * 16)()
    rng = np.random.default_rng(12)
    cases = [0, 1, 2, 127, 128, 129, 255, 256, N - 1, N - 2, 2 ** 255, 2 ** 256 - 2 ** 224] + \
        [int.from_bytes(rng.bytes(32), "big") % N for _ in range(40)]
    from oracle import p256
    for u in cases:
        uw = W(*[(u >> 32 * i) & 0xFFFFFFFF for i in range(8)])
        ra = H.h_comb(uw, g, 0, out_a)
        rb = H.h_comb(uw, g, 1, out_b)
        assert ra == rb
        want = p256.scalar_mult(u % N, p256.G)
        assert bool(ra) == (want is not None)
        if ra:
            assert list(out_a) == list(out_b)
            x = sum(int(v) << 32 * i for i, v in enumerate(out_a[:8]))
            y = sum(int(v) << 32 * i for i, v in enumerate(out_a[8:]))
            assert (x, y) == want


def test_pipeline_crafted_exceptional_sums(H):
    """Chosen-(u1, u2) signatures under Q = G whose comb sums hit doublings and
    cancellations (tests/conftest.py crafted_exceptional) on the 8-bit tables."""
    key, hashes, sigs, kidx, expect = crafted_exceptional()
    g, tabs, valid = _tables(H, key)
    assert valid == [1]
    for i in range(len(kidx)):
        got = H.h_verify(hashes[i].tobytes(), sigs[i].tobytes(), g, tabs[0], 1)
        assert bool(got) == expect[i], i


def test_pipeline_mixed_window_geometry(H, ecdsa_fixtures):
    """A mixed comb geometry (p256_algo.h CombGeom code 11: 15 windows of 12
    bits + 7 top windows of 11 bits = 257, the scheme of the device's 21 and 29
    codes) -- recoding, per-window offsets and the half-size top windows --
    on the golden vectors and the crafted doubling/cancellation sums."""
    words = (15 * 2048 + 7 * 1024) * 16
    g = (ctypes.c_uint32 * words)()
    assert H.h_build_table_w(None, 11, g) == 1
    keys, hashes, sigs, kidx, expect = fixture_arrays(ecdsa_fixtures)
    tabs, valid = {}, {}
    for k in sorted(set(int(x) for x in kidx if x < len(keys))):
        t = (ctypes.c_uint32 * words)()
        valid[k] = H.h_build_table_w(keys[k].tobytes(), 11, t)
        tabs[k] = t
    for i in range(len(kidx)):
        k = int(kidx[i])
        got = H.h_verify_w(11, hashes[i].tobytes(), sigs[i].tobytes(), g, tabs[k], valid[k]) if k in tabs else 0
        assert got in (0, 1)
        assert bool(got) == expect[i], ecdsa_fixtures["vectors"][i]["kind"]
    key, hashes, sigs, kidx, expect = crafted_exceptional()
    for i in range(len(kidx)):  # Q = G: the G table serves as the key table
        assert bool(H.h_verify_w(11, hashes[i].tobytes(), sigs[i].tobytes(), g, g, 1)) == expect[i], i


# ---- safegcd inversion mod n (simple_pbft_amd/csrc/safegcd.h) ----------------
def _w8(v):
    return (ctypes.c_uint32 * 8)(*[(v >> 32 * i) & 0xFFFFFFFF for i in range(8)])


def test_safegcd_inverse_mod_n(H):
    rng = np.random.default_rng(0x5AFE)
    xs = [1, 2, 3, N - 1, N - 2, (N - 1) // 2, 1 << 255, (1 << 256) % N, (1 << 128) - 1, 0xFFFFFFFF,
          N >> 1, (N + 1) // 2, 3 ** 150 % N]
    xs += [int.from_bytes(rng.bytes(32), "big") % N or 1 for _ in range(3000)]
    xs += [1 << k for k in range(256)]
    xs += [(1 << k) - 1 for k in range(1, 256)]
    out = (ctypes.c_uint32 * 8)()
    for x in xs:
        for inv in (H.h_inv_n_words, H.h_inv_n_words_ct):  # variable-time and constant-time divsteps
            inv(_w8(x), out)
            got = sum(int(v) << 32 * i for i, v in enumerate(out))
            assert got == pow(x, -1, N), hex(x)


def test_safegcd_matches_fermat_montgomery(H):
    rng = np.random.default_rng(7)
    R = 1 << 261
    H.h_fn_inv_mont.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    for _ in range(300):
        x = int.from_bytes(rng.bytes(32), "big") % N or 5
        xm = x * R % N
        a, b = (ctypes.c_uint32 * 9)(), (ctypes.c_uint32 * 9)()
        H.h_fn_inv_mont(limbs(xm), 1, a)
        H.h_fn_inv_mont(limbs(xm), 0, b)
        want = pow(x, -1, N) * R % N
        assert val(a) % N == want and val(b) % N == want


# ---- XYZZ mixed addition (p256_algo.h xyzz_madd, the throughput comb's step) ---
def test_xyzz_madd_chain_values_and_bounds(H):
    """A chain of 60 madd-2008-s additions from a random XYZZ start: every
    intermediate (X/ZZ, Y/ZZZ) equals the big-integer sum, limbs stay within
    the fe29.h invariants (X, Y: N-type from fe_sub; ZZ, ZZZ: M-type), and
    adding the accumulator's own point or its negative gives ZZ == ZZZ == 0."""
    from oracle import p256
    rng = np.random.default_rng(7)
    A = ctypes.c_uint32 * 36
    Pt = ctypes.c_uint32 * 18

    def mont(v):
        return v * R % P

    def unmont(v):
        return v * pow(R, -1, P) % P

    def to_acc(pt, z):
        x, y = pt
        vals = [mont(x * z * z % P), mont(y * z * z * z % P), mont(z * z % P), mont(z * z * z % P)]
        return A(*[w for v in vals for w in limbs(v)])

    def from_acc(acc):
        x, y, zz, zzz = (unmont(val(acc[9 * k:9 * k + 9]) % P) for k in range(4))
        assert zz != 0 and zzz != 0
        return x * pow(zz, -1, P) % P, y * pow(zzz, -1, P) % P

    cur = p256.scalar_mult(int(rng.integers(1, 2 ** 62)), p256.G)
    acc = to_acc(cur, int(rng.integers(2, 2 ** 62)))
    # 2p in the borrow form of fe_neg_lazy (p256_consts.h kP2Borrow)
    p2b = [0x3ffffffe, 0x3ffffffe, 0x3ffffffe, 0x200003fe, 0x1fffffff, 0x1fffffff, 0x2007ffff, 0x3fbfffff, 0x01fffffe]
    assert val(p2b) == 2 * P
    for step in range(60):
        q = p256.scalar_mult(int(rng.integers(1, 2 ** 62)), p256.G)
        if step % 2:  # a negative comb digit: y2 = 2p - y lazily, limbs < 2^30 (k_ecdsa_comb fe_cneg_lazy)
            ly = [b - a for a, b in zip(limbs(mont(q[1])), p2b)]
            H.h_xyzz_madd(acc, Pt(*limbs(mont(q[0])), *ly))
            q = (q[0], (P - q[1]) % P)
        else:
            H.h_xyzz_madd(acc, Pt(*limbs(mont(q[0])), *limbs(mont(q[1]))))
        cur = p256.point_add(cur, q)
        assert from_acc(acc) == cur, step
        for k in range(4):
            l = acc[9 * k:9 * k + 9]
            assert all(x < (1 << 29) for x in l), (step, k)
            assert val(l) < (2 ** 256 + 2 ** 237 if k == 0 else M_BOUND), (step, k)
    for neg in (False, True):
        x, y = from_acc(acc)
        y = (P - y) % P if neg else y
        a2 = A(*acc)
        H.h_xyzz_madd(a2, Pt(*limbs(mont(x)), *limbs(mont(y))))
        assert val(a2[18:27]) % P == 0 and val(a2[27:36]) % P == 0


# ---- signed-limb arithmetic (simple_pbft_amd/csrc/fes.h, the comb's hot loop) ----
S_BOUND = int(2 ** 257.5)
D_BOUND = int(2 ** 258.5)


def slimbs(l):
    return (ctypes.c_uint32 * 9)(*[x & 0xFFFFFFFF for x in l])


def sval(l):
    """value of signed 32-bit limbs"""
    return sum((int(x) - (1 << 32) if int(x) & 0x80000000 else int(x)) << (29 * i) for i, x in enumerate(l))


def s_limbs_of(v):
    """S-type limbs of a (possibly negative) value: limbs 0..7 in [0, 2^29), limb 8 the signed rest"""
    l = [(v >> (29 * i)) & M29 for i in range(8)]
    l.append(v >> 232)
    return l


def rand_s(rng, extreme=False):
    if extreme:
        v = int(rng.choice([S_BOUND - 1, -S_BOUND + 1, 0, P - 1, -(P - 1)]))
        l = s_limbs_of(v)
        if v > 0:
            l[:8] = [M29] * 8 if rng.integers(0, 2) else l[:8]
    else:
        v = int.from_bytes(rng.bytes(33), "big") % (2 * S_BOUND) - S_BOUND
        l = s_limbs_of(v)
    while abs(sum(x << (29 * i) for i, x in enumerate(l))) >= S_BOUND:
        l[8] -= 1 if l[8] > 0 else -1
    return l, sum(x << (29 * i) for i, x in enumerate(l))


def rand_d(rng, extreme=False):
    a, va = rand_s(rng, extreme)
    b, vb = rand_s(rng, extreme)
    d = [x - y for x, y in zip(a, b)]
    return d, va - vb


def check_s(out):
    v = sval(out)
    assert all(0 <= int(x) < (1 << 29) for x in out[:8]), list(out)
    assert abs(v) < S_BOUND, v
    return v


def test_fs_mul_sqr_types_and_values(H):
    """fs_mul / fs_sqr / fs_mul2_add on S- and D-type inputs, random and at the
    type bounds: Montgomery product mod p, S-type output, and the output lies
    in (T / 2^261, T / 2^261 + 1.0001 p) (the 29-bit top digit)."""
    rng = np.random.default_rng(0x5161)
    out = (ctypes.c_uint32 * 9)()
    Rinv = pow(R, -1, P)
    for it in range(3000):
        ext = it % 5 == 0
        kinds = [(rand_s, rand_s), (rand_s, rand_d), (rand_d, rand_d)][it % 3]
        (la, a), (lb, b) = kinds[0](rng, ext), kinds[1](rng, ext)
        assert all(abs(x) < (1 << 29) for x in la[:8] + lb[:8])
        H.h_fs_mul(slimbs(la), slimbs(lb), out)
        v = check_s(out)
        assert v % P == a * b * Rinv % P
        assert a * b - R < v * R < a * b + 10001 * P * R // 10000  # exact integers (a float T / R rounds)
        H.h_fs_sqr(slimbs(lb), out)
        v = check_s(out)
        assert v % P == b * b * Rinv % P
        (lc, c), (ld, d) = rand_d(rng, ext), rand_s(rng, ext)
        H.h_fs_mul2_add(slimbs(la), slimbs(lb), slimbs(lc), slimbs(ld), out)
        v = check_s(out)
        assert v % P == (a * b + c * d) * Rinv % P
        # X3 = R^2 - PPP - 2Q folded into the squaring's columns (fs_sqr_sub2):
        # the same limbs as fs_sqr, the limb-wise combination and fs_norm
        (le, e_), (lf, f_) = rand_s(rng, ext), rand_s(rng, ext)
        H.h_fs_sqr_sub2(slimbs(lb), slimbs(le), slimbs(lf), out)
        got = list(out)
        H.h_fs_sqr(slimbs(lb), out)
        comb = [(int(out[i]) - (le[i] & 0xFFFFFFFF) - 2 * (lf[i] & 0xFFFFFFFF)) & 0xFFFFFFFF for i in range(9)]
        H.h_fs_norm((ctypes.c_uint32 * 9)(*comb), out)
        assert got == list(out)
        assert sval(got) % P == (b * b * Rinv - e_ - 2 * f_) % P
        H.h_fs_canon(slimbs(lc), out)
        assert val(out) == c % P
        x = [int(y) for y in rng.integers(-(1 << 30), 1 << 30, 9)]
        H.h_fs_norm(slimbs(x), out)
        assert sval(out) == sum(y << (29 * i) for i, y in enumerate(x))
        assert all(0 <= int(y) < (1 << 29) for y in out[:8])


def test_xyzz_madd_s_chain_values_and_bounds(H):
    """A chain of 200 signed-limb madd-2008-s additions (the comb's step,
    negative digits as negated y): every intermediate equals the big-integer
    sum, every accumulator coordinate stays S-type, and adding the
    accumulator's own point or its negative leaves ZZ == ZZZ == 0."""
    from oracle import p256
    rng = np.random.default_rng(71)
    A = ctypes.c_uint32 * 36
    Pt = ctypes.c_uint32 * 18

    def mont(v):
        return v * R % P

    def unmont(v):
        return v * pow(R, -1, P) % P

    def from_acc(acc):
        x, y, zz, zzz = (unmont(sval(acc[9 * k:9 * k + 9]) % P) for k in range(4))
        assert zz != 0 and zzz != 0
        return x * pow(zz, -1, P) % P, y * pow(zzz, -1, P) % P

    cur = p256.scalar_mult(int(rng.integers(1, 2 ** 62)), p256.G)
    z = int(rng.integers(2, 2 ** 62))
    acc = A(*[w for v in (mont(cur[0] * z * z % P), mont(cur[1] * z ** 3 % P), mont(z * z % P), mont(z ** 3 % P))
              for w in limbs(v)])
    for step in range(200):
        q = p256.scalar_mult(int(rng.integers(1, 2 ** 62)), p256.G)
        neg = step % 2 == 1
        ly = [(-x) & 0xFFFFFFFF if neg else x for x in limbs(mont(q[1]))]
        H.h_xyzz_madd_s(acc, Pt(*limbs(mont(q[0])), *ly))
        if neg:
            q = (q[0], (P - q[1]) % P)
        cur = p256.point_add(cur, q)
        assert from_acc(acc) == cur, step
        for k in range(4):
            check_s(acc[9 * k:9 * k + 9])
    for neg in (False, True):
        x, y = from_acc(acc)
        y = (P - y) % P if neg else y
        a2 = A(*acc)
        H.h_xyzz_madd_s(a2, Pt(*limbs(mont(x)), *limbs(mont(y))))
        assert sval(a2[18:27]) % P == 0 and sval(a2[27:36]) % P == 0


def test_xyzz_madd_s_flip_chain(H):
    """The comb's sign-alternating step (xyzz_madd_s_flip, verify_kernels.h
    k_ecdsa_comb): the accumulator holds W = sigma Y, the point is passed as
    sigma (+-y), sigma flips after every addition.  200 steps with random
    digit signs: sigma W equals the big-integer sum's Y at every step, X / ZZ /
    ZZZ equal it outright, every coordinate stays S-type, and an addition that
    meets the point (or its negative) leaves ZZ == ZZZ == 0."""
    from oracle import p256
    rng = np.random.default_rng(72)
    A = ctypes.c_uint32 * 36
    Pt = ctypes.c_uint32 * 18

    def mont(v):
        return v * R % P

    def unmont(v):
        return v * pow(R, -1, P) % P

    def from_acc(acc, sigma):
        x, w, zz, zzz = (unmont(sval(acc[9 * k:9 * k + 9]) % P) for k in range(4))
        assert zz != 0 and zzz != 0
        return x * pow(zz, -1, P) % P, sigma * w * pow(zzz, -1, P) % P

    cur = p256.scalar_mult(int(rng.integers(1, 2 ** 62)), p256.G)
    acc = A(*[w for v in (mont(cur[0]), mont(cur[1]), mont(1), mont(1)) for w in limbs(v)])
    sigma = 1
    for step in range(200):
        q = p256.scalar_mult(int(rng.integers(1, 2 ** 62)), p256.G)
        neg = bool(rng.integers(0, 2))
        flip = neg != (sigma == -1)  # the kernel's (dc < 0) != neg_y
        ly = [(-x) & 0xFFFFFFFF if flip else x for x in limbs(mont(q[1]))]
        H.h_xyzz_madd_s_flip(acc, Pt(*limbs(mont(q[0])), *ly))
        sigma = -sigma
        if neg:
            q = (q[0], (P - q[1]) % P)
        cur = p256.point_add(cur, q)
        assert from_acc(acc, sigma) == cur, step
        for k in range(4):
            check_s(acc[9 * k:9 * k + 9])
    for neg in (False, True):
        x, y = from_acc(acc, sigma)
        y = (P - y) % P if neg else y
        ys = (P - y) % P if sigma == -1 else y
        a2 = A(*acc)
        H.h_xyzz_madd_s_flip(a2, Pt(*limbs(mont(x)), *limbs(mont(ys))))
        assert sval(a2[18:27]) % P == 0 and sval(a2[27:36]) % P == 0


def test_fs_sqr_mul_add_types_and_values(H):
    """fs_sqr_mul_add (the fused last step's R^2 + PP W under one reduction):
    a D-type, b and c S-type, random and at the type bounds: the Montgomery
    value, S-type output."""
    rng = np.random.default_rng(0x5A11)
    out = (ctypes.c_uint32 * 9)()
    Rinv = pow(R, -1, P)
    for it in range(3000):
        ext = it % 4 == 0
        (la, a), (lb, b), (lc, c) = rand_d(rng, ext), rand_s(rng, ext), rand_s(rng, ext)
        H.h_fs_sqr_mul_add(slimbs(la), slimbs(lb), slimbs(lc), out)
        v = check_s(out)
        assert v % P == (a * a + b * c) * Rinv % P
    # the fused step's multiplicand: fs_norm of -(U2 + X1 + rz), limbs in (-3 2^29, 0]
    for _ in range(500):
        parts = [rand_s(rng, bool(rng.integers(0, 2))) for _ in range(3)]
        w = [-(parts[0][0][i] + parts[1][0][i] + parts[2][0][i]) for i in range(9)]
        H.h_fs_norm(slimbs(w), out)
        assert sval(out) == -(parts[0][1] + parts[1][1] + parts[2][1])
        assert all(0 <= int(x) < (1 << 29) for x in out[:8]) and abs(sval(out[8:9])) < (1 << 28)


def test_fs_is_zero_fold_range(H):
    """fes.h fs_is_zero: fe_fold_carry of an S- or D-type value lies strictly
    inside (0, 2p), so the value is 0 mod p iff the folded digits are p's.
    Random and type-bound values, every multiple k p (|k| <= 5) written as an
    S-type value and as D-type differences of two S-type values."""
    rng = np.random.default_rng(0x2E40)
    out = (ctypes.c_uint32 * 9)()

    def check(l, v):
        H.h_fs_fold(slimbs(l), out)
        f = val(out)
        assert all(0 <= int(x) < (1 << 29) for x in out[:8])
        assert 0 < f < 2 * P and f % P == v % P, (l, v)
        assert H.h_fs_is_zero(slimbs(l)) == (1 if v % P == 0 else 0)

    for it in range(4000):
        (l, v) = (rand_s if it % 2 else rand_d)(rng, it % 3 == 0)
        check(l, v)
    for k in range(-5, 6):
        v = k * P
        if abs(v) < S_BOUND:
            check(s_limbs_of(v), v)
        for _ in range(50):
            a, va = rand_s(rng, False)
            wb = va - v  # b = a - k p: a - b = k p as limb-wise difference
            if abs(wb) >= S_BOUND:
                continue
            b = s_limbs_of(wb)
            check([x - y for x, y in zip(a, b)], v)
            check([x - y for x, y in zip(a, b)][:8] + [a[8] - b[8] + 1], v + (1 << 232))  # one off


def _mont(v):
    return v * R % P


def _unmont(v):
    return v * pow(R, -1, P) % P


def test_xyzz_aff_aff_s_first_pair(H):
    """The comb's first step (fes.h xyzz_aff_aff_s): the affine sum of the first
    two table points, for every sign pair; W carries sigma = -s1; equal or
    opposite points leave ZZ = ZZZ = 0."""
    from oracle import p256
    rng = np.random.default_rng(73)
    acc = (ctypes.c_uint32 * 36)()
    for it in range(300):
        a = p256.scalar_mult(int(rng.integers(1, 2 ** 62)), p256.G)
        b = p256.scalar_mult(int(rng.integers(1, 2 ** 62)), p256.G)
        s0, s1 = int(rng.choice([-1, 1])), int(rng.choice([-1, 1]))
        pts = (ctypes.c_uint32 * 36)(*limbs(_mont(a[0])), *limbs(_mont(a[1])), *limbs(_mont(b[0])), *limbs(_mont(b[1])))
        H.h_xyzz_aff_aff_s(pts, int(s0 != s1), acc)
        for k in range(4):
            check_s(acc[9 * k:9 * k + 9])
        x, w, zz, zzz = (_unmont(sval(acc[9 * k:9 * k + 9]) % P) for k in range(4))
        want = p256.point_add((a[0], a[1] if s0 > 0 else P - a[1]), (b[0], b[1] if s1 > 0 else P - b[1]))
        assert (x * pow(zz, -1, P) % P, -s1 * w * pow(zzz, -1, P) % P) == want, it
    a = p256.scalar_mult(12345, p256.G)
    for s0, s1 in ((1, 1), (1, -1)):  # the same point twice: doubling (or its negative: infinity)
        pts = (ctypes.c_uint32 * 36)(*limbs(_mont(a[0])), *limbs(_mont(a[1])), *limbs(_mont(a[0])), *limbs(_mont(a[1])))
        H.h_xyzz_aff_aff_s(pts, int(s0 != s1), acc)
        assert sval(acc[18:27]) % P == 0 and sval(acc[27:36]) % P == 0


def _w11_digits(u):
    """signed recoding of the mixed W = 11 code (15 x 12 + 7 x 11 bits)"""
    out, c = [], 0
    for i in range(22):
        wd, bit = (12, 12 * i) if i < 15 else (11, 180 + 11 * (i - 15))
        d = ((u >> bit) & ((1 << wd) - 1)) + c
        c = 1 if d > (1 << (wd - 1)) else 0
        out.append((d - (c << wd), bit))
    return out


def test_comb_schedule_first_pair_fused_last_rerun(H):
    """p256_algo.h comb2_verify -- k_ecdsa_comb's schedule: first pair added
    affine + affine, last addition fused with the x check, complete-addition
    rerun -- on chosen (u1, u2, r) with Q = G on the mixed W = 11 tables:
      * random scalars, r = R.x mod n (accept) and r off by one (reject): path
        first pair + fused;
      * a zero first digit (then the generic steps throughout) and a zero
        last digit (the plain check): same bits;
      * the last point equal to the sum before it (doubling) or its negative
        (cancellation): the fused step reports it, the rerun decides;
      * r + n < p: the second candidate of the fused check."""
    from oracle import p256
    words = (15 * 2048 + 7 * 1024) * 16
    g = (ctypes.c_uint32 * words)()
    assert H.h_build_table_w(None, 11, g) == 1
    W = ctypes.c_uint32 * 8
    path = ctypes.c_int()

    def w8(v):
        return W(*[(v >> 32 * i) & 0xFFFFFFFF for i in range(8)])

    def run(u1, u2, r):
        ok = H.h_comb_verify_u(11, w8(u1), w8(u2), w8(r), g, g, ctypes.byref(path))
        assert ok in (0, 1)
        return bool(ok), path.value

    def rx(u):
        pt = p256.scalar_mult(u % N, p256.G)
        return None if pt is None else pt[0] % N

    rng = np.random.default_rng(74)
    for _ in range(40):
        u1, u2 = (int.from_bytes(rng.bytes(32), "big") % N for _ in range(2))
        r = rx(u1 + u2)
        assert run(u1, u2, r) == (True, 3)
        assert run(u1, u2, (r + 1) % N or 1) == (False, 3)
    # zero digits at the ends: u1 with a zero lowest window, u2 with a zero top window
    u1 = (int.from_bytes(rng.bytes(32), "big") % N) & ~0xFFF
    u2 = int.from_bytes(rng.bytes(32), "big") % N
    assert _w11_digits(u1)[0][0] == 0
    assert run(u1, u2, rx(u1 + u2)) == (True, 0)  # no first pair: no fused step either (the kernel's rule)
    u2s = int.from_bytes(rng.bytes(28), "big")
    assert _w11_digits(u2s)[-1][0] == 0
    assert run(u1 | 1, u2s, rx((u1 | 1) + u2s)) == (True, 1)
    # the last point meets the sum before it: u1 + u2 - d 2^b = +-d 2^b
    hits = 0
    for _ in range(40):
        u2 = int.from_bytes(rng.bytes(32), "big") % N
        d, b = _w11_digits(u2)[-1]
        if d == 0:
            continue
        hits += 1
        t = d * (1 << b)
        u1 = (2 * t - u2) % N  # sum R = 2T: a doubling at the last step
        r = rx(u1 + u2)
        ok, pth = run(u1, u2, r)
        assert ok and pth & 4, pth
        ok, pth = run(u1, u2, (r + 1) % N)
        assert not ok and pth & 4
        u1 = (-u2) % N  # R = infinity: a cancellation at the last step
        ok, pth = run(u1, u2, 1)
        assert not ok and pth & 4
    assert hits > 30
    # r + n < p: a sum whose x lies in [n, p) is accepted for r = x - n, by
    # the fused check's second candidate.  No scalar reaches such a point in a
    # test's time (2^-128), so the step runs on a chosen accumulator A = S - T
    # (random Z) and entry T, for a point S with x in [n, p).
    B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
    acc = (ctypes.c_uint32 * 36)()
    ew = (ctypes.c_uint32 * 16)()
    tried = 0
    for xs in range(N + 1, N + 2000):
        rhs = (xs ** 3 - 3 * xs + B) % P
        ys = pow(rhs, (P + 1) // 4, P)
        if ys * ys % P != rhs:
            continue
        tried += 1
        t = p256.scalar_mult(int(rng.integers(1, 2 ** 62)), p256.G)
        a = p256.point_add((xs, ys), (t[0], (P - t[1]) % P))
        z = int(rng.integers(2, 2 ** 62))
        for k, v in enumerate((a[0] * z * z, a[1] * z ** 3, z * z, z ** 3)):
            acc[9 * k:9 * k + 9] = list(limbs(_mont(v % P)))
        ew[:8] = [(_mont(t[0]) >> 32 * i) & 0xFFFFFFFF for i in range(8)]
        ew[8:] = [(_mont(t[1]) >> 32 * i) & 0xFFFFFFFF for i in range(8)]
        assert H.h_comb_last_check_s(acc, 0, 1, ew, w8(xs - N)) == 1
        assert H.h_comb_last_check_s(acc, 0, 1, ew, w8(xs - N + 1)) == 0
        assert H.h_comb_last_check_s(acc, 0, -1, ew, w8(xs - N)) == 0  # the entry negated: another sum
        if tried == 5:
            break
    assert tried == 5


# ---- lane-parallel safegcd of the latency path (verify_kernels.h inv_mod_n_wave) ----
# A restatement of the kernel's scheme with exact integers: one list entry per
# lane-limb, 30-bit signed limbs re-centered after every batch, divsteps on the
# low limbs only, centered md / me, no sign-dependent range keeping, e = R mod n
# at the start.  Checks what the kernel's int32 / int64 arithmetic relies on.
_N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
_M30 = (1 << 30) - 1


def _s32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >> 31 else x


def _i32(x):
    assert -(1 << 31) <= x < (1 << 31)
    return x


def _divsteps30_var(eta, f, g):
    """safegcd.h divsteps30_var on 32-bit words."""
    u, v, q, r, i = 1, 0, 0, 1, 30
    f &= 0xFFFFFFFF
    g &= 0xFFFFFFFF
    while True:
        gg = (g | (0xFFFFFFFF << i)) & 0xFFFFFFFF
        z = (gg & -gg).bit_length() - 1
        g >>= z
        u = (u << z) & 0xFFFFFFFF
        v = (v << z) & 0xFFFFFFFF
        eta -= z
        i -= z
        if i == 0:
            return eta, _s32(u), _s32(v), _s32(q), _s32(r)
        if eta < 0:
            eta = -eta
            f, g, u, q, v, r = g, -f & 0xFFFFFFFF, q, -u & 0xFFFFFFFF, r, -v & 0xFFFFFFFF
        m = (0xFFFFFFFF >> (32 - min(eta + 1, i))) & 63
        w = (f * g * ((f * f - 2) & 0xFFFFFFFF)) & m
        g, q, r = (g + f * w) & 0xFFFFFFFF, (q + u * w) & 0xFFFFFFFF, (r + v * w) & 0xFFFFFFFF


def _center(limbs):
    cs = [((x + (1 << 29)) >> 30) if L < 8 else 0 for L, x in enumerate(limbs)]
    return [_i32(x - (c << 30) + (cs[L - 1] if L else 0)) for L, (x, c) in enumerate(zip(limbs, cs))]


def _shift30(cols):
    for p in cols:
        assert abs(p) < (1 << 61)  # int64 with room: |u A + v B + md n_L| < 2^60.x
    lo = [((p & _M30) ^ (1 << 29)) - (1 << 29) for p in cols]
    assert lo[0] == 0  # the batch's matrix makes the low limb vanish
    hi = [_i32((p - l) >> 30) for p, l in zip(cols, lo)]
    return [_i32(hi[L] + (lo[L + 1] if L < 8 else 0)) for L in range(9)]


def _limbs30(x):
    return [(x >> (30 * L)) & _M30 for L in range(8)] + [x >> 240]


def _value(limbs):
    return sum(v << (30 * L) for L, v in enumerate(limbs))


def _inv_wave(x):
    n_l = _limbs30(_N)
    f, g = _center(n_l), _center(_limbs30(x))
    d, e = [0] * 9, _center(_limbs30((1 << 261) % _N))
    eta, batches = -1, 0
    for _ in range(25):
        batches += 1
        eta, u, v, q, r = _divsteps30_var(eta, f[0], g[0])
        d0, e0 = d[0] & 0xFFFFFFFF, e[0] & 0xFFFFFFFF
        md = _s32((-((u * d0 + v * e0) * 0x11FF43B1)) << 2) >> 2   # center30(0 - c nInv30)
        me = _s32((-((q * d0 + r * e0) * 0x11FF43B1)) << 2) >> 2
        f, g = (_center(_shift30([u * a + v * b for a, b in zip(f, g)])),
                _center(_shift30([q * a + r * b for a, b in zip(f, g)])))
        d, e = (_center(_shift30([u * a + v * b + md * nl for a, b, nl in zip(d, e, n_l)])),
                _center(_shift30([q * a + r * b + me * nl for a, b, nl in zip(d, e, n_l)])))
        for limbs in (f, g, d, e):
            assert all(abs(t) <= (1 << 29) + 2 for t in limbs[:8])
        assert abs(_value(d)) < 13.5 * _N and abs(_value(e)) < 13.5 * _N
        if not any(g):
            break
    fv = _value(f)
    assert fv in (1, -1)
    pos = (f[0] + (f[1] << 30)) & 0xFFFFFFFF == 1  # the kernel's sign test
    assert pos == (fv == 1)
    D = (_value(d) if pos else -_value(d)) + 16 * _N
    assert 0 < D < (1 << 261)
    return D, batches


def test_lane_parallel_safegcd_bounds_and_result():
    import random
    rng = random.Random(0x494E56)
    xs = [1, 2, 3, _N - 1, _N - 2, 1 << 255, (1 << 256) % _N, 0x7FFFFFFF, 1 << 30, (1 << 30) - 1]
    xs += [rng.randrange(1, _N) for _ in range(1500)]
    xs += [rng.randrange(1, 1 << rng.randrange(1, 257)) % _N or 1 for _ in range(300)]
    most = 0
    for x in xs:
        D, batches = _inv_wave(x)
        assert D % _N == (1 << 261) * pow(x, -1, _N) % _N
        most = max(most, batches)
    assert most <= 25
