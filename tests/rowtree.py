"""Chosen-scalar signatures whose partial sums meet INSIDE the latency path's
row tree (verify_kernels.h block_verify_rows, rows.h), for the row-schedule
parity tests (tests/test_gpu_rows_exceptional.py).

Test infrastructure only.  The key is Q = G, so a signature with chosen
scalars (u1, u2) makes the verifier recompute exactly u1 = e/s, u2 = r/s
(conftest.chosen_scalar_sig), and every table point of the verify is a known
multiple of G: window w contributes

    V_w = d1_w 2^sG_w G + d2_w 2^sQ_w G

(d1 / d2 the signed digits of u1 / u2 over the G / key window geometry,
bench.window_widths, sG / sQ the windows' first bits), so two partial sums
meet -- a doubling or a cancellation, x-coordinates equal -- exactly when
their scalars agree up to sign mod n.  The row kernel sums:

  * window w: the G entry + the key entry (mmadd_pairs) when both digits are
    non-zero ("pair"), else the lone entry; both zero is a "rare" window;
  * wave position t (windows 2t, 2t + 1): S_t = V_2t + V_2t+1 ("wave");
  * the tree: at level m (1, 2, 4) position t (a multiple of 2m) adds
    position t + m's subtotal ("level"); level 4 at t = 0 is the root, fused
    with the x check (xyzz_add_check_rows).

`tree_events` restates that schedule on scalars and lists every meeting;
`solve` picks the digits of two disjoint groups of table points so that the
groups' sums meet (sum A = +-sum B, as integers), every other digit random;
`vectors` builds, per geometry, one signature per meeting the geometry has
(both signs), each with an r-wrong twin that keeps (u1, u2) -- so the tree
meets the same way and Go's answer is reject -- plus rare windows and
r + n < p.  Expected bits come from the oracle restatement (oracle/p256.py,
pinned by the golden fixtures), never from this model: the model only says
which signatures must take the exact path."""
from __future__ import annotations

import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import window_widths  # noqa: E402
from oracle import p256  # noqa: E402

N = p256.N
P_MINUS_N = p256.P - p256.N  # r < p - n: r + n is a second x candidate (the exact path)


def starts(widths):
    out, b = [], 0
    for w in widths:
        out.append(b)
        b += w
    return out


def signed_digits(u: int, widths) -> list:
    """p256_algo.h signed recoding: digits in (-2^(w-1), 2^(w-1)]."""
    out, c, bit = [], 0, 0
    for wd in widths:
        d = ((u >> bit) & ((1 << wd) - 1)) + c
        c = 1 if d > (1 << (wd - 1)) else 0
        out.append(d - (c << wd))
        bit += wd
    return out


class Geom:
    def __init__(self, gq):
        self.gq = tuple(gq)
        self.gw, self.qw = window_widths(gq[0]), window_widths(gq[1])
        self.gs, self.qs = starts(self.gw), starts(self.qw)
        self.nG, self.nQ = len(self.gw), len(self.qw)
        self.nW = max(self.nG, self.nQ)
        self.waves = (self.nW + 1) // 2
        assert 8 < self.nW <= 16, "the row schedule's geometries (RowsGeom::ok)"

    def var(self, k: str, w: int):
        """table point k ('G' or 'Q') of window w: (first bit, width)"""
        return (self.gs[w], self.gw[w]) if k == "G" else (self.qs[w], self.qw[w])

    def has(self, k: str, w: int) -> bool:
        return w < (self.nG if k == "G" else self.nQ)

    def window_vars(self, ws):
        return [(k, w) for w in ws for k in ("G", "Q") if self.has(k, w)]

    def position_windows(self, t: int, m: int = 0):
        """windows under tree position t at level m (m = 0: the wave's own two)"""
        span = 2 * max(m, 1)
        lo = 2 * t
        return [w for w in range(lo, lo + span) if w < self.nW]


def _meet(a: int, b: int):
    a, b = a % N, b % N
    if a == 0 or b == 0:
        return None  # infinity: a cancellation below, already listed
    if a == b:
        return "dbl"
    if (a + b) % N == 0:
        return "cancel"
    return None


def tree_events(g: Geom, u1: int, u2: int) -> list:
    """Every meeting of two partial sums in the row tree, in the kernel's
    order: ("pair", w, how), ("rare", w), ("wave", t, how), ("level", m, t, how)."""
    d1, d2 = signed_digits(u1, g.gw), signed_digits(u2, g.qw)
    ev, vals = [], []
    for w in range(g.nW):
        a = d1[w] << g.gs[w] if w < g.nG else 0
        b = d2[w] << g.qs[w] if w < g.nQ else 0
        na, nb = w < g.nG and d1[w] != 0, w < g.nQ and d2[w] != 0
        if not na and not nb:
            ev.append(("rare", w))
        elif na and nb:
            how = _meet(a, b)
            if how:
                ev.append(("pair", w, how))
        vals.append(a + b)
    node = {}
    for t in range(g.waves):
        s = vals[2 * t]
        if 2 * t + 1 < g.nW:
            how = _meet(s, vals[2 * t + 1])
            if how:
                ev.append(("wave", t, how))
            s += vals[2 * t + 1]
        node[t] = s
    for m in (1, 2, 4):
        for t in range(0, g.waves, 2 * m):
            if t + m < g.waves:
                how = _meet(node[t], node[t + m])
                if how:
                    ev.append(("level", m, t, how))
                node[t] += node[t + m]
    assert (node[0] - u1 - u2) % N == 0
    return ev


def _rand_digit(rng, wd, nonzero=True):
    while True:
        d = rng.randint(-(1 << (wd - 1)) + 1, 1 << (wd - 1))
        if d or not nonzero:
            return d


def _compose(g: Geom, dig: dict):
    u1 = sum(dig[("G", w)] << g.gs[w] for w in range(g.nG))
    u2 = sum(dig[("Q", w)] << g.qs[w] for w in range(g.nQ))
    return u1, u2


def _in_range(g: Geom, dig: dict, u1: int, u2: int) -> bool:
    if not (0 < u1 < N and 0 < u2 < N):
        return False
    return (signed_digits(u1, g.gw) == [dig[("G", w)] for w in range(g.nG)] and
            signed_digits(u2, g.qw) == [dig[("Q", w)] for w in range(g.nQ)])


def _random_digits(g: Geom, rng) -> dict:
    dig = {}
    for k, n, ws in (("G", g.nG, g.gw), ("Q", g.nQ, g.qw)):
        for w in range(n):
            # the top window positive and small: 0 < u < 2^255 < n
            dig[(k, w)] = rng.randint(2, 1 << (ws[w] - 3)) if w == n - 1 else _rand_digit(rng, ws[w])
    return dig


def solve(g: Geom, A, B, sign: int, rng, tries: int = 4000, wrap: int = 0, want=None):
    """Digits with sum over A = sign * sum over B + wrap * n (A, B: disjoint
    lists of table points (k, w); wrap -1, 0 or 1: the sums meet modulo n,
    which groups holding the top windows need), every other digit random, u1
    and u2 in (0, n) and recoding to exactly these digits (and, given `want`,
    tree_events exactly [want]).  Points are taken in order of their first
    bit; each one's digit is fixed modulo the gap to the next point's first
    bit so the running difference stays divisible by it (random in its range
    otherwise), and the last one closes the difference exactly."""
    coef = {v: 1 for v in A}
    coef.update({v: -sign for v in B})
    order = sorted(coef, key=lambda v: (g.var(*v)[0], -g.var(*v)[1]))
    for _ in range(tries):
        dig = _random_digits(g, rng)
        R, ok = -wrap * N, True
        for i, v in enumerate(order):
            e, wd = g.var(*v)
            c = coef[v]
            if R % (1 << e):
                return None  # (a wrap by the odd n needs a group that holds bit 0)
            x = R >> e
            lo, hi = -(1 << (wd - 1)) + 1, 1 << (wd - 1)
            if i == len(order) - 1:
                d = -x * c
                if not lo <= d <= hi:
                    ok = False
                    break
            else:
                gap = g.var(*order[i + 1])[0] - e
                if gap == 0:
                    # the next point starts at the same bit: if it closes the
                    # sum, in its (narrower) range; else in this one's whole
                    # range, so the two do not simply cancel
                    last = i + 2 == len(order)
                    d = _rand_digit(rng, min(wd, g.var(*order[i + 1])[1]) if last else wd)
                else:
                    m = 1 << gap
                    base = (-c * x) % m
                    if base > m // 2:
                        base -= m
                    # a random digit of the right residue: -(2^(wd-1)) < base + k m <= 2^(wd-1)
                    # (none when the gap to the next point is wider than this
                    # digit and the residue is large: this try fails)
                    kmin, kmax = -((base - lo) // m), (hi - base) // m
                    if kmin > kmax:
                        ok = False
                        break
                    d = base + rng.randint(kmin, kmax) * m
            dig[v] = d
            R += c * d << e
        if not ok or R != 0:
            continue
        u1, u2 = _compose(g, dig)
        if _in_range(g, dig, u1, u2) and (want is None or tree_events(g, u1, u2) == [want]):
            return u1, u2
    return None


def _sig(u1: int, u2: int, r_mode: str, rng):
    """(hash bytes, r, s) under Q = G recomputing (u1, u2): r_mode "true" (r =
    x(R) mod n; R = infinity -> r = 1, rejected), "wrong" (r = u2 s' for a
    random s': the same scalars, an r that is not x(R)), "small" (r < p - n)."""
    if r_mode == "true":
        R = p256.scalar_mult((u1 + u2) % N, p256.G)
        r = 1 if R is None else R[0] % N
        s = r * pow(u2, -1, N) % N
    else:
        if r_mode == "wrong":
            s = rng.randrange(1, N)
            r = u2 * s % N
        else:
            r = rng.randrange(1, P_MINUS_N)
            s = r * pow(u2, -1, N) % N
    e = u1 * s % N
    return e.to_bytes(32, "big"), r, s


def _groups(g: Geom):
    """Every meeting the geometry's tree has: (tag, A, B, event-prefix)."""
    out = []
    for w in range(min(g.nG, g.nQ)):
        out.append((f"pair w{w}", [("G", w)], [("Q", w)], ("pair", w)))
    for t in range(g.waves):
        if 2 * t + 1 < g.nW:
            out.append((f"wave t{t}", g.window_vars([2 * t]), g.window_vars([2 * t + 1]), ("wave", t)))
    for m in (1, 2, 4):
        for t in range(0, g.waves, 2 * m):
            if t + m < g.waves:
                A = g.window_vars(range(2 * t, min(2 * (t + m), g.nW)))
                B = g.window_vars(range(2 * (t + m), min(2 * (t + 2 * m), g.nW)))
                out.append((f"level{m} t{t}", A, B, ("level", m, t)))
    return out


def vectors(gq, seed: int = 1):
    """Signatures for geometry gq under key 0 = G: a list of dicts
    {kind, hash (32 B), r, s, u1, u2, events, exceptional, expect}.
    exceptional: the row kernel must take its exact path (a meeting, a rare
    window, r + n < p); expect: the oracle's verdict."""
    g = Geom(gq)
    rng = random.Random(seed * 1000003 + gq[0] * 64 + gq[1])
    cases = []
    for tag, A, B, pre in _groups(g):
        for sign, how in ((1, "dbl"), (-1, "cancel")):
            if sign < 0 and len(A) + len(B) == g.nG + g.nQ:
                # the root's cancellation: sum A = -sum B over EVERY window
                # is u1 + u2 = 0, impossible as integers; mod n it is
                # u2 = n - u1 (R = infinity: Go rejects)
                for _ in range(100):
                    dig = _random_digits(g, rng)
                    u1 = _compose(g, dig)[0]
                    if 0 < u1 < N and tree_events(g, u1, N - u1) == [pre + (how,)]:
                        cases.append((f"{tag} {how}", (u1, N - u1)))
                        break
                continue
            # exactly this one meeting; as integers, else modulo n (a group
            # with the top windows); some meetings no digits can reach (a
            # pair past the windows where the G and key digits overlap, a
            # position whose partner sits too high): skipped
            for wrap in (0, 1, -1):
                uu = solve(g, A, B, sign, rng, tries=3000, wrap=wrap, want=pre + (how,))
                if uu:
                    cases.append((f"{tag} {how}" + (f" mod n{wrap:+d}" if wrap else ""), uu))
                    break
    # rare windows: a live window with both digits zero (a middle one, and one
    # past the G windows where only the key digit is live)
    for w in sorted({g.nW // 2, g.nW - 2}):
        for _ in range(100):
            dig = _random_digits(g, rng)
            for k in ("G", "Q"):
                if g.has(k, w):
                    dig[(k, w)] = 0
            uu = _compose(g, dig)
            if _in_range(g, dig, *uu) and tree_events(g, *uu) == [("rare", w)]:
                cases.append((f"rare w{w}", uu))
                break
    plain = None
    for _ in range(100):
        dig = _random_digits(g, rng)
        uu = _compose(g, dig)
        if _in_range(g, dig, *uu) and not tree_events(g, *uu):
            plain = uu
            break
    out = []
    for kind, (u1, u2) in cases:
        for mode in ("true", "wrong"):
            h, r, s = _sig(u1, u2, mode, rng)
            out.append({"kind": f"{kind} r={mode}", "hash": h, "r": r, "s": s, "u1": u1, "u2": u2,
                        "events": tree_events(g, u1, u2), "exceptional": True})
    # r + n < p with no meeting (the exact path's second x candidate; Go rejects it here)
    h, r, s = _sig(*plain, "small", rng)
    out.append({"kind": "r+n<p", "hash": h, "r": r, "s": s, "u1": plain[0], "u2": plain[1], "events": [],
                "exceptional": True})
    # and a plain one (the fast path: no exact rerun)
    h, r, s = _sig(*plain, "true", rng)
    out.append({"kind": "plain", "hash": h, "r": r, "s": s, "u1": plain[0], "u2": plain[1], "events": [],
                "exceptional": False})
    for v in out:
        v["expect"] = p256.verify(v["hash"], v["r"], v["s"], p256.GX, p256.GY)
    return out


def arrays(vecs):
    """(hashes[n, 32], sigs[n, 64] r||s big-endian) uint8 arrays of vectors()."""
    import numpy as np
    H = np.array([list(v["hash"]) for v in vecs], np.uint8).reshape(-1, 32)
    S = np.array([list(v["r"].to_bytes(32, "big") + v["s"].to_bytes(32, "big")) for v in vecs],
                 np.uint8).reshape(-1, 64)
    return H, S


def g_key():
    import numpy as np
    return np.frombuffer(p256.GX.to_bytes(32, "big") + p256.GY.to_bytes(32, "big"), np.uint8)[None, :].copy()
