"""The row schedule's exceptional paths, pinned.

block_verify_rows (verify_kernels.h) adds a signature's table points in a
tree of waves whose partial sums are grouped unlike the lane comb's and the
quad schedule's.  A doubling or a cancellation anywhere in that tree leaves a
zero ZZ that the fused root check must see (else X = r ZZ = 0 accepts any
r), a live window with two zero digits and r + n < p must take the exact
path too.  The armed kernel hands such a certificate back (result byte 2) and
the host reruns it with the launched kernel, whose wave 0 recomputes the sum
exactly.

The vectors (tests/golden/rows_exceptional.json, tests/rowtree.py) meet at
every place the geometry's digits can reach -- a pair (G entry = +-key
entry) at windows 0..4, a wave's own pair, tree levels 1 and 2, the fused
root -- as doublings and cancellations, each with an r-wrong twin of the same
scalars, plus rare windows and r + n < p; the golden vectors (other keys) ride
along.  Each is served through (a) the armed narrow kernel (4-signature
certificates), (b) the armed wide kernel (67-signature certificates, the
crafted ones both in slot workgroups and in helpers), (c) the launched
k_ecdsa_rows, (d) a 67-signature certificate split between the armed narrow
slots and one launch (PBFTV_QC_WIDE=split), at the 100-key geometry (29, 21), the 4-key geometry (29, 24)
and a seven-wave one (29, 20).  pbftv_qc_counters says which kernel served
each call, that an armed call with an exceptional signature was rerun, and
how many signatures took the launched kernel's exact path -- exactly the
ones the tree model flags -- and every bit is the oracle's."""
from __future__ import annotations

import json
import os
import time

import numpy as np
import pytest

import rowtree
from conftest import GOLDEN, fixture_arrays

pytestmark = pytest.mark.gpu

# golden kinds whose row-tree meetings cannot be predicted (crafted doublings
# under keys other than G): not used here
_UNPREDICTABLE = ("u1G==u2Q doubling valid", "u1G==-u2Q infinity")


def _golden_rows(ecdsa_fixtures):
    """golden vectors (keys shifted by one: key 0 is G) with their exact-path
    flag: range checks pass, the key is valid and r < p - n (no meeting in
    the tree for random scalars, probability ~2^-200 of one)."""
    keys, H, S, K, E = fixture_arrays(ecdsa_fixtures)
    vk = [k["valid"] for k in ecdsa_fixtures["keys"]]
    rows = []
    for i, v in enumerate(ecdsa_fixtures["vectors"]):
        if v["kind"] in _UNPREDICTABLE:
            continue
        r, s, k = int(v["r"], 16), int(v["s"], 16), int(v["key"])
        in_range = 0 < r < rowtree.N and 0 < s < rowtree.N and k < len(vk) and vk[k]
        exc = bool(in_range and (r < rowtree.P_MINUS_N or v["kind"].startswith("R.x>=n valid (u1=0")))
        rows.append((H[i], S[i], K[i] + 1, bool(E[i]), exc, v["kind"]))
    return keys, rows


def _all_rows(gq, ecdsa_fixtures):
    with open(os.path.join(GOLDEN, "rows_exceptional.json")) as f:
        vs = json.load(f)["geometries"][f"{gq[0]},{gq[1]}"]
    crafted = [(np.frombuffer(bytes.fromhex(v["hash"]), np.uint8),
                np.frombuffer(bytes.fromhex(v["r"]) + bytes.fromhex(v["s"]), np.uint8),
                0, v["expect"], v["exceptional"], v["kind"]) for v in vs]
    gkeys, golden = _golden_rows(ecdsa_fixtures)
    keys = np.concatenate([rowtree.g_key(), gkeys])
    return keys, crafted, golden


def _call(v, rows):
    H = np.stack([x[0] for x in rows])
    S = np.stack([x[1] for x in rows])
    K = np.array([x[2] for x in rows], np.uint32)
    c0 = v.qc_counters(0)
    got = v.verify_batch(H, S, K)
    c1 = v.qc_counters(0)
    d = {k: c1[k] - c0[k] for k in ("calls", "armed", "reruns", "exact_sigs", "launches")}
    want = np.array([x[3] for x in rows], bool)
    bad = [rows[i][5] for i in np.nonzero(got != want)[0]]
    assert not bad, bad
    return d, sum(x[4] for x in rows)


def _wait_armed(v, rows, wide: bool, limit_s: float = 5.0):
    """plain certificates until one is served by the armed kernel of the right
    shape (the keeper arms after the first call; a wide kernel needs all of its
    workgroups resident)"""
    t0 = time.monotonic()
    while time.monotonic() - t0 < limit_s:
        d, _ = _call(v, rows)
        c = v.qc_counters(0)
        if d["armed"] == 1 and c["armed_wide"] == wide:
            return
        time.sleep(0.01)
    raise AssertionError(f"no armed {'wide' if wide else 'narrow'} kernel within {limit_s} s: {v.qc_counters(0)}")


@pytest.mark.parametrize("gq", [(29, 21), (29, 24), (29, 20)])
def test_row_tree_exceptional_paths(gq, ecdsa_fixtures, monkeypatch):
    from simple_pbft_amd import Verifier
    monkeypatch.setenv("PBFTV_GBITS", str(gq[0]))
    monkeypatch.setenv("PBFTV_QBITS", str(gq[1]))
    monkeypatch.setenv("PBFTV_QC_ARM", "0")        # phase (c) first: every call launched
    monkeypatch.setenv("PBFTV_QC_ARM_MS", "30000")  # then no keeper rotation during the phases
    keys, crafted, golden = _all_rows(gq, ecdsa_fixtures)
    plain = [x for x in golden if not x[4]]
    n_exc = sum(x[4] for x in crafted)
    assert n_exc >= 40 and any(not x[4] for x in crafted)
    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        assert v.table_config()[:2] == gq
        # (c) the launched row kernel: its own exact path, no armed kernel
        allrows = crafted + golden
        for a in range(0, len(allrows), 128):
            d, exc = _call(v, allrows[a:a + 128])
            assert d == {"calls": 1, "armed": 0, "reruns": 0, "exact_sigs": exc, "launches": 1}, (a, d, exc)
        # (a) the armed narrow kernel, certificates of 4: two crafted (a
        # signature and its twin, or two of a kind) and two plain golden ones
        monkeypatch.setenv("PBFTV_QC_ARM", "1")
        monkeypatch.setenv("PBFTV_QC_WIDE", "0")  # (phase (c)'s 128s would arm the wide kernel)
        _wait_armed(v, plain[:3], wide=False)
        for a in range(0, len(crafted), 2):
            rows = crafted[a:a + 2] + plain[(a % 40):(a % 40) + 2]
            d, exc = _call(v, rows)
            want = {"calls": 1, "armed": 1, "reruns": 1 if exc else 0, "exact_sigs": exc,
                    "launches": 1 if exc else 0}
            assert d == want, (rows[0][5], d, want)
        # every golden vector through the narrow kernel too (R.x >= n: r + n < p)
        for a in range(0, len(golden), 4):
            rows = golden[a:a + 4]
            d, exc = _call(v, rows)
            assert d["armed"] == 1 and d["exact_sigs"] == exc and d["reruns"] == (1 if exc else 0), (a, d)
        # (d) split wide certificates (PBFTV_QC_WIDE=split): the first na
        # signatures go to the armed narrow slots, the rest to one launch; an
        # exceptional one among the armed part reruns the whole certificate
        filler = (plain * 4)[:67]
        monkeypatch.setenv("PBFTV_QC_WIDE", "split")
        na = v.qc_counters(0)["armed_waves"]
        assert 1 <= na <= 8 and not v.qc_counters(0)["armed_wide"]
        for a in range(0, len(crafted), 20):
            rows = list(filler)
            for j, x in enumerate(crafted[a:a + 20]):
                rows[(j * 7 + a) % 67] = x
            d, exc = _call(v, rows)
            head = sum(x[4] for x in rows[:na])
            want = {"calls": 1, "armed": 1, "reruns": 1 if head else 0, "exact_sigs": exc,
                    "launches": 2 if head else 1}
            assert d == want, (a, d, want)
        # (b) the armed wide kernel: 67-signature certificates, crafted ones
        # at slot positions (< 8) and helper positions (>= 8)
        monkeypatch.delenv("PBFTV_QC_WIDE")
        _wait_armed(v, filler, wide=True)  # (the first wide call is launched, the next arming is wide)
        per = 20
        for a in range(0, len(crafted), per):
            part = crafted[a:a + per]
            rows = list(filler)
            for j, x in enumerate(part):
                rows[(j * 7 + a) % 67] = x
            d, exc = _call(v, rows)
            want = {"calls": 1, "armed": 1, "reruns": 1 if exc else 0, "exact_sigs": exc,
                    "launches": 1 if exc else 0}
            assert d == want, (a, d, want)
        assert v.qc_counters(0)["armed_wide"]


@pytest.mark.parametrize("kernel", ["one_wave", "quad"])
def test_row_tree_vectors_through_the_one_wave_kernels(kernel, ecdsa_fixtures, monkeypatch):
    """The same vectors (and the golden ones, and conftest's crafted sums)
    through the launched ONE-wave kernels, whose sums are grouped otherwise:
    "one_wave" is k_ecdsa_wave_lean (128 VGPRs, what a certificate launched
    beside a batch gets; PBFTV_QC_BUSY_ONE_WAVE=2 forces it), "quad" the quad
    schedule's k_ecdsa_wave (PBFTV_QC_ROWS=0).  Every bit against the oracle's
    expectation."""
    from conftest import crafted_exceptional
    from simple_pbft_amd import Verifier
    gq = (29, 21)
    monkeypatch.setenv("PBFTV_GBITS", str(gq[0]))
    monkeypatch.setenv("PBFTV_QBITS", str(gq[1]))
    monkeypatch.setenv("PBFTV_QC_ARM", "0")
    if kernel == "one_wave":
        monkeypatch.setenv("PBFTV_QC_BUSY_ONE_WAVE", "2")
    else:
        monkeypatch.setenv("PBFTV_QC_ROWS", "0")
    keys, crafted, golden = _all_rows(gq, ecdsa_fixtures)
    _, H2, S2, K2, E2 = crafted_exceptional()
    extra = [(H2[i], S2[i], 0, bool(E2[i]), None, f"crafted {i}") for i in range(len(K2))]
    allrows = crafted + golden + extra
    with Verifier(device_mask=1) as v:
        v.register_keys(keys)
        assert v.table_config()[:2] == gq
        for a in range(0, len(allrows), 100):
            d, _ = _call(v, [r if r[4] is not None else r[:4] + (False,) + r[5:] for r in allrows[a:a + 100]])
            assert d["launches"] == 1 and d["armed"] == 0 and d["exact_sigs"] == 0, d
