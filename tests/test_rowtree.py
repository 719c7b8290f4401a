"""CPU checks of the row-tree vectors (tests/golden/rows_exceptional.json,
made by tests/golden/make_rows_fixtures.py from tests/rowtree.py) that the
GPU test tests/test_gpu_rows_exceptional.py serves through the armed and the
launched row kernels: each signature recomputes the committed (u1, u2), the
tree model finds exactly the committed meetings, every geometry covers every
kind of meeting its digits can reach, and the committed verdict is the C
oracle's (oracle/p256_ref.c -- an algorithm unlike the kernel's and unlike
oracle/p256.py, which made the fixture)."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

import rowtree
from conftest import GOLDEN

N = rowtree.N


@pytest.fixture(scope="module")
def rows_fx():
    with open(os.path.join(GOLDEN, "rows_exceptional.json")) as f:
        return json.load(f)["geometries"]


def test_rows_fixture_scalars_and_events(rows_fx):
    for key, vs in rows_fx.items():
        g = rowtree.Geom(tuple(int(x) for x in key.split(",")))
        for v in vs:
            e, r, s = int(v["hash"], 16), int(v["r"], 16), int(v["s"], 16)
            w = pow(s, -1, N)
            u1, u2 = e * w % N, r * w % N
            assert (u1, u2) == (int(v["u1"], 16), int(v["u2"], 16)), (key, v["kind"])
            ev = rowtree.tree_events(g, u1, u2)
            assert [list(x) for x in ev] == v["events"], (key, v["kind"])
            assert v["exceptional"] == (bool(ev) or r < rowtree.P_MINUS_N), (key, v["kind"])


def test_rows_fixture_covers_every_reachable_meeting(rows_fx):
    """Every geometry holds a doubling and a cancellation at a pair of window
    0 and of a higher window, at a wave's own pair, at tree levels 1 and 2 and
    at the fused root, plus rare windows, r + n < p and a plain signature --
    each once with r = x(R) and once with an r-wrong twin of the same scalars."""
    for key, vs in rows_fx.items():
        kinds = [v["kind"] for v in vs]
        ev = {tuple(e[:-1]) + (e[-1],) for v in vs for e in v["events"] if e[0] != "rare"}
        for how in ("dbl", "cancel"):
            for need in (("pair", 0), ("pair", 1), ("wave", 0), ("wave", 1), ("level", 1, 0), ("level", 2, 0),
                         ("level", 4, 0)):
                assert need + (how,) in ev, (key, need, how)
        assert any(e[0] == "rare" for v in vs for e in v["events"]), key
        assert "r+n<p" in kinds and "plain" in kinds
        for k in kinds:
            if k.endswith("r=true"):
                assert k[:-len("r=true")] + "r=wrong" in kinds
        # the wrong-r twins are rejects whatever the tree does: a zero ZZ
        # mistaken for a sum would accept them (X = r ZZ = 0)
        assert not any(v["expect"] for v in vs if v["kind"].endswith("r=wrong"))
        assert any(v["expect"] for v in vs if v["kind"].endswith("r=true"))


def test_rows_fixture_expect_matches_c_oracle(rows_fx, oracle_lib):
    key = rowtree.g_key()
    for gk, vs in rows_fx.items():
        H = np.array([list(bytes.fromhex(v["hash"])) for v in vs], np.uint8)
        S = np.array([list(bytes.fromhex(v["r"]) + bytes.fromhex(v["s"])) for v in vs], np.uint8)
        K = np.zeros(len(vs), np.uint32)
        bm = np.zeros((len(vs) + 7) // 8, np.uint8)
        oracle_lib.oracle_ecdsa_p256_verify_batch(H.ctypes.data, S.ctypes.data, K.ctypes.data, len(vs),
                                                  key.ctypes.data, 1, bm.ctypes.data, 4)
        got = np.unpackbits(bm, bitorder="little")[:len(vs)].astype(bool)
        assert got.tolist() == [v["expect"] for v in vs], gk


def test_solver_meets_where_asked():
    """rowtree.solve on a fresh seed: the digits it returns recode to the
    scalars and meet exactly where asked (the generator is not only its
    committed output)."""
    import random
    g = rowtree.Geom((29, 21))
    rng = random.Random(7)
    for tag, A, B, pre in rowtree._groups(g)[:12]:
        uu = rowtree.solve(g, A, B, 1, rng, tries=500, want=pre + ("dbl",))
        if uu is not None:
            assert rowtree.tree_events(g, *uu) == [pre + ("dbl",)]
