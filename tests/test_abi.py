"""The C ABI library (CPU-side checks): it loads, exports every symbol
include/pbftv.h declares, its host-only entry points (Go-JSON preimages,
State.verifyMsg) match the oracle, and it refuses to run without a GPU
(no CPU fallback)."""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from oracle import gojson


@pytest.fixture(scope="module")
def pb():
    from simple_pbft_amd import pbftv
    so = pbftv.LIB_PATH
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "simple_pbft_amd"), "-j8"], check=True)
    return pbftv


def test_library_exports_every_header_symbol(pb):
    L = pb.lib()
    syms = pb.header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", pb.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(syms) <= exported


def test_library_is_gfx950_code(pb):
    """The embedded offload bundle targets gfx950 (and nothing else)."""
    blob = open(pb.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100", b"sm_"):
        assert other not in blob


def test_no_cpu_fallback(pb):
    """Without a GPU the context cannot be opened: the product never falls back to the CPU."""
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("a GPU is visible")
    except Exception:
        pass
    with pytest.raises(pb.PbftvError) as ei:
        pb.Verifier()
    assert ei.value.code == pb.PBFTV_ENODEV


def test_gojson_product_matches_fixtures(pb, digest_kats):
    for r in digest_kats["requests"] + digest_kats["escapes"]:
        got = pb.gojson_request(r["timestamp"], bytes.fromhex(r["clientID"]), bytes.fromhex(r["operation"]),
                                r["sequenceID"])
        assert got.hex() == r["preimage"]
    for v in digest_kats["votes"]:
        got = pb.gojson_vote(v["viewID"], v["sequenceID"], bytes.fromhex(v["digest"]), bytes.fromhex(v["nodeID"]),
                             v["msgType"])
        assert got.hex() == v["preimage"]
    for p in digest_kats["preprepares"]:
        req = None
        if p["request"] is not None:
            ts, cid, op, seq = p["request"]
            req = (ts, bytes.fromhex(cid), bytes.fromhex(op), seq)
        assert pb.gojson_preprepare(p["viewID"], p["sequenceID"], bytes.fromhex(p["digest"]), req).hex() == p["preimage"]
    for r in digest_kats["replies"]:
        got = pb.gojson_reply(r["viewID"], r["timestamp"], bytes.fromhex(r["clientID"]), bytes.fromhex(r["nodeID"]),
                              bytes.fromhex(r["result"]))
        assert got.hex() == r["preimage"]


def test_gojson_product_random_vs_restatement(pb):
    rng = np.random.default_rng(9)
    alphabet = [b"x", b"<", b">", b"&", b'"', b"\\", b"\t", b"\x01", b"\x7f", b"\xe2\x80\xa8", b"\xe2\x80\xa9",
                b"\xff", b"\xc2\xa2", b"\xe0\x9f\xbf", b"\xf0\x90\x80\x80", b"\xef\xbf\xbd", b"\xe2\x82", b"\xc0\x80"]
    for _ in range(2000):
        a = b"".join(alphabet[i] for i in rng.integers(0, len(alphabet), rng.integers(0, 10)))
        b = rng.bytes(int(rng.integers(0, 16)))
        ts, seq = int(rng.integers(-2 ** 63, 2 ** 63 - 1)), int(rng.integers(-2 ** 63, 2 ** 63 - 1))
        assert pb.gojson_request(ts, a, b, seq) == gojson.request(ts, a, b, seq)
        mt = int(rng.integers(0, 2))
        assert pb.gojson_vote(ts, seq, a, b, mt) == gojson.vote(ts, seq, a, b, mt)
        assert pb.gojson_reply(ts, seq, a, b, a + b) == gojson.reply(ts, seq, a, b, a + b)


def test_verify_msg_batch_matches_oracle(pb, oracle_lib):
    rng = np.random.default_rng(4)
    d = hashlib.sha256(b"request").digest()
    good = d.hex().encode()
    cases = []
    for _ in range(600):
        view = int(rng.choice([10, 11]))
        seq = int(rng.integers(0, 10))
        kind = int(rng.integers(0, 5))
        dg = [good, good.upper(), good[:-1], good + b"0", hashlib.sha256(b"other").hexdigest().encode()][kind]
        cases.append((view, seq, dg))
    for last in (-1, 4):
        got = pb.verify_msg_batch(10, last, d, [c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases])
        want = [oracle_lib.oracle_verify_msg(10, last, d, v, s, g, len(g)) == 1 for v, s, g in cases]
        assert got.tolist() == want
        assert any(want) and not all(want)


def _call_args(text: str, start: int) -> list[str]:
    """Top-level comma-separated arguments of the call whose '(' is at start."""
    depth, cur, out = 0, "", []
    for ch in text[start:]:
        if ch in "([{":
            depth += 1
            if depth == 1:
                continue
        elif ch in ")]}":
            depth -= 1
            if depth == 0:
                out.append(cur.strip())
                break
        if ch == "," and depth == 1:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    return [a for a in out if a]


def test_go_binding_calls_only_header_functions_with_their_arity():
    """go/pbftv (the cgo package; no Go toolchain here) calls only functions
    include/pbftv.h declares, each with the header's parameter count."""
    import glob
    import re
    from simple_pbft_amd.pbftv import HEADER_PATH
    with open(HEADER_PATH) as f:
        hdr = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    arity = {}
    for m in re.finditer(r"\b(pbftv_[a-z0-9_]+)\s*\(", hdr):
        args = _call_args(hdr, m.end() - 1)
        arity[m.group(1)] = 0 if args == ["void"] else len(args)
    calls = 0
    for path in glob.glob(os.path.join(ROOT, "go", "pbftv", "*.go")):
        with open(path) as f:
            src = f.read()
        for m in re.finditer(r"\bC\.(pbftv_[a-z0-9_]+)\(", src):
            name = m.group(1)
            assert name in arity, f"{path}: {name} is not in include/pbftv.h"
            n_args = len(_call_args(src, m.end() - 1))
            assert n_args == arity[name], f"{path}: {name} called with {n_args} args, header has {arity[name]}"
            calls += 1
    assert calls >= 20
