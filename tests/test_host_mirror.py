"""The C++ host mirror of the reference's consensus State and message pools
(simple_pbft_amd/csrc/host/pbft.h), driven by tests/cpp/test_consensus.cpp.

The program replays the reference's logged 4-node run (log/node1.log: three
client requests, their sequence IDs and digests) through State exactly as
pbft/network/node.go drives it, flushing every pool snapshot as one signature
batch; it also checks verifyMsg / Prepare / Commit error semantics
(pbft_impl.go:115-202), the 2f quorum with a corrupted vote in the snapshot,
and the pools' Add/Del/DelAll/MsgNum/GetAll under concurrent adds.

CPU: the crypto backend is the oracle (a test double behind pbft::Crypto).
GPU: the same program with pbft::GpuCrypto -- the product path over the C ABI.
"""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
BIN = os.path.join(CPP, "test_consensus")
LIB = os.path.join(ROOT, "simple_pbft_amd", "libpbftv.so")
ORACLE = os.path.join(ROOT, "oracle", "liboracle.so")


def build_consensus_test() -> str:
    srcs = [os.path.join(CPP, "test_consensus.cpp"),
            os.path.join(ROOT, "simple_pbft_amd", "csrc", "host", "pbft.h"), LIB, ORACLE]
    for so, d in ((LIB, "simple_pbft_amd"), (ORACLE, "oracle")):
        if not os.path.exists(so):
            subprocess.run(["make", "-C", os.path.join(ROOT, d), "-s", "-j8"], check=True)
    if os.path.exists(BIN) and all(os.path.getmtime(s) <= os.path.getmtime(BIN) for s in srcs):
        return BIN
    subprocess.run(
        ["g++", "-O1", "-std=c++17", "-Wall", "-o", BIN, os.path.join(CPP, "test_consensus.cpp"),
         "-I", os.path.join(ROOT, "simple_pbft_amd", "csrc", "host"), "-I", os.path.join(ROOT, "include"),
         "-L", os.path.dirname(LIB), "-lpbftv", "-L", os.path.dirname(ORACLE), "-loracle",
         "-Wl,-rpath,$ORIGIN/../../simple_pbft_amd", "-Wl,-rpath,$ORIGIN/../../oracle", "-lpthread"],
        check=True)
    return BIN


CGO = os.path.join(CPP, "test_cgo_pattern")


def build_cgo_pattern_test() -> str:
    """tests/cpp/test_cgo_pattern.cpp: the C ABI driven as a cgo shim drives it."""
    src = os.path.join(CPP, "test_cgo_pattern.cpp")
    for so, d in ((LIB, "simple_pbft_amd"), (ORACLE, "oracle")):
        if not os.path.exists(so):
            subprocess.run(["make", "-C", os.path.join(ROOT, d), "-s", "-j8"], check=True)
    if os.path.exists(CGO) and all(os.path.getmtime(s) <= os.path.getmtime(CGO) for s in (src, LIB, ORACLE)):
        return CGO
    subprocess.run(
        ["g++", "-O1", "-std=c++17", "-Wall", "-o", CGO, src, "-L", os.path.dirname(LIB), "-lpbftv", "-L",
         os.path.dirname(ORACLE), "-loracle", "-Wl,-rpath,$ORIGIN/../../simple_pbft_amd",
         "-Wl,-rpath,$ORIGIN/../../oracle", "-lpthread"], check=True)
    return CGO


def test_cgo_pattern_program_builds():
    assert os.path.exists(build_cgo_pattern_test())


@pytest.mark.gpu
def test_cgo_calling_pattern_gpu():
    """Concurrent calls on one context from caller threads, caller-owned buffers
    poisoned right after each return, every result vs the oracle."""
    p = subprocess.run([build_cgo_pattern_test()], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert " 0 failed" in p.stdout


def _run(mode: str, timeout: int):
    exe = build_consensus_test()
    p = subprocess.run([exe, mode], capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "0 failed" in p.stdout
    return p.stdout


def test_consensus_mirror_cpu_double():
    out = _run("oracle", 120)
    assert f"oracle: " in out


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present")
def test_gpu_crypto_fails_loudly_without_gpu():
    """The product backend has no CPU fallback: constructing it without a GPU throws."""
    p = subprocess.run([build_consensus_test(), "gpu"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 3, p.stdout + p.stderr
    assert "pbftv_open" in p.stderr


@pytest.mark.gpu
def test_consensus_mirror_gpu():
    out = _run("gpu", 600)
    assert "gpu: " in out
