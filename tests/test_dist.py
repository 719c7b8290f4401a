"""N>1 path on CPU: world-size-2 gloo.  Each rank takes its contiguous shard
(simple_pbft_amd.sharding -- the split bench.py uses across processes and
pbftv_api.cpp uses across a context's devices), verifies it with the CPU
oracle standing in for its GPU, and the gathered shard bitmaps must equal the
single-process result.  Also checks bench.py's barrier / max-over-ranks
reduction.  No collective is on the data path of the product: the gather here
is only the test's check."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, fixture_arrays

sys.path.insert(0, ROOT)
from simple_pbft_amd.sharding import concat_bitmaps, plan_shards, shard_of  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    import ctypes
    import json

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    from conftest import fixture_arrays as fa

    d = bench.Dist(ws)
    with open(os.path.join(ROOT, "tests", "golden", "ecdsa.json")) as f:
        fx = json.load(f)
    keys, hashes, sigs, kidx, expect = fa(fx)
    reps = 8
    H, S, K = np.tile(hashes, (reps, 1)), np.tile(sigs, (reps, 1)), np.tile(kidx, reps)
    n = len(K)
    lo, hi = shard_of(n, ws, rank)
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    vp = ctypes.c_void_p
    L.oracle_ecdsa_p256_verify_batch.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint32, vp, ctypes.c_int]
    m = hi - lo
    bm = np.zeros((m + 7) // 8 + 1, np.uint8)
    h, s, k = (np.ascontiguousarray(a[lo:hi]) for a in (H, S, K))
    L.oracle_ecdsa_p256_verify_batch(h.ctypes.data, s.ctypes.data, k.ctypes.data, m, keys.ctypes.data, len(keys),
                                     bm.ctypes.data, 2)
    width = (n + 7) // 8 + 1
    buf = torch.zeros(width, dtype=torch.uint8)
    buf[:len(bm)] = torch.from_numpy(bm)
    out = [torch.zeros(width, dtype=torch.uint8) for _ in range(ws)]
    dist.all_gather(out, buf)
    d.barrier()
    tmax = d.max(float(rank + 1))
    tsum = d.sum(1.0)
    if rank == 0:
        shards = plan_shards(n, ws)
        full = concat_bitmaps(n, shards, [o.numpy() for o in out])
        got = np.unpackbits(full, bitorder="little")[:n].astype(bool)
        q.put((bool((got == np.tile(expect, reps)).all()), tmax, tsum, shards))
    d.close()


def test_plan_shards_properties():
    for n in [0, 1, 511, 512, 513, 1 << 20, 1_000_003]:
        for parts in [1, 2, 3, 4, 8]:
            sh = plan_shards(n, parts)
            assert len(sh) <= parts
            assert sum(hi - lo for lo, hi in sh) == n
            assert all(lo % 512 == 0 for lo, _ in sh)
            assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))


def test_gloo_world2_sharded_verify_matches_single_process(ecdsa_fixtures):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ok, tmax, tsum, shards = res
    assert ok
    assert tmax == 2.0 and tsum == 2.0
    assert len(shards) == 2


def _bench(args, env_extra, timeout=240):
    import subprocess
    env = dict(os.environ, PBFTV_BENCH_PROBE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("gpus", [1, 2, 3])
def test_bench_gpus_flag_starts_that_many_ranks(gpus):
    """`python bench.py --gpus N` (the driver's plain command, no torch.distributed.run)
    starts N rank processes itself -- gloo barrier, max-over-ranks -- and the
    ranks see WORLD_SIZE = N; --gpus 1 stays one process.  PBFTV_BENCH_PROBE
    stops every rank right after the rendezvous, before any GPU call."""
    import json
    r = _bench(["--gpus", str(gpus), "--n", "4096"], {})
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["world_size"] == gpus and line["ranks_seen"] == gpus
    assert line["spawned"] == (gpus > 1) and line["shared_data"] == (gpus > 1)


@pytest.mark.parametrize("stub", ["raise", "devices", "check", "ok"])
def test_bench_in_context_failure_fails_the_run(stub):
    """A failure of the one-process multi-device leg (an exception, a context
    that does not span --gpus devices, a wrong bitmap) makes `bench.py --gpus N`
    exit non-zero, with the line still printed.  The same
    judgement (bench.in_context_result) as the real leg, on a stub leg."""
    import json
    r = _bench(["--gpus", "2", "--n", "4096"], {"PBFTV_BENCH_PROBE": f"in_context:{stub}"})
    line = json.loads(r.stdout.strip().splitlines()[-1])
    if stub == "ok":
        assert r.returncode == 0, r.stderr[-2000:]
        assert line["in_context"]["devices"] == [0, 1]
    else:
        assert r.returncode != 0
        assert "bench.py: in_context" in r.stderr


def test_bench_gpus_mismatch_fails_loudly():
    """Under torch.distributed.run with a world size other than --gpus, bench.py refuses."""
    r = _bench(["--gpus", "2", "--n", "4096"], {"WORLD_SIZE": "1"})
    assert r.returncode != 0 and "--gpus 2 but WORLD_SIZE=1" in r.stderr


def test_bench_numa_pinning_helpers(monkeypatch):
    """bench.py pins each rank to its GPU's NUMA node:
    the cpulist parser, the opt-out, and a graceful no-op where the GPU's
    bus id or node cannot be read (this container has no GPU) -- the
    affinity is left as it was."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench._cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert bench._cpulist("") == []
    before = os.sched_getaffinity(0)
    monkeypatch.setenv("PBFTV_BENCH_PIN", "0")
    assert bench.pin_to_gpu_node(0) == {"pinned": False, "why": "PBFTV_BENCH_PIN=0"}
    monkeypatch.delenv("PBFTV_BENCH_PIN")
    r = bench.pin_to_gpu_node(0)
    assert r["pinned"] is False and r["why"]
    assert os.sched_getaffinity(0) == before
