#!/usr/bin/env python3
"""Benchmark: ECDSA-P256 signature verifies/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n SIGS_PER_RANK]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Workload (BASELINE.json configs[3]): 1,048,576
signatures per rank over a 100-key table, 1 % corrupted evenly across the 8
corruption classes; synthetic (OpenSSL-signed, tools/synth.py).  One "step" =
one pass of the verify path (scalar kernel + comb kernel) over the rank's
whole batch, inputs already resident in HBM.  Consecutive steps alternate
over two library streams (--streams 2, pbftv_stream_create: each owns its
verify scratch), as a node flushing pool snapshots back to back would: step
j + 1's scalar stage runs in the wave slots step j's comb leaves free.  Every
step is still a complete verify of the batch, checked against the
construction; --streams 0 queues every step on one stream.  Multi-GPU: one process per GPU,
each verifying its own shard -- no collective on the data path; torch.distributed
(gloo, CPU) is used only for the barrier and the max-over-ranks time, so torch
never touches the GPU (it bundles its own HIP runtime).

Also reported on rank 0: p50 quorum-certificate verify latency (host submit ->
bitmap on host, configs[1]/[2] certificate sizes), the roofline of the
dominant kernel (HIP-event kernel durations from the timed region), and the
CPU baseline (oracle port, multi-threaded, bounded sample) beside an OpenSSL
stand-in.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402
from simple_pbft_amd.pbftv import K_ECDSA_COMB, K_ECDSA_SCALARS  # noqa: E402

METRIC = "sig verifies/sec at 1/2/4/8 MI355X; p50 quorum-cert verify latency"

# ---- algorithmic work per verify (DESIGN.md "Roofline"): limb MACs ----------
# One MAC = one 29x29-bit limb product accumulated into a 64-bit column
# (one v_mad_u64_u32).  fe_mul 81, fe_sqr 45, fn_mul 81 + 81 (n-reduction).
N_ORDER = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
FE_MUL, FE_SQR, FN_MUL = 81, 45, 162
MADD = 8 * FE_MUL + 2 * FE_SQR                     # XYZZ madd-2008-s (fes.h xyzz_madd_s_flip)
AFF_ADD = 4 * FE_MUL + 2 * FE_SQR                  # first pair, affine + affine (fes.h xyzz_aff_aff_s)
LAST_ADD = 4 * FE_MUL + 2 * FE_SQR                 # last addition fused with the x check (fes.h xyzz_last_*):
                                                   # U2, S2, PP, r ZZ1, R^2 + PP W under one reduction
JADD = 12 * FE_MUL + 4 * FE_SQR                    # add-2007-bl (final complete add)
CHECK = FE_MUL                                      # r to Montgomery form (r ZZ1 is in LAST_ADD)


def window_widths(code: int) -> list:
    """Window widths of a comb geometry code (p256_algo.h CombGeom): W-bit
    windows, or the mixed codes splitting 257 bits into wide bottom windows and
    one-bit-narrower top ones (21: 5 x 22 + 7 x 21, 29: 5 x 29 + 4 x 28)."""
    mixed = {11: (12, 22), 21: (22, 12), 29: (29, 9)}
    if code in mixed:
        kw, nwin = mixed[code]
        low = nwin * kw - 257
        return [kw] * (nwin - low) + [kw - 1] * low
    return [code] * (256 // code + 1)


def macs_comb(gbits: int, qbits: int) -> float:
    """Joint comb (verify_kernels.h k_ecdsa_comb, schedule p256_algo.h
    comb2_verify): one addition per nonzero signed digit of u1 (G table) and u2
    (key table) but the first (a load); of those, the first is affine + affine
    and the last is fused with the x check, the rest are mixed XYZZ additions.
    Windows below 256 bits are nonzero w.p. 1 - 2^-W; the top (carry) window
    w.p. ~1/2 when 256 % W == 0, else its 256 % W real bits make it nonzero."""
    def nonzero(w):
        ws = window_widths(w)
        top_bits = 256 - sum(ws[:-1])
        top = 0.5 if top_bits <= 0 else 1.0
        return sum(1 - 2.0 ** -x for x in ws[:-1]) + top
    return (nonzero(gbits) + nonzero(qbits) - 3) * MADD + AFF_ADD + LAST_ADD + CHECK


# safegcd inversion (safegcd.h): at most 25 batches of 30 divsteps, each applying
# its 2x2 matrix to (f, g) (36 signed 32x32 products) and (d, e) (54 incl. the
# n multiples), plus one Montgomery product by R^3.  The divsteps themselves are
# 32-bit shift/compare work, not MACs.
INV_N_MACS = 25 * (36 + 54) + 162


# the comb's table reads alone, in the comb's own pattern (key-ordered lanes,
# XCD-aware blocks, the 234 GB G29 + 100 x key21 footprint, one-deep LDS
# streaming), no arithmetic: 0.69 ms for 1M x 21 x 64 B (tools/gather_comb.hip,
# profiles/r03_gather_comb.txt).  The comb moves the same bytes in ~1.04 ms:
# it is NOT gather-bound (round 2's 1.2 TB/s figure came from uniform gathers
# over a 64 GiB table without key order and was withdrawn).
GATHER_ONLY_TBPS = 2.04


def table_points(gb: int, qb: int) -> int:
    """Table points per verify: windows of the G and the key geometry (one 64-B entry each)."""
    return len(window_widths(gb)) + len(window_widths(qb))


def macs_scalars(k: int) -> float:
    """k signatures per lane, 64 k per wave share one inversion (Montgomery's trick per
    lane and across the wave over PLAIN s values, p256_kernels.hip k_ecdsa_scalars /
    wave_batch_inv_n): per signature u1, u2 (2 products) + 3 (k - 1) / k for the
    lane's prefix, back-substitution and running inverse; per lane 15 for the wave
    scans and 2 (1 at k = 1) R-power fixes; 1/(64 k) of an inversion.  From k = 4
    one scan and inversion per 256-thread block (block_batch_inv_n)."""
    per_sig = 2 + 3 * (k - 1) / k
    if k >= 4:  # block_batch_inv_n: quad scans 4 + recovery 2 per lane, wave 0's 15 shared by 4 waves
        return per_sig * FN_MUL + (6 + 15 / 4 + 2) * FN_MUL / k + INV_N_MACS / (256 * k)
    per_lane = 15 + (2 if k > 1 else 1)
    return per_sig * FN_MUL + per_lane * FN_MUL / k + INV_N_MACS / (64 * k)
# v_mad_u64_u32 issue peak: 256 CU x 4 SIMD x 16 lanes/clk x 2.4 GHz (4-cycle wave64 issue);
# measured 30.9 T lane-ops/s in profiles/r01_valu_microbench.txt
MAD_PEAK = 256 * 4 * 16 * 2.4e9


def scalar_batch(n: int) -> int:
    """Mirror of pbftv::scalar_batch (p256_kernels.hip)."""
    e = os.environ.get("PBFTV_SCALAR_BATCH")
    if e in ("1", "2", "4", "8", "16"):
        return int(e)
    lanes, k = 65536, 1
    while k < 4 and n >= 2 * k * lanes:
        k *= 2
    return k


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, local


def register_with_phases(ver, pub):
    """pbftv_register_keys timed, with its per-phase wall times: the library's
    PBFTV_TRACE lines (pbftv_api.cpp trace(): quiesce, geometry, release old key
    tables, G table allocation / build, key table allocation / build, and inside
    each build its table scratch and table kernels) read from this process's
    stderr for the duration of the call.  PBFTV_TRACE is set by main() before
    the first registration (the library reads it once)."""
    import re
    import tempfile
    sys.stderr.flush()
    saved = os.dup(2)
    with tempfile.TemporaryFile() as f:
        os.dup2(f.fileno(), 2)
        try:
            t0 = time.perf_counter()
            valid = ver.register_keys(pub)
            wall = time.perf_counter() - t0
        finally:
            os.dup2(saved, 2)
            os.close(saved)
        f.seek(0)
        text = f.read().decode(errors="replace")
    phases = {}
    for line in text.splitlines():
        m = re.match(r"pbftv\[dev (\d+)\] (.+): ([0-9.]+) ms$", line)
        if m:
            phases[m.group(2)] = round(phases.get(m.group(2), 0.0) + float(m.group(3)), 1)
        elif line:
            sys.stderr.write(line + "\n")
    return valid, wall, phases


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv: list, data_dir: str | None) -> int:
    """`bench.py --gpus N` started as ONE process (the driver's plain form):
    start N rank processes of this script, one per GPU, exactly as
    torch.distributed.run would (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*),
    and exit with the first failing rank's code.  This process never touches
    a GPU (it only generated the batch, shared read-only via data_dir), so
    starting children from it is safe.  Rank 0's stdout is ours: the JSON line."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PBFTV_BENCH_SPAWNED="1")
        if data_dir:
            env["PBFTV_BENCH_DATA"] = data_dir
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else sys.stderr, start_new_session=True))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    sys.stderr.write(f"bench.py: rank {procs.index(p)} exited with {c}; stopping the others\n")
                    for q in live:
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()
    return rc


def save_batch(n_global: int, keys: int) -> str:
    """config 4 generated once by the launching process and shared with the
    ranks through read-only files (tmpfs when there is one): N ranks would
    otherwise each sign the same million messages on the same host cores."""
    import tempfile
    need = 2 * 110 * n_global + (1 << 20)  # ~101 B per signature (hash, r||s, key, ok) with room to spare
    base = None
    if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK):
        st = os.statvfs("/dev/shm")
        if st.f_bavail * st.f_frsize >= need:  # (a container's /dev/shm can be as small as 64 MB)
            base = "/dev/shm"
    dd = tempfile.mkdtemp(prefix="pbftv_bench_", dir=base)
    pub, H, S, K, ok = synth.config4(n_global, n_keys=keys, seed=0x50424654)
    for name, a in (("pub", pub), ("H", H), ("S", S), ("K", K), ("ok", ok)):
        np.save(os.path.join(dd, name + ".npy"), a)
    return dd


def load_batch(dd: str):
    return tuple(np.load(os.path.join(dd, name + ".npy"), mmap_mode="r") for name in ("pub", "H", "S", "K", "ok"))


def in_context_leg(ws: int, share: bool, pub, H, S, K, ok, steps: int, warmup_ms: float, reps: int = 5) -> dict:
    """The product's own multi-device path, in ONE process: one context over the
    N GPUs, what the Go drop-in gets from pbftv_open(&ctx, 0).
      host_path:     the global batch from host memory through
                     pbftv_ecdsa_p256_verify_batch, which splits it into
                     contiguous 512-aligned shards, one host thread + stream
                     per device, and concatenates the bitmaps (run_sharded,
                     pbftv_api.cpp plan_shards);
      device_resident: the same shards resident in each device's HBM, one
                     caller thread per device issuing pbftv_ecdsa_p256_verify_batch_dev
                     on two library streams (as the per-rank processes do).
    share: every logical device on GPU 0 (PBFTV_ALIAS_DEVICES; a flow rehearsal
    on a one-GPU box, not a scaling number)."""
    import threading
    from simple_pbft_amd.sharding import plan_shards
    saved = os.environ.get("PBFTV_ALIAS_DEVICES")
    if share:
        os.environ["PBFTV_ALIAS_DEVICES"] = str(ws)
    ver = Verifier(device_mask=1 if share else (1 << ws) - 1)
    out = {"what": "one process, one pbftv context over the N devices (pbftv_open device_mask = all)",
           "shared_device_rehearsal": share}
    bufs = []
    try:
        ndev = ver.device_count()
        if ndev != ws:
            raise RuntimeError(f"in_context: the context sees {ndev} devices, --gpus asked for {ws}")
        out["devices"] = [ver.device_id(i) for i in range(ndev)]
        H, S, K = (np.ascontiguousarray(a) for a in (H, S, K))
        ok = np.asarray(ok, bool)
        n = len(K)
        valid, out["registration_wall_s"], out["registration_phases_ms"] = register_with_phases(
            ver, np.ascontiguousarray(pub))
        assert valid.all()
        gb, qb, tb = ver.table_config()
        out["comb_window_bits"] = {"G": gb, "keys": qb}
        ver.verify_batch(H[:65536], S[:65536], K[:65536])  # first-touch of the host pipeline
        best, got = 1e9, None
        for _ in range(reps):
            t0 = time.perf_counter()
            got = ver.verify_batch(H, S, K)
            best = min(best, time.perf_counter() - t0)
        out["host_path"] = {"verifies_per_s": n / best, "ms": best * 1e3, "check": bool((got == ok).all()),
                            "reps": reps, "what": "pageable host buffers, the best of reps"}
        shards = plan_shards(n, ndev)
        per = []
        for dv, (lo, hi) in enumerate(shards):
            dh, ds, dk = (ver.to_device(dv, a[lo:hi]) for a in (H, S, K))
            sts = [ver.stream_create(dv) for _ in range(2)]
            dbs = [ver.alloc(dv, (hi - lo + 7) // 8 + 1) for _ in sts]
            bufs += [dh, ds, dk] + dbs
            per.append((dv, lo, hi, dh, ds, dk, sts, dbs))

        def run(item, k):
            dv, lo, hi, dh, ds, dk, sts, dbs = item
            for j in range(k):
                ver.verify_batch_dev(dv, dh.ptr, ds.ptr, dk.ptr, hi - lo, dbs[j & 1].ptr, stream=sts[j & 1])
            for st in sts:
                ver.stream_wait(dv, st)

        def all_devices(k):
            th = [threading.Thread(target=run, args=(it, k)) for it in per]
            for x in th:
                x.start()
            for x in th:
                x.join()

        t_w = time.perf_counter()
        while time.perf_counter() - t_w < warmup_ms * 1e-3:
            all_devices(8)
        t0 = time.perf_counter()
        all_devices(steps)
        el = time.perf_counter() - t0
        chk = True
        for dv, lo, hi, dh, ds, dk, sts, dbs in per:
            for db in dbs:
                chk &= bool((np.unpackbits(db.to_host(), bitorder="little")[:hi - lo].astype(bool) == ok[lo:hi]).all())
        out["device_resident"] = {"verifies_per_s": n * steps / el, "ms_per_step": el / steps * 1e3,
                                  "steps": steps, "check": chk, "shards": [[lo, hi] for _, lo, hi, *_ in per]}
    finally:
        for b in bufs:
            b.free()
        ver.close()
        if share:
            if saved is None:
                os.environ.pop("PBFTV_ALIAS_DEVICES", None)
            else:
                os.environ["PBFTV_ALIAS_DEVICES"] = saved
    return out


def in_context_result(ws: int, leg) -> tuple[dict, str | None]:
    """Run the in_context leg (leg() -> its dict) and judge it: an exception,
    a context that does not span --gpus devices, or a failed bitmap check is a
    failure of the product's own multi-device path, and bench.py then exits
    non-zero after printing its line (the driver's 8-GPU run
    must not report a green line over a broken run_sharded).  Returns
    (the leg's dict, the failure or None)."""
    try:
        res = leg()
    except Exception as e:  # noqa: BLE001 -- reported in the line AND in the exit status
        return {"error": repr(e)}, f"in_context raised {e!r}"
    if len(res.get("devices", [])) != ws:
        return res, f"in_context ran on {len(res.get('devices', []))} devices, --gpus {ws}"
    for part in ("host_path", "device_resident"):
        if not res.get(part, {}).get("check", False):
            return res, f"in_context {part} bitmap check failed"
    return res, None


class Dist:
    def __init__(self, ws):
        self.ws = ws
        self.dist = None
        if ws > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo's C++ connect log goes to stdout; keep stdout to the one JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo")
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


_QC_DRIVER = None


def qc_driver():
    """tools/qc_driver.c (built by __graft_entry__.build()): the per-certificate
    caller loop in C, calling pbftv_qc_verify through its function pointer."""
    global _QC_DRIVER
    if _QC_DRIVER is None:
        L = ctypes.CDLL(os.path.join(ROOT, "tools", "libqc_driver.so"))
        vp = ctypes.c_void_p
        L.qc_drive.restype = ctypes.c_int
        L.qc_drive.argtypes = [vp, vp, vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.c_double, vp, vp, vp]
        _QC_DRIVER = L
    return _QC_DRIVER


# the reference's own 99-byte request preimage (log/node1.log:3, tests/golden/digest_kats.json)
REQUEST_PREIMAGE = (b'{"timestamp":1668519246,"clientID":"client1","operation":"printf",'
                    b'"sequenceID":1668519247222762700}')


def single_calls(ver: Verifier, reps: int = 2000) -> dict:
    """The single-call drop-ins, each called from C (tools/qc_driver.c) as a
    cgo caller would, p50 / p99 over reps back-to-back calls (VERDICT r5 item
    7), beside the same single call on the CPU:
      hash_hex:    pbftv_hash_hex (utils.Hash, utils/utils.go:13-17) on the
                   99-byte request preimage -- the reference hashes once per
                   request at pbft_impl.go:73 (StartConsensus) and re-hashes
                   the request for every vote in verifyMsg (:190);
      verify_msg:  pbftv_verify_msg_batch at n = 1 (verifyMsg's compare, host code);
      verify_1sig: a 1-signature pbftv_qc_verify (the armed latency kernel);
    and OpenSSL's EVP_Digest + hex (oracle/openssl_standin.c), a 1-signature
    ECDSA_do_verify on one thread."""
    D = qc_driver()
    vp = ctypes.c_void_p
    D.hash_drive.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_char_p]
    D.vmsg_drive.argtypes = [vp, vp, ctypes.c_char_p, ctypes.c_uint32, vp]
    L = lib_handle(ver)
    msg = np.frombuffer(REQUEST_PREIMAGE, np.uint8)
    import hashlib
    want = hashlib.sha256(REQUEST_PREIMAGE).hexdigest()

    def pct(us):
        return {"p50": float(np.percentile(us, 50)), "p99": float(np.percentile(us, 99)), "min": float(us.min()),
                "calls": len(us)}
    out = {"message_bytes": len(REQUEST_PREIMAGE)}
    us = np.zeros(reps)
    hx = ctypes.create_string_buffer(65)
    D.hash_drive(ctypes.cast(L.pbftv_hash_hex, vp).value, ver.handle.value, msg.ctypes.data, len(msg), 50,
                 us.ctypes.data, hx)  # (warm)
    bad = D.hash_drive(ctypes.cast(L.pbftv_hash_hex, vp).value, ver.handle.value, msg.ctypes.data, len(msg), reps,
                       us.ctypes.data, hx)
    out["hash_hex"] = {**pct(us), "ok": bad == 0 and hx.value.decode() == want}
    dg = np.frombuffer(bytes.fromhex(want), np.uint8).copy()
    bad = D.vmsg_drive(ctypes.cast(L.pbftv_verify_msg_batch, vp).value, dg.ctypes.data, want.encode(), reps,
                       us.ctypes.data)
    out["verify_msg"] = {**pct(us), "ok": bad == 0}
    q1 = qc_latency(ver, 4, 1, reps, 17)
    out["verify_1sig"] = {k: q1[k] for k in ("p50", "p99", "min", "calls", "armed_frac")}
    so = os.path.join(ROOT, "oracle", "libopenssl_standin.so")
    if os.path.exists(so):
        S = ctypes.CDLL(so)
        S.standin_hash_hex_drive.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_char_p]
        S.standin_hash_hex_drive(msg.ctypes.data, len(msg), 50, us.ctypes.data, hx)
        bad = S.standin_hash_hex_drive(msg.ctypes.data, len(msg), reps, us.ctypes.data, hx)
        out["cpu_hash_hex"] = {**pct(us), "ok": bad == 0 and hx.value.decode() == want,
                               "kind": "openssl_standin EVP_Digest, caller's thread"}
        S.standin_qc_latency.restype = ctypes.c_int64
        S.standin_qc_latency.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_uint32,
                                         ctypes.c_int, ctypes.c_double, vp, vp]
        pub, H, S1, K = synth.certs(4, 1, 400, 18)
        us1 = np.zeros(400)
        bm = np.zeros(64, np.uint8)
        acc = S.standin_qc_latency(H.ctypes.data, S1.ctypes.data, K.ctypes.data, 400, 1, pub.ctypes.data, len(pub),
                                   1, 0.0, us1.ctypes.data, bm.ctypes.data)
        out["cpu_verify_1sig"] = {**pct(us1), "ok": acc == 400, "kind": "openssl_standin ECDSA_do_verify, 1 thread"}
    return out


def qc_latency(ver: Verifier, n_keys: int, sigs: int, iters: int, seed: int, gap_s: float = 0.0, warm: int = 20,
               register: bool = True, certs=None):
    """Latency of pbftv_qc_verify on one certificate from host buffers: every
    call verifies a DIFFERENT certificate (its table entries come cold from HBM,
    as for fresh votes), made from C (tools/qc_driver.c: nanosleep(gap) before
    each call, CLOCK_MONOTONIC around it) as a compiled cgo caller would make
    it.  gap_s = 1.0 is the reference's cadence: one flush per 1-s alarm
    (pbft/network/node.go:44, :513-518).  Returns p50 / p90 / p99 / min in us
    and the medians of the library's own diagnostics (pbftv_qc_stamps): host
    time inside the call, and for armed serves the GPU's serve time and clock."""
    if certs is None:
        pub, H, S, K = synth.certs(n_keys, sigs, iters + warm, seed)
        if register:
            ver.register_keys(pub)
    else:
        H, S, K = certs
    H, S, K = (np.ascontiguousarray(a) for a in (H, S, K))
    L = lib_handle(ver)
    fn = ctypes.cast(L.pbftv_qc_verify, ctypes.c_void_p).value
    st = ctypes.cast(L.pbftv_qc_stamps, ctypes.c_void_p).value
    D = qc_driver()

    def drive(lo, cnt, gap):
        us = np.zeros(cnt)
        acc = np.zeros(cnt, np.uint64)
        stamps = np.zeros((cnt, 8), np.uint64)
        bad = D.qc_drive(fn, st, ver.handle.value, H[lo * sigs:].ctypes.data, S[lo * sigs:].ctypes.data,
                         K[lo * sigs:].ctypes.data, cnt, sigs, sigs, gap * 1e6, us.ctypes.data, acc.ctypes.data,
                         stamps.ctypes.data)
        assert bad == 0 and (acc == sigs).all(), (bad, acc[acc != sigs][:4])
        return us, stamps
    drive(0, warm, 0.0)
    us, stamps = drive(warm, iters, gap_s)
    out = {"p50": float(np.percentile(us, 50)), "p90": float(np.percentile(us, 90)),
           "p99": float(np.percentile(us, 99)), "min": float(us.min()), "calls": iters, "gap_s": gap_s}
    out["in_library_us_p50"] = float(np.median(stamps[:, 1])) * 1e-3
    out["in_library_handover_us_p50"] = float(np.median(stamps[:, 0])) * 1e-3
    out["in_library_to_lock_us_p50"] = float(np.median(stamps[:, 2] >> np.uint64(32))) * 1e-3
    out["in_library_slots_in_us_p50"] = float(np.median((stamps[:, 2] >> np.uint64(1)) & np.uint64(0x7FFFFFFF))) * 1e-3
    armed = (stamps[:, 2] & np.uint64(1)) == 1
    out["armed_frac"] = float(armed.mean())
    armed &= stamps[:, 5] > stamps[:, 3]  # GPU stamps present (PBFTV_QC_STAMPS=1 when armed)
    if armed.any():
        a = stamps[armed].astype(np.float64)
        wall = (a[:, 5] - a[:, 3]) / (a[:, 7] * 1e3)
        out["gpu_serve_us_p50"] = float(np.median(wall)) * 1e6
        out["gpu_sclk_mhz_p50"] = float(np.median((a[:, 6] - a[:, 4]) / np.maximum(wall, 1e-9))) * 1e-6
    return out


def lib_handle(ver: Verifier):
    return ver._L


def qc_under_load(ver: Verifier, dh, ds, dk, n: int, ok, seed: int, calls3: int = 300, calls67: int = 100):
    """QC latency (2 ms between certificates) with the GPU idle and then with a
    stream of 1M-signature batches running on another library stream of the
    same context (a background thread enqueues two batches, waits, repeats):
    what a certificate costs while the node also drains a large pool snapshot.
    Certificates are signed by the registered config-4 committee (its keys:
    synth.certs with the same seed).  A node sees ONE certificate size (its
    committee's), so the sizes are measured one after the other, each in the
    state its own calls leave: 3 signatures (n = 4) idle then loaded -- the
    8-wave armed kernel, whole CUs -- then 67 (n = 100) idle then loaded -- the
    128-wave kernel.  The stream's rate alone (no certificate, nothing armed
    yet) is measured first, for the ratio."""
    import threading
    _, H3, S3, K3 = synth.certs(100, 3, 2 * calls3 + 80, seed)
    _, H67, S67, K67 = synth.certs(100, 67, 2 * calls67 + 20, seed)

    def part(H, S, K, sigs, lo, cnt):
        sl = slice(lo * sigs, (lo + cnt + 10) * sigs)
        return qc_latency(ver, 100, sigs, cnt, 0, gap_s=0.002, warm=10, certs=(H[sl], S[sl], K[sl]))
    st = ver.stream_create(0)
    db = ver.alloc(0, n // 8 + 1)

    def loaded(fn):
        """fn() while the stream runs; returns (fn's result, stream verifies/s meanwhile)"""
        stop = threading.Event()
        done = [0]

        def stream():
            while not stop.is_set():
                ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr, stream=st)
                ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr, stream=st)
                ver.stream_wait(0, st)
                done[0] += 2
        th = threading.Thread(target=stream)
        th.start()
        try:
            time.sleep(0.05)
            t0 = time.perf_counter()
            b0 = done[0]
            r = fn()
            rate = (done[0] - b0) * n / (time.perf_counter() - t0)
        finally:
            stop.set()
            th.join()
        return r, rate
    def forced(fn):
        """fn() with PBFTV_QC_YIELD=0: a server stays resident beside the batches"""
        saved = os.environ.get("PBFTV_QC_YIELD")
        os.environ["PBFTV_QC_YIELD"] = "0"
        try:
            return fn()
        finally:
            if saved is None:
                os.environ.pop("PBFTV_QC_YIELD", None)
            else:
                os.environ["PBFTV_QC_YIELD"] = saved

    out = {"yield_policy": os.environ.get("PBFTV_QC_YIELD", "adaptive (PBFTV_QC_YIELD unset: a batch halts the "
                                          "server when no certificate came for PBFTV_QC_YIELD_IDLE_MS = 50 ms)")}
    _, out["stream_verifies_per_s_alone"] = loaded(lambda: time.sleep(0.6))
    out["idle_3sigs"] = part(H3, S3, K3, 3, 0, calls3)
    out["loaded_3sigs"], r3 = loaded(lambda: part(H3, S3, K3, 3, calls3 + 20, calls3))
    # the stream right after those certificates, no call meanwhile: the default
    # policy (the first batch after 50 ms without a certificate halts the server) ...
    _, out["stream_verifies_per_s_after_3sigs_no_calls"] = loaded(lambda: time.sleep(0.6))
    # ... and with the narrow server held resident beside it (PBFTV_QC_YIELD=0)
    def narrow_resident():
        part(H3, S3, K3, 3, 2 * calls3 + 30, 2)
        return loaded(lambda: time.sleep(0.6))[1]
    out["stream_verifies_per_s_armed_narrow"] = forced(narrow_resident)
    # sparse certificates (one per 100 ms) while the stream runs: the default
    # policy serves each with a launch beside the batches (the server was halted)
    out["loaded_3sigs_every_100ms"], _ = loaded(lambda: qc_latency(
        ver, 100, 3, 20, 0, gap_s=0.1, warm=2,
        certs=(H3[3 * (calls3 + 2):], S3[3 * (calls3 + 2):], K3[3 * (calls3 + 2):])))
    out["idle_67sigs"] = part(H67, S67, K67, 67, 0, calls67)
    out["loaded_67sigs"], r67 = loaded(lambda: part(H67, S67, K67, 67, calls67 + 10, calls67))

    def wide_resident():
        part(H67, S67, K67, 67, 0, 2)
        return loaded(lambda: time.sleep(0.6))[1]
    out["stream_verifies_per_s_armed_wide"] = forced(wide_resident)
    out["stream_verifies_per_s_during"] = {"3sigs": r3, "67sigs": r67}
    alone = out["stream_verifies_per_s_alone"]
    out["stream_rate_ratio"] = {"3sigs": r3 / alone, "67sigs": r67 / alone,
                                "after_3sigs_no_calls": out["stream_verifies_per_s_after_3sigs_no_calls"] / alone,
                                "armed_narrow_no_calls": out["stream_verifies_per_s_armed_narrow"] / alone,
                                "armed_wide_no_calls": out["stream_verifies_per_s_armed_wide"] / alone}
    out["stream_check"] = bool((np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool) == ok).all())
    db.free()
    ver.stream_destroy(0, st)
    out["p50_ratio_3sigs"] = out["loaded_3sigs"]["p50"] / out["idle_3sigs"]["p50"]
    out["p50_ratio_67sigs"] = out["loaded_67sigs"]["p50"] / out["idle_67sigs"]["p50"]
    return out


def cpu_qc_latency(threads_allot: int, tick_calls: int = 15):
    """The CPU side of the QC-latency metric ("p50 QC verify
    latency ... single-threaded per QC"): the OpenSSL stand-in verifying ONE
    certificate at a time (oracle/openssl_standin.c standin_qc_latency: the
    caller's thread plus persistent spinning workers, keys parsed once, as a
    replica holds its peers' public keys), back to back and with the
    reference's 1-s gap before each certificate.  p50 in us."""
    so = os.path.join(ROOT, "oracle", "libopenssl_standin.so")
    if not os.path.exists(so):
        return None
    L = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    L.standin_qc_latency.restype = ctypes.c_int64
    L.standin_qc_latency.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_uint32, ctypes.c_int,
                                     ctypes.c_double, vp, vp]
    out = {"kind": "openssl_standin", "threads_allotment": threads_allot}
    for nk, sg, thr, cnt, gap in ((4, 3, 1, 400, 0.0), (4, 3, 3, 400, 0.0), (100, 67, threads_allot, 200, 0.0),
                                  (100, 67, 1, 30, 0.0), (4, 3, 1, tick_calls, 1.0), (4, 3, 3, tick_calls, 1.0)):
        pub, H, S, K = synth.certs(nk, sg, cnt, 21 + nk)
        us = np.zeros(cnt)
        bm = np.zeros((cnt * sg + 7) // 8, np.uint8)
        acc = L.standin_qc_latency(H.ctypes.data, S.ctypes.data, K.ctypes.data, cnt, sg, pub.ctypes.data, len(pub),
                                   thr, gap * 1e6, us.ctypes.data, bm.ctypes.data)
        assert acc == cnt * sg, (acc, cnt * sg)
        key = f"n{nk}_{sg}sigs_{thr}thr" + ("_tick" if gap else "")
        out[key] = {"p50": float(np.percentile(us, 50)), "p99": float(np.percentile(us, 99)), "calls": cnt}
    return out


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _read(path: str):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _cpulist(text: str) -> list:
    out = []
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out.extend(range(int(a), int(b or a) + 1))
    return out


def pin_to_gpu_node(dev: int):
    """Run this process on the CPUs of the NUMA node its GPU hangs off
    (sysfs numa_node of the GPU's PCI device, intersected with the allowed
    CPUs), as INTEGRATION.md §3 asks of a node's caller: on a two-socket host
    a 67-vote certificate from the other socket takes ~36 instead of ~31 us
    (profiles/r06_numa/summary.txt).  PBFTV_BENCH_PIN=0 leaves the affinity
    alone.  Returns what was done (for the JSON line)."""
    if os.environ.get("PBFTV_BENCH_PIN") == "0" or not hasattr(os, "sched_setaffinity"):
        return {"pinned": False, "why": "PBFTV_BENCH_PIN=0" if hasattr(os, "sched_setaffinity") else "no affinity API"}
    try:
        hip = ctypes.CDLL("libamdhip64.so.7")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, dev) != 0:
            return {"pinned": False, "why": "hipDeviceGetPCIBusId failed"}
        bus = buf.value.decode().lower()
        node = int(_read(f"/sys/bus/pci/devices/{bus}/numa_node") or -1)
        if node < 0:
            return {"pinned": False, "why": f"no NUMA node for {bus}"}
        cpus = sorted(set(_cpulist(_read(f"/sys/devices/system/node/node{node}/cpulist") or "")) &
                      os.sched_getaffinity(0))
        if not cpus:
            return {"pinned": False, "why": f"no allowed CPU on node {node}"}
        os.sched_setaffinity(0, cpus)
        return {"pinned": True, "numa_node": node, "cpus": len(cpus), "gpu_bus": bus}
    except (OSError, ValueError) as e:
        return {"pinned": False, "why": repr(e)}


def cpu_allotment() -> dict:
    """The host CPUs this process may actually use, with the evidence: the
    scheduler affinity mask (os.sched_getaffinity), the cgroup-v2 CPU quota
    (/sys/fs/cgroup/cpu.max, "max" = none; cgroup v1 cfs_quota/period as a
    fallback), and the physical cores / SMT threads behind the allowed CPUs
    (/sys/devices/system/cpu/cpuN/topology).  `threads` = min(affinity,
    floor(quota)) is what the CPU baselines run on."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    quota = None
    cm = _read("/sys/fs/cgroup/cpu.max")
    src = "/sys/fs/cgroup/cpu.max"
    if cm:
        q, _, per = cm.partition(" ")
        if q != "max" and per:
            quota = int(q) / int(per)
    else:
        q, per = _read("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), _read("/sys/fs/cgroup/cpu/cpu.cfs_period_us")
        src = "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"
        if q and per and int(q) > 0:
            quota = int(q) / int(per)
    cores = set()
    for c in aff:
        pkg = _read(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id")
        core = _read(f"/sys/devices/system/cpu/cpu{c}/topology/core_id")
        if core is not None:
            cores.add((pkg, core))
    threads = len(aff)
    if quota is not None:
        threads = max(1, min(threads, int(quota)))
    return {"threads": threads, "affinity_cpus": len(aff), "cgroup_quota_cpus": quota,
            "cgroup_cpu_max": cm, "cgroup_source": src if cm is not None or quota is not None else None,
            "physical_cores_in_affinity": len(cores) or None,
            "smt_threads_per_core": (len(aff) / len(cores)) if cores else None,
            "smt_active": _read("/sys/devices/system/cpu/smt/active"), "nproc": os.cpu_count(),
            "cpu_model": cpu_model()}


def _cpu_verify(so_name, fn_name, pub, H, S, K, sample: int, threads: int):
    so = os.path.join(ROOT, "oracle", so_name)
    if not os.path.exists(so):
        return None
    L = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    fn = getattr(L, fn_name)
    fn.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint32, vp, ctypes.c_int]
    h, s, k = (np.ascontiguousarray(a[:sample]) for a in (H, S, K))
    bm = np.zeros((sample + 7) // 8, np.uint8)
    t0 = time.perf_counter()
    fn(h.ctypes.data, s.ctypes.data, k.ctypes.data, sample, pub.ctypes.data, len(pub), bm.ctypes.data, threads)
    dt = time.perf_counter() - t0
    return {"value": sample / dt, "unit": "verifies/s", "cores": threads, "nproc": os.cpu_count(),
            "cpu_model": cpu_model(), "seconds": dt, "_bitmap": bm}


def openssl_standin(pub, H, S, K, sample: int, threads: int):
    """cpu_baseline: OpenSSL 3 libcrypto ECDSA_do_verify on host threads
    (oracle/openssl_standin.c).  Go 1.19's amd64 P-256
    (crypto/elliptic p256_asm) is a port of OpenSSL's nistz256 assembly, so this
    is the faithful stand-in for the reference's CPU verify path, which cannot
    run here (no Go toolchain)."""
    r = _cpu_verify("libopenssl_standin.so", "standin_ecdsa_p256_verify_batch", pub, H, S, K, sample, threads)
    if r is not None:
        r["kind"] = "openssl_standin"
        r["sample"] = (f"first {sample} signatures of the config-4 batch (oracle/openssl_standin.c, {r['cores']} "
                       "pthreads, OpenSSL 3 nistz256)")
    return r


def cpu_standin_sample(threads: int, n: int) -> int:
    """A bounded sample: ~0.5 s of wall time at ~27k verifies/s per thread,
    at least 262,144 signatures (~10 thread-seconds), at most the batch, in
    whole 512-signature groups."""
    want = max(262144, threads * 27_000 // 2)
    return n if want >= n else want // 512 * 512


def cpu_oracle_port(pub, H, S, K, sample: int, threads: int):
    """The oracle port (oracle/p256_ref.c: 4x64-bit CIOS, bit-serial Shamir --
    deliberately simple, for parity) on host threads; reported beside the
    stand-in, not as the baseline."""
    r = _cpu_verify("liboracle.so", "oracle_ecdsa_p256_verify_batch", pub, H, S, K, sample, threads)
    if r is not None:
        r["kind"] = "port"
        r["sample"] = f"first {sample} signatures of the config-4 batch (oracle/p256_ref.c, {r['cores']} pthreads)"
    return r


def host_path(ver, H, S, K, ok, reps=5):
    """pbftv_ecdsa_p256_verify_batch on the full batch from host memory: the
    drop-in path a pool flush would call (PCIe in, bitmap out), pipelined in
    chunks (pbftv_api.cpp verify_host_pipelined).  Pageable numpy inputs (staged
    through pinned memory by parallel memcpy) and pinned inputs (pbftv_host_alloc:
    DMA straight from the caller's buffers).  Best-of wall time."""
    n = len(K)
    res = {}
    for label, arrays in (("pageable", (H, S, K)), ("pinned", None)):
        pins = None
        if arrays is None:
            pins = [ver.pinned(a) for a in (H, S, K)]
            arrays = tuple(p.a for p in pins)
        got = ver.verify_batch(*arrays)
        good = bool((got == ok).all())
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            ver.verify_batch(*arrays)
            ts.append(time.perf_counter() - t0)
        res[label] = {"verifies_per_s": n / min(ts), "ms": min(ts) * 1e3, "check": good}
        if pins:
            for p in pins:
                p.free()
    return res


# ---------------------------------------------------------------- other BASELINE configs
def _timed(ver, fn, reps):
    """Best-of wall time of fn() (each call synchronises the device)."""
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ver.sync(0)
        ts.append(time.perf_counter() - t0)
    return min(ts), float(np.median(ts))


def run_config1(ver, n_req=1000, outputs=None):
    """configs[0]: the reference 4-node pattern for 1k requests with every
    message signed, end to end from host buffers, one device
    round trip per message kind (Go-JSON preimage + SHA-256 + checks + ECDSA on
    the device):
      requests     pbftv_flush_requests: client signature over the request as
                   sent, plus the StartConsensus digest with the assigned
                   sequence ID (pbft_impl.go:57-73)
      pre-prepares pbftv_flush_preprepares: primary's signature + verifyMsg
                   against each receiving replica's State, 3 receipts/request
      votes        pbftv_flush_votes: 9 prepare + 12 commit receipts/request,
                   verifyMsg against the request's State + signature
      replies      pbftv_flush_replies: 4 per request, the client checks them
    2 % of each message kind is corrupted (synth.config1_cluster: bad
    signatures; validly signed pre-prepares/votes with a wrong digest, wrong
    view or stale sequence ID), and every bit of every flush is compared with
    the construction (check_config1).  The messages are laid out column-wise
    before timing, as a cgo shim would hand over a pool snapshot.  `outputs`
    (a dict) receives the inputs and the last flush results (for the GPU test's
    oracle comparison)."""
    from simple_pbft_amd.pbftv import PrePrepareColumns, ReplyColumns, RequestColumns, VoteColumns
    c = synth.config1_cluster(n_req)
    ver.register_keys(c["pub"])
    node_of = {nid: j for j, nid in enumerate(synth.NODES)}
    checks = c["checks"]

    def idx(kind):
        return np.array([x[1] for x in checks if x[0] == kind], np.int64)
    qi, pi, vi, ri = idx("request"), idx("preprepare"), idx("vote"), idx("reply")
    votes, replies, pps = c["votes"], c["replies"], c["preprepares"]
    req_cols = RequestColumns([c["requests"][j] for j in qi])
    qS, qK = np.ascontiguousarray(c["request_sigs"][qi]), np.full(len(qi), synth.CLIENT_KEY, np.uint32)
    aseq = np.ascontiguousarray(c["assigned_seqs"][qi])
    pp_cols = PrePrepareColumns([pps[j] for j in pi])          # one entry per replica receipt
    pS, pK = np.ascontiguousarray(c["preprepare_sigs"][pi]), np.zeros(len(pi), np.uint32)
    p_state = np.ascontiguousarray(c["preprepare_state"][pi])
    vote_cols = VoteColumns([votes[j] for j in vi])            # one entry per received vote
    vS = np.ascontiguousarray(c["vote_sigs"][vi])
    vK = np.array([node_of[votes[j][3]] for j in vi], np.uint32)
    v_state = np.ascontiguousarray(c["vote_state"][vi])
    s_view, s_last = c["state_view"], c["state_last"]
    rep_cols = ReplyColumns([replies[j] for j in ri])
    rS = np.ascontiguousarray(c["reply_sigs"][ri])
    rK = np.array([node_of[replies[j][3]] for j in ri], np.uint32)
    expect = {"request_sig": c["request_sig_ok"][qi], "preprepare_sig": c["preprepare_sig_ok"][pi],
              "preprepare_msg": c["preprepare_msg_ok"][pi], "vote_sig": c["vote_sig_ok"][vi],
              "vote_msg": c["vote_msg_ok"][vi], "reply_sig": c["reply_sig_ok"][ri]}
    state = {}

    def flow():
        _, q_ok, req_d = ver.flush_requests(req_cols, qS, qK, aseq, digests=False)
        _, _, p_ok, pm_ok = ver.flush_preprepares(pp_cols, pS, pK, (s_view, s_last), p_state, digests=False)
        _, v_ok, vm_ok = ver.flush_votes(vote_cols, vS, vK, (s_view, s_last, req_d), v_state, digests=False)
        _, r_ok = ver.flush_replies(rep_cols, rS, rK, digests=False)
        state["got"] = {"request_sig": q_ok, "preprepare_sig": p_ok, "preprepare_msg": pm_ok, "vote_sig": v_ok,
                        "vote_msg": vm_ok, "reply_sig": r_ok, "request_digests": req_d}

    best, med = _timed(ver, flow, 5)
    n_sig = len(qi) + len(pi) + len(vi) + len(ri)
    n_dig = 2 * len(qi) + 2 * len(pi) + len(vi) + len(ri)
    ok, rejected = check_config1(state["got"], expect)
    if outputs is not None:
        outputs.update(cluster=c, got=state["got"], expect=expect, index={"request": qi, "preprepare": pi,
                                                                          "vote": vi, "reply": ri})
    return {"workload": f"config1: 4-node pattern, {n_req} requests, every message signed: {n_sig} signature "
                        f"checks ({len(qi)} requests, {len(pi)} pre-prepares, {len(vi)} votes, {len(ri)} replies), "
                        f"{n_dig} Go-JSON digests built on the device, {len(pi) + len(vi)} verifyMsg, "
                        "4 flush calls end-to-end from host buffers; 2% of each message kind corrupted",
            "verifies_per_s": n_sig / best, "ms": best * 1e3, "ms_median": med * 1e3, "rejected": rejected,
            "check": ok}


def check_config1(got: dict, expect: dict):
    """Every bit of every config-1 flush equals the construction, and each flush
    rejects >= 1 % of its receipts, some for a bad signature (so an all-accept
    verifier fails).  Returns
    (ok, rejected receipts per output)."""
    ok = True
    rejected = {}
    for k, want in expect.items():
        g = np.asarray(got[k], bool)
        ok = ok and g.shape == want.shape and bool((g == want).all())
        rejected[k] = int((~want).sum())
    for kind in ("request", "preprepare", "vote", "reply"):
        bad = ~expect[kind + "_sig"]
        if kind + "_msg" in expect:
            bad = bad | ~expect[kind + "_msg"]
        ok = ok and bad.sum() >= 0.01 * len(bad) and (kind + "_sig") in rejected and rejected[kind + "_sig"] > 0
    return bool(ok), rejected


def run_certs(ver, n_keys, per_cert, n_certs, label, outputs=None):
    """Configs 2 and 3: n_certs quorum certificates of per_cert distinct votes in
    ONE device-resident launch; 1 % of the certificates carry one bad vote and
    0.5 % two (synth.corrupt_certs, the 8 corruption classes in turn).  The
    check: every bit equals the construction, the 2f+1 QC fails exactly at the
    certificates with a bad vote, and the reference's 2f count
    (pbft_impl.go:212,227) exactly at those with two."""
    pub, H, S, K = synth.certs(n_keys, per_cert, n_certs, seed=per_cert * 7 + n_keys)  # every signature distinct
    want, bad_any, bad_two = synth.corrupt_certs(H, S, K, per_cert, n_keys)
    ver.register_keys(pub)
    n = len(K)
    dh, ds, dk = ver.to_device(0, H), ver.to_device(0, S), ver.to_device(0, K)
    db = ver.alloc(0, (n + 7) // 8)
    best, med = _timed(ver, lambda: ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, db.ptr), 10)
    bits = np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool)
    for b in (dh, ds, dk, db):
        b.free()
    f = (per_cert - 1) // 2
    ok = check_certs(bits, want, per_cert, bad_any, bad_two, quorum_ref=2 * f)
    if outputs is not None:
        outputs.update(pub=pub, H=H, S=S, K=K, bits=bits, want=want, bad_any=bad_any, bad_two=bad_two)
    return {"workload": label + "; 1% of certificates with one bad vote, 0.5% with two", "verifies_per_s": n / best,
            "ms": best * 1e3, "ms_median": med * 1e3, "certs": n_certs, "rejected": int((~want).sum()), "check": ok}


def check_certs(bits, want, per_cert, bad_any, bad_two, quorum_ref):
    """Bits equal the construction; QC (all per_cert votes, 2f+1 of n = 3f+1)
    fails exactly at bad_any; the reference's >= 2f count exactly at bad_two."""
    bits = np.asarray(bits, bool)
    n_certs = len(bits) // per_cert
    acc = bits.reshape(n_certs, per_cert).sum(1)
    qc_fail = np.nonzero(acc < per_cert)[0]
    ref_fail = np.nonzero(acc < quorum_ref)[0]
    return bool(len(bad_any) > 0 and (bits == want).all() and np.array_equal(qc_fail, np.sort(bad_any))
                and np.array_equal(ref_fail, np.sort(bad_two)))


def run_config5(ver, n=1_000_000, steps=5):
    """configs[4]: SHA-256 over 1M messages of 256 B..4 KiB (digest kernel alone)."""
    data, off, ln = synth.sha_config5(n)
    return _sha_run(ver, data, off, ln, steps, "config5: SHA-256 of {n} messages, {lens} B, {gb:.2f} GB, {blocks} blocks")


def run_sha_pbft(ver, n=1_000_000, steps=5):
    """The digests utils.Hash actually computes (utils/utils.go:13-17 via
    digest(), pbft_impl.go:235-243): Go-JSON preimages of 99-244 B -- RequestMsg
    99 B (2 blocks), ReplyMsg 110 B (2), VoteMsg 167 B (3), PrePrepareMsg 244 B
    (4) -- in the reference's per-request mix (1 request : 3
    pre-prepares : 21 votes : 4 replies)."""
    rng = np.random.default_rng(0x50424655)
    kinds = np.array([99, 244, 167, 110])
    ln = kinds[rng.choice(4, size=n, p=np.array([1, 3, 21, 4]) / 29.0)].astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    data = rng.integers(32, 127, int(ln.sum()), dtype=np.uint8)
    return _sha_run(ver, data, off, ln, steps,
                    "PBFT digests: SHA-256 of {n} Go-JSON-sized messages, {lens} B (request/pre-prepare/vote/reply "
                    "mix), {gb:.2f} GB, {blocks} blocks")


def _sha_run(ver, data, off, ln, steps, label):
    import hashlib
    n = len(ln)
    dd = ver.to_device(0, data, pad=64)
    do, dl = ver.to_device(0, off), ver.to_device(0, ln)
    dord, dg = ver.alloc(0, 4 * n), ver.alloc(0, 32 * n)
    ver.sha256_order_dev(0, dl.ptr, n, dord.ptr)
    ver.sync(0)
    # wall clock and kernel time over exactly the same calls: one untimed
    # warm-up call, then per rep the HIP-event kernel time (library events on
    # the launch stream) and the wall time around the same synchronised call;
    # the kernel runs inside its wall window, so kernel_ms <= ms rep by rep
    ver.sha256_batch_dev(0, dd.ptr, do.ptr, dl.ptr, dord.ptr, n, dg.ptr)
    ver.sync(0)
    ver.set_kernel_timing(True)
    walls, kerns = [], []
    for _ in range(steps):
        ver.reset_kernel_times()
        t0 = time.perf_counter()
        ver.sha256_batch_dev(0, dd.ptr, do.ptr, dl.ptr, dord.ptr, n, dg.ptr)
        ver.sync(0)
        walls.append(time.perf_counter() - t0)
        k_ms, k_cnt = ver.kernel_time_ms(0, 2)
        assert k_cnt == 1
        kerns.append(k_ms * 1e-3)
    ver.set_kernel_timing(False)
    wall, kavg = float(np.mean(walls)), float(np.mean(kerns))
    best = wall
    dig = dg.to_host().reshape(n, 32)
    rng = np.random.default_rng(1)
    ok = all(dig[i].tobytes() == hashlib.sha256(data[off[i]:off[i] + ln[i]].tobytes()).digest()
             for i in rng.integers(0, n, 2000))
    total = int(ln.sum())
    blocks = int(((ln.astype(np.int64) + 8) // 64 + 1).sum())
    for b in (dd, do, dl, dord, dg):
        b.free()
    ops = blocks * SHA_OPS_PER_BLOCK
    cpu = openssl_sha256(data, off, ln, dig)
    return {"workload": label.format(n=n, lens=lo_hi(ln), gb=total / 1e9, blocks=blocks), "cpu_baseline": cpu,
            "digests_per_s": n / best, "GB_per_s": total / best / 1e9, "ms": best * 1e3, "kernel_ms": kavg * 1e3,
            "ms_min": min(walls) * 1e3, "kernel_ms_per_rep": [k * 1e3 for k in kerns], "reps": steps,
            "timing": "ms = mean wall time of `reps` synchronised calls; kernel_ms = mean HIP-event time of k_sha256 "
                      "in the same calls (frac from kernel_ms)",
            "roofline": {"bound": "valu", "achieved": ops / kavg / 1e12, "peak": VALU_PEAK / 1e12,
                         "unit": "T VALU ops/s (1528 per 64-B block, SURVEY §8(d))",
                         "frac": ops / kavg / VALU_PEAK, "hbm_GB_per_s": (total + 32 * n) / kavg / 1e9,
                         "hbm_frac": (total + 32 * n) / kavg / 8e12},
            "check": ok}


def openssl_sha256(data, off, ln, gpu_digests):
    """The same messages through OpenSSL 3 EVP_Digest SHA-256 (SHA-NI, like Go's
    crypto/sha256 assembly) on 16 host threads (oracle/openssl_standin.c,
    SURVEY.md §8(d)(ii)); best of 3, digests compared with the GPU's."""
    so = os.path.join(ROOT, "oracle", "libopenssl_standin.so")
    if not os.path.exists(so):
        return None
    L = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    L.standin_sha256_batch.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_int]
    n = len(ln)
    off64, ln32 = np.ascontiguousarray(off, np.uint64), np.ascontiguousarray(ln, np.uint32)
    out = np.zeros((n, 32), np.uint8)
    threads = cpu_allotment()["threads"]
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        L.standin_sha256_batch(data.ctypes.data, off64.ctypes.data, ln32.ctypes.data, n, out.ctypes.data, threads)
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    return {"value": n / t, "unit": "digests/s", "GB_per_s": float(ln32.sum()) / t / 1e9, "cores": threads,
            "nproc": os.cpu_count(), "cpu_model": cpu_model(), "kind": "openssl_standin",
            "sample": f"all {n} messages (oracle/openssl_standin.c EVP_Digest, {threads} pthreads = the process's "
                      "CPU allotment)",
            "agrees_with_gpu": bool((out == gpu_digests).all())}


def lo_hi(ln):
    return f"{int(ln.min())}-{int(ln.max())}"


SHA_OPS_PER_BLOCK = 1528
VALU_PEAK = 256 * 4 * 32 * 2.4e9   # full-rate 32-bit VALU: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz


PMC_JSON = os.path.join(ROOT, "profiles", "r06_final_pmc.json")


def pmc_figures(kernel: str, geometry):
    """Counter-derived figures of one kernel from the committed PMC summary
    (tools/pmc_passes.sh + tools/pmc_summary.py); the comb's only when the
    summary was measured at the same table geometry."""
    if not os.path.exists(PMC_JSON):
        return {}
    with open(PMC_JSON) as f:
        pm = json.load(f).get("kernels", {})
    e = pm.get(kernel, {})
    if kernel == "ecdsa_comb" and e.get("geometry") != list(geometry):
        return {}
    keep = ("valu_issue_frac", "valu_busy_frac", "valu_insts_per_wave", "hbm_bytes_per_launch", "clock_ghz",
            "kernel_ms")
    return {k: e[k] for k in keep if k in e}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--warmup-ms", type=float, default=100.0,
                    help="keep warming up until this much wall time has passed (the comb's ~40 ms ramp after idle)")
    ap.add_argument("--n", type=int, default=1 << 20,
                    help="global batch (strong scaling, the default: BASELINE configs[3] shards N/k over k GPUs); "
                         "with --weak: signatures per rank")
    ap.add_argument("--weak", action="store_true", help="weak scaling: every rank verifies its own --n batch")
    ap.add_argument("--keys", type=int, default=100)
    ap.add_argument("--streams", type=int, default=2,
                    help="consecutive batches alternate over this many library streams (pbftv_stream_create: each "
                         "owns its verify scratch), so batch j+1's scalar stage overlaps batch j's comb; 0 = the "
                         "context's own stream")
    ap.add_argument("--no-extras", action="store_true", help="skip QC latency, host path, CPU baselines, other configs")
    ap.add_argument("--no-in-context", action="store_true",
                    help="N > 1: skip the one-process leg over one N-device context (in_context)")
    ap.add_argument("--sha-only", action="store_true", help="only configs[4] (SHA-256 digest kernel), one JSON line")
    args = ap.parse_args()
    if args.sha_only:
        ver = Verifier(device_mask=1)
        print(json.dumps({"config5": run_config5(ver), "pbft_digests": run_sha_pbft(ver)}), flush=True)
        ver.close()
        return

    ws, rank, local = dist_env()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the plain `python bench.py --gpus N`: one rank process per GPU, started here
        dd = None if args.weak else save_batch(args.n, args.keys)
        try:
            rc = spawn_ranks(args.gpus, sys.argv[1:], dd)
        finally:
            if dd:
                import shutil
                shutil.rmtree(dd, ignore_errors=True)
        sys.exit(rc)
    os.environ.setdefault("PBFTV_TRACE", "1")  # registration phases (register_with_phases)
    if args.gpus != ws:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws} rank processes: launch with "
                         f"--nproc-per-node {args.gpus}, or without torch.distributed.run")
    d = Dist(ws)
    probe = os.environ.get("PBFTV_BENCH_PROBE")
    if probe:
        # launcher check without a GPU (tests/test_dist.py): the ranks that came
        # up; "in_context:<stub>" also runs rank 0's in_context judgement on a
        # stub leg ("raise", "devices": one device short, "check": a failed
        # bitmap, "ok") -- the exit status the driver would see
        seen = d.sum(1.0)
        failure = None
        line = {"probe": True, "world_size": ws, "ranks_seen": seen, "gpus": args.gpus,
                "spawned": os.environ.get("PBFTV_BENCH_SPAWNED") == "1",
                "shared_data": os.environ.get("PBFTV_BENCH_DATA") is not None}
        if rank == 0 and probe.startswith("in_context:"):
            stub = probe.split(":", 1)[1]

            def leg():
                if stub == "raise":
                    raise RuntimeError("stub in_context leg failed")
                devs = list(range(ws - 1 if stub == "devices" else ws))
                return {"devices": devs, "host_path": {"check": True}, "device_resident": {"check": stub != "check"}}
            line["in_context"], failure = in_context_result(ws, leg)
        if rank == 0:
            print(json.dumps(line), flush=True)
        d.barrier()
        d.close()
        if failure:
            raise SystemExit(f"bench.py: {failure}")
        return
    # one GPU per rank; PBFTV_BENCH_SHARE_DEVICE=1 puts every rank on device 0
    # (only to rehearse the N > 1 flow on a 1-GPU box -- not a scaling number)
    share = os.environ.get("PBFTV_BENCH_SHARE_DEVICE") == "1"
    affinity = pin_to_gpu_node(0 if share else local)
    ver = Verifier(device_mask=1 if share else 1 << local)
    if ver.device_count() != 1 or (not share and ver.device_id(0) != local):
        raise SystemExit(f"bench.py rank {rank}: expected GPU {local}, the context has "
                         f"{[ver.device_id(i) for i in range(ver.device_count())]}")
    glob = None
    if args.weak:
        n_global, lo = args.n * ws, 0
        n = args.n
        pub, H, S, K, ok = synth.config4(n, n_keys=args.keys, seed=0x50424654 + rank)
    else:
        # strong scaling: the one global batch, contiguous shards of whole 512-signature groups
        n_global = args.n
        per = -(-n_global // ws)
        per = -(-per // 512) * 512
        lo, hi = min(n_global, rank * per), min(n_global, (rank + 1) * per)
        n = hi - lo
        if os.environ.get("PBFTV_BENCH_DATA"):
            pub, H, S, K, ok = load_batch(os.environ["PBFTV_BENCH_DATA"])
        else:
            pub, H, S, K, ok = synth.config4(n_global, n_keys=args.keys, seed=0x50424654)
        glob = (pub, H, S, K, ok)
        H, S, K, ok = (np.ascontiguousarray(a[lo:hi]) for a in (H, S, K, ok))
        pub = np.ascontiguousarray(pub)
    if share:  # ranks sharing one GPU register one after the other: each sizes its tables from what is free
        for r in range(ws):
            if r == rank:
                valid, t_reg, reg_phases = register_with_phases(ver, pub)
            d.barrier()
    else:
        valid, t_reg, reg_phases = register_with_phases(ver, pub)  # G table + one table per key, built on the device
    assert valid.all()
    dh, ds, dk = ver.to_device(0, H), ver.to_device(0, S), ver.to_device(0, K)
    ver.reserve(n)
    # one bitmap per stream; batches alternate over the streams (each stream's
    # verifies are ordered, the streams overlap)
    streams = [ver.stream_create(0) for _ in range(args.streams)] or [None]
    dbs = [ver.alloc(0, (n + 7) // 8 + 1) for _ in streams]
    db = dbs[0]
    turn = [0]

    def step():
        if n:
            j = turn[0] % len(streams)
            ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, dbs[j].ptr, stream=streams[j])
            turn[0] += 1

    def sync_all():
        ver.sync(0)
        for st in streams:
            if st is not None:
                ver.stream_wait(0, st)

    for _ in streams:
        step()
    sync_all()
    got = np.unpackbits(db.to_host(), bitorder="little")[:n].astype(bool)
    check = all(bool((np.unpackbits(b.to_host(), bitorder="little")[:n].astype(bool) == ok).all()) for b in dbs)
    # Warm-up right before the timed steps, with no idle gap in between: after
    # the GPU idles a few ms the comb needs ~40 ms of load to get back to its
    # steady speed (first step after an 8 ms pause 1.37 ms, then 1.14, 1.24 ...
    # 0.96 ms after 30 steps; rocprof trace profiles/r02_warm_ramp.txt).
    t_w = time.perf_counter()
    w = 0
    while w < args.warmup or time.perf_counter() - t_w < args.warmup_ms * 1e-3:
        step()
        w += 1
        if w % 8 == 0:
            sync_all()  # (the host clock follows the GPU)

    # wall clock over K steps, uninstrumented: a timing event between two
    # kernels costs the GPU a ~6 us gap (rocprof timeline, tools/rocpd_timeline.py)
    d.barrier()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync_all()
    d.barrier()
    elapsed = time.perf_counter() - t0
    # the same K steps queued on the context stream only (no overlap between
    # consecutive batches), reported beside the headline
    one_stream_ms = None
    if args.streams and not args.no_extras:
        d.barrier()
        sync_all()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            if n:
                ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, dbs[0].ptr)
        sync_all()
        d.barrier()
        one_stream_ms = d.max(time.perf_counter() - t1) / args.steps * 1e3
    # kernel durations for the roofline: the same K steps again, with HIP events
    # recorded by the library around each scalar / comb launch on its stream
    # (on ONE stream, so no kernel's event window includes another batch's
    # overlapping work: these are the kernels' own durations)
    ver.set_kernel_timing(True)
    ver.reset_kernel_times()
    for _ in range(args.steps):
        if n:
            ver.verify_batch_dev(0, dh.ptr, ds.ptr, dk.ptr, n, dbs[0].ptr, stream=streams[0])
    sync_all()
    comb_ms, comb_cnt = ver.kernel_time_ms(0, K_ECDSA_COMB)
    scal_ms, scal_cnt = ver.kernel_time_ms(0, K_ECDSA_SCALARS)
    ver.set_kernel_timing(False)
    check = check and all(bool((np.unpackbits(b.to_host(), bitorder="little")[:n].astype(bool) == ok).all())
                          for b in dbs)
    t_max = d.max(elapsed)
    all_ok = d.sum(0.0 if check else 1.0) == 0.0
    total = n_global * args.steps
    value = total / t_max

    mode = "weak" if args.weak else "strong"
    out = {
        "metric": METRIC, "value": value, "unit": "verifies/s", "n_gpus": ws, "steps": args.steps,
        "warmup": args.warmup, "warmup_steps_run": w, "ms_per_step": t_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": mode, "vs_baseline": None, "dtype": "u32",
        "data": "synthetic: distinct OpenSSL-signed P-256 votes, 1% corrupted (tools/synth.py)",
        "config": {"workload": (f"config4: {n_global} ECDSA-P256 sigs" +
                                (f" ({args.n} per rank)" if args.weak else f" sharded N/{ws}") +
                                f", {args.keys}-key table, 1% corrupted (8 classes)"),
                   "global_batch": n_global, "keys": args.keys,
                   "parallelism": f"shard{ws} ({mode} scaling: independent per-GPU shards, no collective)",
                   "streams": args.streams},
        "check": "pass" if all_ok else "FAIL",
    }
    if one_stream_ms is not None:
        out["ms_per_step_one_stream"] = one_stream_ms
    out["affinity"] = affinity
    if rank == 0:
        comb_avg = comb_ms / max(comb_cnt, 1) * 1e-3
        scal_avg = scal_ms / max(scal_cnt, 1) * 1e-3
        kb = scalar_batch(n)
        ms = macs_scalars(kb)
        gb, qb, tb = ver.table_config()
        mc = macs_comb(gb, qb)
        kern = {
            "ecdsa_comb": {"avg_ms": comb_avg * 1e3, "macs_per_verify": mc, "window_bits": [gb, qb],
                           "achieved_tmacs": n * mc / max(comb_avg, 1e-12) / 1e12},
            "ecdsa_scalars": {"avg_ms": scal_avg * 1e3, "macs_per_verify": ms, "sigs_per_lane": kb,
                              "achieved_tmacs": n * ms / max(scal_avg, 1e-12) / 1e12},
        }
        dom = "ecdsa_comb" if comb_avg >= scal_avg else "ecdsa_scalars"
        ach = kern[dom]["achieved_tmacs"]
        pmc = pmc_figures(dom, (gb, qb))
        out["roofline"] = {"bound": "valu", "kernel": dom, "achieved": ach, "peak": MAD_PEAK / 1e12,
                           "unit": "TMAC/s (v_mad limb MACs)", "frac": ach * 1e12 / MAD_PEAK,
                           "traffic": pmc.get("hbm_bytes_per_launch"),
                           "valu_issue_frac": pmc.get("valu_issue_frac"),
                           "valu_busy_frac": pmc.get("valu_busy_frac"),
                           "valu_insts_per_wave": pmc.get("valu_insts_per_wave"),
                           "pmc_source": os.path.relpath(PMC_JSON, ROOT) if pmc else None}
        if dom == "ecdsa_comb":
            # the comb's table reads (one 64-B entry per table point, ~21 per verify) against
            # the same reads alone in the comb's pattern (tools/gather_comb.hip: 2.04 TB/s,
            # profiles/r03_gather_comb.txt): the comb is not gather-bound
            pts = table_points(gb, qb)
            gbytes = n * pts * 64
            out["roofline"]["table_gathers"] = {"bytes_per_launch": gbytes, "points_per_verify": pts,
                                                "TBps": gbytes / max(comb_avg, 1e-12) / 1e12,
                                                "gather_only_TBps": GATHER_ONLY_TBPS,
                                                "frac_of_gather_only": gbytes / max(comb_avg, 1e-12) / 1e12 /
                                                GATHER_ONLY_TBPS,
                                                "source": "tools/gather_comb.hip, profiles/r03_gather_comb.txt"}
        out["kernels"] = kern
        out["config"]["comb_window_bits"] = {"G": gb, "keys": qb, "table_bytes_per_gpu": tb}
        out["registration_s"] = {"keys": args.keys, "wall_s": t_reg, "phases_ms": reg_phases,
                                 "what": "pbftv_register_keys: G table + the key tables built on the device (incl. "
                                         "allocation); phases_ms from the library's PBFTV_TRACE (the table scratch / "
                                         "table kernels lines are the parts of each build)"}
        if not args.no_extras and ws == 1:
            # host-buffer path with no armed latency kernel on the GPU (none armed yet)
            out["host_path"] = host_path(ver, H, S, K, ok)
            out["host_path_verifies_per_s"] = out["host_path"]["pageable"]["verifies_per_s"]
            # certificates while a 1M stream runs on another stream of this context
            load = qc_under_load(ver, dh, ds, dk, n, ok, seed=0x50424654)
            # ... and the host path again with the armed kernel kept waiting
            # (the keeper holds one for PBFTV_QC_KEEP_MS after the last call)
            hp_armed = host_path(ver, H, S, K, ok)
            out["host_path_with_armed_kernel"] = {
                **hp_armed, "ratio_pageable": hp_armed["pageable"]["verifies_per_s"] /
                out["host_path"]["pageable"]["verifies_per_s"],
                "ratio_pinned": hp_armed["pinned"]["verifies_per_s"] / out["host_path"]["pinned"]["verifies_per_s"]}
            q4 = qc_latency(ver, 4, 3, 10000, 11)
            q4_tick = qc_latency(ver, 4, 3, 30, 13, gap_s=1.0, warm=3)
            q4_100 = qc_latency(ver, 4, 3, 30, 14, gap_s=0.1, warm=3)
            q100 = qc_latency(ver, 100, 67, 2000, 12)
            q100_tick = qc_latency(ver, 100, 67, 20, 15, gap_s=1.0, warm=3)
            out["qc_latency_us"] = {
                "p50_n4_3sigs": q4["p50"], "p99_n4_3sigs": q4["p99"],
                "p50_n100_67sigs": q100["p50"], "p99_n100_67sigs": q100["p99"],
                "p50_n4_3sigs_tick": q4_tick["p50"], "p50_n4_3sigs_gap100ms": q4_100["p50"],
                "p50_n100_67sigs_tick": q100_tick["p50"],
                "tick_over_back_to_back_n4": q4_tick["p50"] / q4["p50"],
                "tick_over_back_to_back_n100": q100_tick["p50"] / q100["p50"],
                "p50_n4_3sigs_under_1M_stream": load["loaded_3sigs"]["p50"],
                "p50_n100_67sigs_under_1M_stream": load["loaded_67sigs"]["p50"],
                "calls": {"n4": q4["calls"], "n100": q100["calls"], "n4_tick": q4_tick["calls"],
                          "n4_gap100ms": q4_100["calls"], "n100_tick": q100_tick["calls"]},
                "definition": "host submit -> accept bitmap + quorum on host, pbftv_qc_verify, one FRESH "
                              "certificate per call (SURVEY.md §8(d)), called from C (tools/qc_driver.c) as a cgo "
                              "caller would; _tick = a 1-s idle gap before every call (the reference's alarm, "
                              "pbft/network/node.go:44)",
                "detail": {"n4": q4, "n4_tick": q4_tick, "n4_gap100ms": q4_100, "n100": q100, "n100_tick": q100_tick},
                "under_load": load}
            # the single-call drop-ins beside their CPU counterparts
            out["single_calls_us"] = single_calls(ver)
            # the CPU baseline on every host CPU this process may use (affinity
            # mask capped by the cgroup quota, with the evidence), plus the
            # 16-thread figure of the box's nominal per-GPU share as a labelled extra
            allot = cpu_allotment()
            thr = allot["threads"]
            out["cpu_qc_latency_us"] = cpu_qc_latency(thr)
            sample = cpu_standin_sample(thr, n)
            cb = openssl_standin(pub, H, S, K, sample=sample, threads=thr)
            if cb is not None:
                bm = cb.pop("_bitmap")
                cb["agrees_with_gpu"] = bool((np.unpackbits(bm, bitorder="little")[:sample].astype(bool) ==
                                              got[:sample]).all())
                cb["allotment"] = allot
                out["cpu_baseline"] = cb
                out["gpu_vs_cpu"] = value / cb["value"]
                if thr != 16:
                    s16 = cpu_standin_sample(16, n)
                    c16 = openssl_standin(pub, H, S, K, sample=s16, threads=min(16, thr))
                    if c16 is not None:
                        c16.pop("_bitmap")
                        out["cpu_baseline_16_threads"] = c16
            port = cpu_oracle_port(pub, H, S, K, sample=32768, threads=min(thr, 64))
            if port is not None:
                bm = port.pop("_bitmap")
                port["agrees_with_gpu"] = bool((np.unpackbits(bm, bitorder="little")[:32768].astype(bool) ==
                                                got[:32768]).all())
                out["cpu_oracle_port"] = port
            out["other_configs"] = {
                "config1": run_config1(ver),
                "config2": run_certs(ver, 4, 3, 20000,
                                     "config2: n=4, 10k requests x (prepare QC + commit QC) x 3 sigs = 60k in one launch"),
                "config3": run_certs(ver, 100, 67, 10000,
                                     "config3: n=100 committee, 10k certificates x 67 sigs = 670k on one GPU"),
                "config5": run_config5(ver),
                "pbft_digests": run_sha_pbft(ver),
            }
            # the same certificates inside large batches: device time per certificate
            oc = out["other_configs"]
            out["qc_latency_us"]["in_batch_us_per_cert"] = {
                "n4_3sigs": oc["config2"]["ms"] * 1e3 / oc["config2"]["certs"],
                "n100_67sigs": oc["config3"]["ms"] * 1e3 / oc["config3"]["certs"]}
    for b in [dh, ds, dk] + dbs:
        b.free()
    for st in streams:
        if st is not None:
            ver.stream_destroy(0, st)
    ver.close()  # every rank's tables leave HBM before the one-context leg builds its own
    d.barrier()
    failure = None
    if rank == 0 and ws > 1 and glob is not None and not args.no_in_context:
        out["in_context"], failure = in_context_result(
            ws, lambda: in_context_leg(ws, share, *glob, steps=args.steps, warmup_ms=args.warmup_ms))
        if failure:
            out["in_context_check"] = "FAIL"
    if rank == 0:
        print(json.dumps(out), flush=True)
    d.barrier()
    d.close()
    if failure:
        raise SystemExit(f"bench.py: {failure}")


if __name__ == "__main__":
    main()
