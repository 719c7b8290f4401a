"""Summarise tools/ab.sh output: one line per (workload, variant), medians over
the rounds.   python tools/ab_summary.py OUT"""
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def last_json(path):
    lines = [l for l in open(path).read().strip().splitlines() if l.startswith("{")]
    return [json.loads(l) for l in lines]


def med(xs):
    xs = [x for x in xs if x is not None]
    return statistics.median(xs) if xs else float("nan")


def summarise(w, runs):
    """runs: list of lists of JSON objects (one list per round) -> text"""
    kind = w.split("-")[0]
    if kind in ("bench", "streams"):
        js = [r[-1] for r in runs]
        ks = {k: med([j["kernels"][k]["avg_ms"] for j in js]) for k in js[0]["kernels"]}
        return (f"Mverif/s {med([j['value'] / 1e6 for j in js]):7.1f}  step {med([j['ms_per_step'] for j in js]):.4f} ms  " +
                "  ".join(f"{k} {t:.4f} ms" for k, t in ks.items()) + f"  checks {[j['check'] for j in js]}")
    if kind == "sha":
        js = [r[-1] for r in runs]
        return (f"config5 kernel {med([j['config5']['kernel_ms'] for j in js]):.4f} ms frac "
                f"{med([j['config5']['roofline']['frac'] for j in js]):.4f}  pbft kernel "
                f"{med([j['pbft_digests']['kernel_ms'] for j in js]):.4f} ms  checks "
                f"{[(j['config5']['check'], j['pbft_digests']['check']) for j in js]}")
    if kind == "qc":
        js = [r[-1] for r in runs]
        return "  ".join(f"{k} p50 {med([j[k]['p50_us'] for j in js]):.2f} us" for k in js[0]
                         if isinstance(js[0][k], dict) and "p50_us" in js[0][k])
    if kind == "tick":
        js = [r[-1] for r in runs]
        keys = [k for k in js[0] if isinstance(js[0][k], dict) and "p50" in js[0][k]]
        return "  ".join(f"{k} {med([j[k]['p50'] for j in js]):.1f}" for k in keys)
    if kind == "load":
        js = [r[-1] for r in runs]
        p = "  ".join(f"{k} {med([j[k]['p50'] for j in js]):.1f}" for k in
                      ("idle_3sigs", "loaded_3sigs", "loaded_3sigs_every_100ms", "idle_67sigs", "loaded_67sigs")
                      if k in js[0])
        rr = {k: round(med([j["stream_rate_ratio"][k] for j in js]), 3) for k in js[0]["stream_rate_ratio"]}
        return f"p50 us: {p}  stream ratio {rr}"
    if kind == "idle":
        js = [r[-1] for r in runs]
        return f"stream rate armed / alone {med([j['ratio'] for j in js]):.4f}  per round {[round(j['ratio'], 4) for j in js]}"
    if kind == "reg":
        js = [r[-1] for r in runs]
        return "  ".join(f"{k} {med([j[k]['wall_s'] for j in js]):.3f} s" for k in ("first", "again", "reopened") if k in js[0])
    return json.dumps(runs[-1][-1])[:300]


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
    res = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "*__*__*.json"))):
        w, v, _ = os.path.basename(f)[:-5].split("__")
        try:
            res[(w, v)].append(last_json(f))
        except Exception:  # noqa: BLE001
            print(f"{w:18s} {v:28s} FAILED", open(f).read()[-300:])
    for (w, v), runs in res.items():
        try:
            print(f"{w:18s} {v:28s} {summarise(w, runs)}")
        except Exception as e:  # noqa: BLE001
            print(f"{w:18s} {v:28s} unreadable ({e!r})")


if __name__ == "__main__":
    main()
