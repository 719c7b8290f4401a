#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 --kernel-trace database: the
dispatches of the last few steps in start order, with each kernel's duration
and the idle gap before it (microseconds).

    python tools/rocpd_timeline.py gpurun_out/prof/run_results.db [--last 12] [--skip 0]"""
import argparse
import re
import sqlite3


def short(name):
    m = re.search(r"(k_\w+|__amd_rocclr_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=12)
    ap.add_argument("--skip", type=int, default=0, help="drop this many of the newest dispatches first")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, vgpr_count, accum_vgpr_count, sgpr_count, lds_size "
                          "from kernels order by start"))
    rows = rows[:len(rows) - a.skip][-a.last:]
    prev = None
    for name, s, e, v, av, sg, lds in rows:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{short(name):40s} dur {(e - s) / 1e3:9.2f} us  gap {gap:7.2f} us  vgpr {v} agpr {av} sgpr {sg} lds {lds}")
        prev = e


if __name__ == "__main__":
    main()
